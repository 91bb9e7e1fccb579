"""Per-step kernel time breakdown from a rocprofv3 kernel trace (CSV):
python tools/step_breakdown.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "amsgrad_kernel" in r["Kernel_Name"]]
s, e = idx[-2] + 1, idx[-1] + 1
step = rows[s:e + 1]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"one replayed step: {len(step)} kernels, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    n = r["Kernel_Name"]
    key = n.replace("_ZN5fpnmt11gemm_kernelIDF16bLi", "gemm<").split("EEEvNS_")[0][:60]
    if "gemm" in key:
        key += " grid=%s/%s" % (r["Grid_Size_X"], r["Workgroup_Size_X"])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
cat = collections.defaultdict(float)
for k, (c, t) in agg.items():
    kk = "gemm" if "gemm" in k else k.split("(")[0].split("<")[0][-40:]
    cat[kk] += t
print("by family:")
for k, t in sorted(cat.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {t:9.1f} us  {100 * t / (busy / 1e3):5.1f}%  {k}")
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
print("top entries:")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"  {t:8.1f} us {c:4d}x avg {t / c:7.1f}  {k}")
