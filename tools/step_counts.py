"""Launch count and time per kernel name of one replayed step (the launches
between the last two AMSGrad kernels) of a rocprofv3 kernel trace:
python tools/step_counts.py <run_kernel_trace.csv> [substring ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "amsgrad_kernel" in r["Kernel_Name"]]
step = rows[idx[-2] + 1:idx[-1] + 1]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    k = r["Kernel_Name"].split("(")[0][:90]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
keys = sys.argv[2:]
print(f"{len(step)} kernels in the step")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    if not keys or any(s in k for s in keys):
        print(f"{c:4d} {t:9.1f} us  {k}")
