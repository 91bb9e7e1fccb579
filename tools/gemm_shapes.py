"""Join FPNMT_GEMM_LOG lines with a rocprofv3 kernel trace of the same process
(GEMM launches in issue order) and report per-shape time and TFLOP/s.

  export FPNMT_GEMM_LOG=gpurun_out/gemm.log
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gs -o gs -- \
      python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-extra
  python tools/gemm_shapes.py gpurun_out/gemm.log gpurun_out/gs/gs_kernel_trace.csv [last_n_steps]

Only the last eager step is reported (the GEMMs after the second-to-last
amsgrad kernel)."""
import collections
import csv
import re
import sys

AMODE = {0: "ROW", 1: "COL", 2: "IM2COL", 3: "IM2COL_T"}
BMODE = {0: "NK", 1: "KN"}
CFG = {0: "128x128x64", 1: "64x64x32", 2: "64x64x64", 3: "128x128x32", 4: "32x32x32", 5: "small",
       110: "pipeWG128", 130: "pipe128x64e0", 131: "pipe64x64", 132: "pipe64x64s2", 133: "pipe128x256s2",
       134: "pipe64x64s4", 150: "wgjobs"}

log = [dict(kv.split("=") for kv in ln.split()[1:]) for ln in open(sys.argv[1]) if ln.strip()]
# deferred weight-gradient GEMMs (cfg 150) are queued, not launched: they run
# at the flush as grouped gemm_wg_jobs_kernel launches, reported separately
jobs_log = [g for g in log if g["cfg"] == "150"]
log = [g for g in log if g["cfg"] != "150"]
rows = list(csv.DictReader(open(sys.argv[2])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
jobs_k = [r for r in rows if "gemm_wg_jobs_kernel" in r["Kernel_Name"]]
rows_nojobs = [r for r in rows if "gemm_wg_jobs_kernel" not in r["Kernel_Name"]]
# a split small GEMM is two launches (partials + reduce): the reduce's time is
# charged to the GEMM launch before it
gemm = []
for r in rows_nojobs:
    n = r["Kernel_Name"]
    if "gemm" not in n or "fpnmt" not in n:
        continue
    if "reduce" in n and gemm:
        gemm[-1] = dict(gemm[-1], End_Timestamp=r["End_Timestamp"])
        continue
    gemm.append(r)
assert len(gemm) == len(log), (len(gemm), len(log))
ams = [i for i, r in enumerate(rows) if "amsgrad_kernel" in r["Kernel_Name"]]
if "--last-half" in sys.argv:  # forward-only probes: the second of two identical passes
    sys.argv.remove("--last-half")
    t_lo = int(gemm[len(gemm) // 2]["Start_Timestamp"]) - 1
    t_hi = int(gemm[-1]["Start_Timestamp"]) + 1
else:
    t_lo = int(rows[ams[-2]]["Start_Timestamp"]) if len(ams) >= 2 else 0
    t_hi = int(rows[ams[-1]]["Start_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
tot_t = tot_f = 0.0
for g, r in zip(log, gemm):
    t0 = int(r["Start_Timestamp"])
    if not (t_lo < t0 < t_hi):
        continue
    dt = (int(r["End_Timestamp"]) - t0) / 1e3
    M, N, K, B = (int(g[k]) for k in ("M", "N", "K", "batch"))
    flop = 2.0 * M * N * K * B
    key = "%-8s %-5s %-3s acc=%s %-10s M=%-7d N=%-6d K=%-6d b=%-3d split=%s" % (
        AMODE[int(g["a"])], BMODE[int(g["b"])], "SC" if g["c"] == "1" else "", g["acc"], CFG[int(g["cfg"])],
        M, N, K, B, g["split"])
    a = agg[key]
    a[0] += 1
    a[1] += dt
    a[2] += flop
    tot_t += dt
    tot_f += flop
jt = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in jobs_k
      if t_lo < int(r["Start_Timestamp"]) < t_hi]
if jt:
    print(f"deferred weight-gradient GEMM jobs: {len(jt)} grouped launches, {sum(jt):.1f} us "
          f"(queued jobs in the log: {len(jobs_log)})")
    tot_t += sum(jt)
print(f"GEMM time in step: {tot_t:.1f} us, {tot_f / 1e9:.1f} GFLOP (excluding the grouped jobs), "
      f"{tot_f / max(tot_t, 1e-9) / 1e6:.1f} TFLOP/s")
for k, (c, t, f) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[3]) if len(sys.argv) > 3 else 60]:
    print(f"{t:8.1f} us {c:3d}x avg {t / c:7.1f} {f / t / 1e6:7.1f} TF  {k}")
