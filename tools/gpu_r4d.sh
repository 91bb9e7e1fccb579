#!/bin/bash
# Round-4 session D: the whole -m gpu suite (fused encoder view projection,
# DP / SyncBN / trained-decode / C2-parity tests), smoke(), a C2 step bench
# and one profiled step (kernel count, breakdown). Stops at the first
# abnormal exit.
set -u
D=gpurun_out/r4d
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 1000 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed" $D/tests.txt | tail -12; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
# 0 = green, 1 = assertion failures (read them afterwards); anything else
# (a crash, a fault, a time limit) ends the session here
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1; rc=$?
echo "== smoke rc=$rc"; tail -2 $D/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
echo "== bench rc=$rc"; cat $D/bench_step.json | cut -c1-600; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(ls $D/step/*/step_kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -22 $D/step_breakdown.txt
timeout -k 10 200 python tools/probes/headline_blas.py > $D/headline_blas.txt 2>&1; rc=$?
echo "== headline blas rc=$rc"; cat $D/headline_blas.txt
