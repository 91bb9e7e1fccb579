#!/bin/bash
# C2 step: bench line (no CPU baseline / probes) + rocprofv3 kernel stats of the step.
set -u
R=${ROUND:-r02}
mkdir -p gpurun_out/$R
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/$R/bench_step.json 2> gpurun_out/$R/bench_step.err; rc=$?
echo "== bench rc=$rc"; cat gpurun_out/$R/bench_step.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$R/bench_step.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/$R/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; exit $rc
