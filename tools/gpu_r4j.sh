#!/bin/bash
# Round-4 session J: int32 step targets, P7 in the heads stage:
# (grouped view attention / view LayerNorms, embedding dropout, step
# targets kernel), then a C2 step bench and one profiled step.
set -u
D=gpurun_out/r4j
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -15; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
echo "== bench rc=$rc"; cut -c1-400 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -5 $D/step_breakdown.txt
python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -40 $D/step_counts.txt
