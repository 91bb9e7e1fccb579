#!/bin/bash
# Round-4 session H: grouped view attention / view LayerNorms, C5 warm-up schedule:
set -u
D=gpurun_out/r4h
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -m gpu -q --timeout 900 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_dp_step.py tests/test_gpu_kernels.py \
  "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
  "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -15; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
echo "== bench rc=$rc"; cut -c1-500 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -22 $D/step_breakdown.txt
