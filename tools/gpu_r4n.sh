#!/bin/bash
# Round-4 session N: ffn1's LeakyReLU backward in ffn2's bwd-data epilogue
# (fpnmt_gemm_act_in): the model tests, the C2 bench, one profiled step.
set -u
D=gpurun_out/r4n
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 600 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_dp_step.py "tests/test_gpu_configs.py::test_c2_logits_and_loss_parity_fp32" "tests/test_gpu_configs.py::test_c2_train_step_fp32_then_bf16" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 30 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
echo "== bench rc=$rc"; cut -c1-300 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -12 $D/step_counts.txt
