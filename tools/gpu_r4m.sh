#!/bin/bash
# Round-4 session M: the transformer's Dense weight gradients deferred and
# run as grouped whole-K tile launches at the backward's flush
# (gemm_wg_jobs_kernel): targeted GPU tests, a C2 step bench, one profiled
# step and the per-shape GEMM table of an eager step.
set -u
D=gpurun_out/r4m
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 600 --timeout-method thread \
  "tests/test_gpu_model.py::test_deferred_dense_wgrads_match_immediate" tests/test_gpu_model.py \
  tests/test_gpu_dp_step.py > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error|largest" $D/tests.txt | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
echo "== bench rc=$rc"; cut -c1-300 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -25 $D/step_counts.txt
rm -f gpurun_out/gemm.log
FPNMT_GEMM_LOG=$D/gemm.log timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/gs -o gs -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-extra > $D/gs.log 2>&1; rc=$?
echo "== gemm shapes rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/gemm_shapes.py $D/gemm.log $(find $D/gs -name "*kernel_trace.csv" | head -1) > $D/gemm_shapes.txt 2>&1; head -30 $D/gemm_shapes.txt
