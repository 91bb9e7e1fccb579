#!/bin/bash
# Round-3 session I: GPU tests of the fused paths, an A/B of the identity-
# bottleneck gradient fusion (same library, config flag), the AMSGrad kernel
# time under rocprofv3.
set -u
D=gpurun_out/r3i
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_checkpoint.py -m gpu -x -q --timeout 500 --timeout-method thread \
  -k "fused_optimizer_prep or checkpoint or bitwise or identity_residual or split" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -le 1 ] || exit $rc
for f in "--fuse-identity off" "--fuse-identity on" "--fuse-identity off" "--fuse-identity on"; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra $f > $D/ab.json 2>$D/ab.err || { tail -5 $D/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$D/ab.json'));print('[$f]', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof rc=$rc"; grep -E "amsgrad|vectorized_elementwise" $D/step/step_kernel_stats.csv | cut -c1-160
exit $rc
