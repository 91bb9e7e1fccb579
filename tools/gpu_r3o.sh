#!/bin/bash
# Block-output ReLU' fused into the identity block's bwd-data epilogue: the
# model / kernel GPU tests, then a same-box flag A/B (two rounds).
set -u
D=gpurun_out/r3o
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $D/tests.txt | head -20; exit $rc; }
for r in 1 2; do
  for f in off on; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --fuse-block-act $f > $D/ab_$f.json 2>$D/ab_$f.err || { tail -5 $D/ab_$f.err; exit 1; }
    python -c "import json;d=json.load(open('$D/ab_$f.json'));print('[$f]', d['ms_per_step'], d['loss'])"
  done
done
