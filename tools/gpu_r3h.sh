#!/bin/bash
# Same-box A/B of the in-tree library against abbase/libfpnmt_base.so
# (swapped in place, restored), C2 step + the dominant-conv probe, then the
# split-step GPU tests (the G1 / G2 split).
set -u
D=gpurun_out/r3h
mkdir -p $D
L=fpn-mt-image-captioning_amd/fpnmt/libfpnmt.so
cp $L /tmp/new.so
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then cp abbase/libfpnmt_base.so $L; else cp /tmp/new.so $L; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $D/ab.json 2>$D/ab.err || { cp /tmp/new.so $L; tail -5 $D/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$D/ab.json'));print('[$lib]', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
cp /tmp/new.so $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_checkpoint.py -m gpu -x -q --timeout 500 --timeout-method thread \
  -k "fused_optimizer_prep or checkpoint or bitwise or identity_residual" > $D/tests.txt 2>&1; rc=$?
echo "== split tests rc=$rc"; tail -3 $D/tests.txt
exit $rc
