#!/bin/bash
# 16-B M2 loads in the staged row epilogue: model / kernel GPU tests, then a
# same-box A/B of the in-tree library against abbase/libfpnmt_base.so.
set -u
D=gpurun_out/r3r
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $D/tests.txt | head -20; exit $rc; }
L=fpn-mt-image-captioning_amd/fpnmt/libfpnmt.so
cp $L /tmp/new.so
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then cp abbase/libfpnmt_base.so $L; else cp /tmp/new.so $L; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $D/ab.json 2>$D/ab.err || { cp /tmp/new.so $L; tail -5 $D/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$D/ab.json'));print('[$lib]', d['ms_per_step'], repr(d['loss']))"
  done
done
cp /tmp/new.so $L
