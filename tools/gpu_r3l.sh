#!/bin/bash
# Same-box A/B of the in-tree library against abbase/libfpnmt_base.so (C2
# step, swapped in place, restored), the transformer / decode GPU tests, and
# the C5 decode probe on both.
set -u
D=gpurun_out/r3l
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
for lib in base new; do
  if [ $lib = base ]; then cp abbase/libfpnmt_base.so $L; else cp /tmp/new.so $L; fi
  timeout -k 10 200 python bench.py --c5-only > $D/c5.json 2>$D/c5.err || { cp /tmp/new.so $L; tail -5 $D/c5.err; exit 1; }
  python -c "import json;d=json.load(open('$D/c5.json'));print('[$lib] c5', d['c5_decode']['ms'])"
done
cp /tmp/new.so $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_decode.py tests/test_gpu_configs.py -m gpu -x -q --timeout 500 --timeout-method thread \
  --deselect tests/test_gpu_model.py::test_train_step_parity_c2_model_fp32 > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt
exit $rc
