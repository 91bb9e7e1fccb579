#!/bin/bash
# Round-4 session S: the EPI-0 pipe kernel's residual / act-mask rows
# prefetched before its K loop: kernel + fused-epilogue model tests, then a
# same-box A/B against the previous build (slab8).
set -u
D=gpurun_out/r4s
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_model.py -k "not c2_model and not parity_c2" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_libs.sh 2 slab8 rpre; rc=$?
echo "== ab rc=$rc"; exit $rc
