#!/bin/bash
# Round-4 session P: the FFN-fusion test (norm-wise FE bar), then a same-box
# A/B of the spread-DMA pipe kernel in the dispatch: base (cfg 3 = 128x256
# 2-stage), c3 (cfg 3 = 3-stage, DMA spread between k-steps, MFMA priority),
# c34 (also cfg 4 = 64x64 4-stage spread).
set -u
D=gpurun_out/r4p
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_model.py::test_ffn_act_fused_matches" "tests/test_gpu_kernels.py" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_libs.sh 2 base c3 c34; rc=$?
echo "== ab rc=$rc"; exit $rc
