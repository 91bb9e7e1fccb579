#!/bin/bash
# Round-4 session C: the C2-model gradient parity at the 1e-5 bulk floor
# (medians over three inputs), the peaked co-attention backward test, the
# trained-model C5 decode parity. Stops at the first abnormal exit.
set -u
D=gpurun_out/r4c
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v --timeout 1000 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_spatial_softmax_peaked_bwd_vs_fp64" \
  "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
  "tests/test_gpu_model.py::test_train_step_parity_c2_model_fp32" -s > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "^image|passed|failed|Error|peaked|grad p90|grad max" $D/tests.txt | head -40; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
exit $rc
