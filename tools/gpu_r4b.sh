#!/bin/bash
# Round-4 session B: the P4-path probe with perturbed inputs (lr 0), the
# trained-model decode parity tests. Stops at the first abnormal exit.
set -u
D=gpurun_out/r4b
mkdir -p $D
export TMPDIR=/tmp
P4_PERTURB=4 timeout -k 10 900 python -u tools/probes/p4_chain.py 6 10000 > $D/p4_chain.txt 2>&1; rc=$?
echo "== p4_chain rc=$rc"; grep -A8 "perturbed inputs" $D/p4_chain.txt; [ $rc -eq 0 ] || { tail -5 $D/p4_chain.txt; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread \
  "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32" \
  "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
  "tests/test_gpu_configs.py::test_c5_beam8_decode_matches_oracle_fp32" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "^image|passed|failed|Error" $D/tests.txt | head -30; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
exit $rc
