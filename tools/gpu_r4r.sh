#!/bin/bash
# Round-4 session R: the ordered slab sum with its last round's loads in
# flight together (predicated adds): the determinism / deferred-reduction
# tests, then a same-box A/B against the previous build (c34).
set -u
D=gpurun_out/r4r
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread \
  tests/test_gpu_model.py -k "determin or deferred or graph" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_libs.sh 2 c34 slab8; rc=$?
echo "== ab rc=$rc"; exit $rc
