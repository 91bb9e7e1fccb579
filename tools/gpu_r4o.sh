#!/bin/bash
# Round-4 session O: the FFN-fusion test's bf16 bar (norm-wise over the
# feature extractor), and the pipe kernel's spread-DMA variants
# (tools/fwd_bench.hip -DFB_SPREAD, built beforehand into tools/bin).
set -u
D=gpurun_out/r4o
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_model.py::test_ffn_act_fused_matches" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
FB_FILTER=b32 timeout -k 10 300 tools/bin/fwd_bench_spread > $D/spread_b32.txt 2>&1; rc=$?
echo "== spread b32 rc=$rc"; cat $D/spread_b32.txt; [ $rc -eq 0 ] || exit $rc
FB_FILTER="P3 3x3" FB_WARM=1 timeout -k 10 300 tools/bin/fwd_bench_spread > $D/spread_p3_warm.txt 2>&1; rc=$?
echo "== spread P3 warm rc=$rc"; cat $D/spread_p3_warm.txt; [ $rc -eq 0 ] || exit $rc
