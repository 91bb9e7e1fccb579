#!/bin/bash
# Round-3 final: the whole -m gpu suite, smoke(), then the round's evidence
# (tools/gpu_profile_round.sh -> gpurun_out/r03f). Stops at the first failure.
set -u
D=gpurun_out/r3m
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1; rc=$?
echo "== smoke rc=$rc"; tail -2 $D/smoke.txt; [ $rc -eq 0 ] || exit $rc
ROUND=r03 bash tools/gpu_profile_round.sh
