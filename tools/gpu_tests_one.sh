#!/bin/bash
# Runs the given GPU test files in ONE pytest process (-x, per-test timeout).
mkdir -p gpurun_out
name=${LOGNAME_TAG:-gputests}
timeout -k 10 1000 python -u -m pytest "$@" -x -v -m gpu -s --timeout 300 --timeout-method thread > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" "gpurun_out/$name.log" | tail -40
exit $rc
