#!/bin/bash
# Full GPU test suite (one pytest process, per-test time limits), then the
# bench line. Stops at the first abnormal exit.
mkdir -p gpurun_out
timeout -k 10 2400 python -u -m pytest tests -m gpu -x -q -s --timeout 1200 --timeout-method thread > gpurun_out/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/full_tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/full_bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -1 gpurun_out/full_bench.log | cut -c1-200
exit $rc
