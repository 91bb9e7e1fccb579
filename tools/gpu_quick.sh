#!/bin/bash
# Quick GPU check after a kernel change: the kernel parity tests, then the
# bench line (N=1). Each step under its own time limit; stops at the first
# abnormal exit.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parts.py -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/quick_bench.log | cut -c1-200
exit $rc
