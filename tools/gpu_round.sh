#!/bin/bash
# One GPU session: tests, smoke, bench (+CPU baseline), rocprof kernel stats of
# the bench and of the roofline probe, PMC traffic of the roofline probe.
# Stops at the first abnormal exit (fault / timeout). Outputs in gpurun_out/.
set -u
mkdir -p gpurun_out
R=${ROUND:-r01b}
./tools/gpu_tests.sh tests/test_gpu_kernels.py tests/test_gpu_parts.py tests/test_gpu_model.py tests/test_gpu_decode.py || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "== smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err; rc=$?
echo "== bench rc=$rc"; cat gpurun_out/bench_$R.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$R.err; exit $rc; }
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R/roof -o roof -- python3 bench.py --roofline-only > gpurun_out/prof_roof.log 2>&1; rc=$?
echo "== prof roof rc=$rc"; tail -1 gpurun_out/prof_roof.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R/head -o head -- python3 bench.py --headline-only > gpurun_out/prof_head.log 2>&1; rc=$?
echo "== prof headline rc=$rc"; tail -1 gpurun_out/prof_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$R/pmc_fetch -o fetch -- python3 bench.py --roofline-only > gpurun_out/prof_fetch.log 2>&1; rc=$?
echo "== pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$R/pmc_write -o write -- python3 bench.py --roofline-only > gpurun_out/prof_write.log 2>&1; rc=$?
echo "== pmc write rc=$rc"
exit $rc
