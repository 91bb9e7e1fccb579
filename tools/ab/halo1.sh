set -u
mkdir -p gpurun_out/h1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "halo or conv or grouped" --timeout 120 --timeout-method thread > gpurun_out/h1/tests.log 2>&1; rc=$?
tail -4 gpurun_out/h1/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/conv_bench.py --only r2_3x3,r3_3x3,r4_3x3,r5_3x3,fpn_p3,c2_p3_b32 --lib tools/ab/libfpnmt_base.so > gpurun_out/h1/cb_base.log 2>&1 && \
timeout -k 10 120 python tools/conv_bench.py --only r2_3x3,r3_3x3,r4_3x3,r5_3x3,fpn_p3,c2_p3_b32 --check > gpurun_out/h1/cb_new.log 2>&1 && \
cat gpurun_out/h1/cb_base.log gpurun_out/h1/cb_new.log && \
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h1/bench_base.json 2>gpurun_out/h1/bench_base.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h1/bench_new.json 2>gpurun_out/h1/bench_new.err && \
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h1/bench_base2.json 2>gpurun_out/h1/bench_base2.err && \
cut -c1-250 gpurun_out/h1/bench_*.json
