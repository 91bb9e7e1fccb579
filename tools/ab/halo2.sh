set -u
mkdir -p gpurun_out/h5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "halo or conv or grouped" --timeout 120 --timeout-method thread > gpurun_out/h5/tests.log 2>&1; rc=$?
tail -3 gpurun_out/h5/tests.log; [ $rc -eq 0 ] || exit $rc
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h5/bench_base.json 2>gpurun_out/h5/bench_base.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h5/bench_new.json 2>gpurun_out/h5/bench_new.err && \
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h5/bench_base2.json 2>gpurun_out/h5/bench_base2.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h5/bench_new2.json 2>gpurun_out/h5/bench_new2.err && \
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/h5/bench_*.json')):
    d=json.load(open(f)); print(f, d['ms_per_step'], d['value'])" && \
rm -f gpurun_out/gemm.log && FPNMT_GEMM_LOG=gpurun_out/gemm.log timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gs -o gs -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-extra > gpurun_out/gs.log 2>&1 && \
python3 tools/gemm_shapes.py gpurun_out/gemm.log gpurun_out/gs/gs_kernel_trace.csv > gpurun_out/h5/gemm_shapes.txt && head -45 gpurun_out/h5/gemm_shapes.txt
