set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/gemm.log
FPNMT_GEMM_LOG=gpurun_out/gemm.log timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gs -o gs -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-extra > gpurun_out/gs.log 2>&1
python3 tools/gemm_shapes.py gpurun_out/gemm.log gpurun_out/gs/gs_kernel_trace.csv > gpurun_out/gemm_shapes.txt
