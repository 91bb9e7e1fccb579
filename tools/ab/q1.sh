set -u
mkdir -p gpurun_out/q1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_configs.py -x -q -m gpu -k "attention or logits or parity or bitwise or graph or c2" --timeout 300 --timeout-method thread > gpurun_out/q1/tests.log 2>&1; rc=$?
tail -3 gpurun_out/q1/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/q1/bench_base$i.json 2>gpurun_out/q1/bench_base$i.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/q1/bench_new$i.json 2>gpurun_out/q1/bench_new$i.err || exit 1
done
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/q1/*.json')):
    d=json.load(open(f)); print(f, d['ms_per_step'], d['value'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q1/step -o step -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/q1/prof.log 2>&1 && grep -i "attn_q1" gpurun_out/q1/step/step_kernel_stats.csv | cut -c1-160
