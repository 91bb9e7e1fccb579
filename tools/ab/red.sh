set -u
mkdir -p gpurun_out/red
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q -m gpu -k "determin or deferred or split or atomic or bitwise or graph" --timeout 200 --timeout-method thread > gpurun_out/red/tests.log 2>&1; rc=$?
tail -3 gpurun_out/red/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/red/bench_base$i.json 2>gpurun_out/red/bench_base$i.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/red/bench_new$i.json 2>gpurun_out/red/bench_new$i.err || exit 1
done
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/red/*.json')):
    d=json.load(open(f)); print(f, d['ms_per_step'], d['value'])"
