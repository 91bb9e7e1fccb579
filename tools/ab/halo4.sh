set -u
mkdir -p gpurun_out/h7
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "halo or conv or grouped" --timeout 120 --timeout-method thread > gpurun_out/h7/tests.log 2>&1; rc=$?
tail -3 gpurun_out/h7/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h7/bench_base$i.json 2>gpurun_out/h7/bench_base$i.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 > gpurun_out/h7/bench_new$i.json 2>gpurun_out/h7/bench_new$i.err || exit 1
done
for lib in base new; do
  if [ $lib = base ]; then export FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so; else unset FPNMT_LIBRARY; fi
  timeout -k 10 200 python bench.py --headline-only > gpurun_out/h7/head_$lib.json 2>gpurun_out/h7/head_$lib.err || exit $?
  timeout -k 10 200 python bench.py --c3-only > gpurun_out/h7/c3_$lib.json 2>gpurun_out/h7/c3_$lib.err || exit $?
done
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/h7/*.json')):
    d=json.load(open(f)); print(f, d.get('ms_per_step'), d.get('value'), {k: v.get('ms') for k, v in d.items() if isinstance(v, dict) and 'ms' in v})"
