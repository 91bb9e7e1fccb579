set -u
mkdir -p gpurun_out/h6
for lib in base new; do
  if [ $lib = base ]; then export FPNMT_LIBRARY=$PWD/tools/ab/libfpnmt_base.so; else unset FPNMT_LIBRARY; fi
  timeout -k 10 200 python bench.py --headline-only > gpurun_out/h6/head_$lib.json 2>gpurun_out/h6/head_$lib.err || exit $?
  timeout -k 10 200 python bench.py --c3-only > gpurun_out/h6/c3_$lib.json 2>gpurun_out/h6/c3_$lib.err || exit $?
done
unset FPNMT_LIBRARY
timeout -k 10 120 python tools/probes/launch_floor.py > gpurun_out/h6/floor.log 2>&1
tail -c 600 gpurun_out/h6/head_*.json gpurun_out/h6/c3_*.json; cat gpurun_out/h6/floor.log
