#!/bin/bash
set -e
for c in 1 2; do
  FPNMT_WG_CFG=$c timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv_fwd_bwd or dense or linear" > gpurun_out/t_wg$c.log 2>&1
done
for c in 0 1 2; do
  FPNMT_WG_CFG=$c timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > gpurun_out/bench_wg$c.log 2>&1
done
FPNMT_NO_PIPE_WG=1 timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > gpurun_out/bench_wgoff.log 2>&1
