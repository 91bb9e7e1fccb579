#!/bin/bash
# A/B of two bench.py flag sets on one box (C2 step, no extras), alternating:
#   bash tools/ab_bench.sh "--defer off" "--defer on"
mkdir -p gpurun_out/ab
A="$1"; B="$2"
for r in 1 2; do
  for f in "$A" "$B"; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra $f > gpurun_out/ab/run.json 2>gpurun_out/ab/run.err || { tail -5 gpurun_out/ab/run.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab/run.json'));print('[$f]', d['ms_per_step'])"
  done
done
