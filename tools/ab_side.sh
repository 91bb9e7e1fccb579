#!/bin/bash
# A/B of the weight-gradient side stream on one box (C2 step, no extras).
mkdir -p gpurun_out/ab
for m in off dense off dense; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --side-wgrad $m > gpurun_out/ab/$m.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab/$m.json'));print('$m', d['ms_per_step'])"
done
