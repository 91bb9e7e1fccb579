#!/bin/bash
# Same-box A/B of the in-tree libfpnmt.so against another build of it (the
# C2 step, no extras), alternating, two rounds:
#   hipcc ... -shared build/csrc/*.o -o tools/ab/libfpnmt_base.so   (before the change)
#   bash tools/ab_lib.sh tools/ab/libfpnmt_base.so
# FPNMT_LIBRARY (fpnmt/_lib.py) points the loader at the baseline build.
BASE=$(realpath "$1")
mkdir -p gpurun_out/ablib
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export FPNMT_LIBRARY=$BASE; else unset FPNMT_LIBRARY; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/ablib/run.json 2>gpurun_out/ablib/run.err || { tail -5 gpurun_out/ablib/run.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ablib/run.json'));print('[$lib]', d['ms_per_step'])"
  done
done
