#!/bin/bash
# A/B of the deferred weight-gradient job launches: builds of the library in
# tools/abj/ copied over the in-tree libfpnmt.so of the GPU box's copy of the
# tree (bench.py only measures the in-tree build), C2 step, alternating, two
# rounds; the sorted build is restored at the end.
LIB=fpn-mt-image-captioning_amd/fpnmt/libfpnmt.so
mkdir -p gpurun_out/abj
for r in 1 2; do
  for v in base sorted s2 kmax; do
    cp tools/abj/lib_jobs_$v.so $LIB
    timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/abj/run.json 2>gpurun_out/abj/run.err || { tail -5 gpurun_out/abj/run.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abj/run.json'));print('[$v]', d['ms_per_step'])" | tee -a gpurun_out/abj/ab.txt
  done
done
cp tools/abj/lib_jobs_sorted.so $LIB
