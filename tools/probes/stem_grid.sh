#!/bin/bash
set -e
export TMPDIR=/tmp
for g in 768 1536 100000; do
  FPNMT_DBG_STEM_GRID=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sg$g -o sg -- python3 tools/probes/headline_shapes.py > gpurun_out/sg$g.log 2>&1
done
