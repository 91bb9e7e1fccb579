#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/hgemm.log
FPNMT_GEMM_LOG=gpurun_out/hgemm.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hs -o hs -- python3 tools/probes/headline_shapes.py > gpurun_out/hs.log 2>&1
