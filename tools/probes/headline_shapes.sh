#!/bin/bash
# Per-GEMM-shape times of the R50-FPN forward at batch 64 (two eager passes
# under a kernel trace; the second is reported by tools/gemm_shapes.py).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/hgemm.log gpurun_out/hs
FPNMT_GEMM_LOG=gpurun_out/hgemm.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hs -o hs -- python3 tools/probes/headline_shapes.py > gpurun_out/hs.log 2>&1
