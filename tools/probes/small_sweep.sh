#!/bin/bash
# A/B of the small-M GEMM path: split-K factor and tiled-kernel configs
F="${F:-ffn2,vocab,view,enc,proj,wgrad}"
for v in "" "FPNMT_DBG_SMALL_SPLIT=1" "FPNMT_DBG_SMALL_SPLIT=2" "FPNMT_DBG_SMALL_SPLIT=4"; do
  echo "== $v"
  env $v timeout -k 10 100 python tools/probes/gemm_bench.py 30 "$F" || exit $?
done
