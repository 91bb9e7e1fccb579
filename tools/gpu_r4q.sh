#!/bin/bash
# Round-4 session Q: the weight-gradient pipe kernel with its next K-tile's
# DMA spread between the k-steps (tools/wg_bench.hip -DWB_SPREAD), then a
# same-box A/B of the library with it dispatched: c34 (in-tree, no wgrad
# spread), w1 (spread), w2 (spread + MFMA priority).
set -u
D=gpurun_out/r4q
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 tools/bin/wg_bench_spread > $D/wg_spread.txt 2>&1; rc=$?
echo "== wg spread rc=$rc"; cat $D/wg_spread.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh 2 c34 w1 w2; rc=$?
echo "== ab rc=$rc"; exit $rc
