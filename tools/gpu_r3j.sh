#!/bin/bash
# Round-3 session J: forward / bwd-data conv tile variants on the C2 step's
# batch-32 shapes (tools/fwd_bench_l, FB_LIGHT build).
set -u
D=gpurun_out/r3j
mkdir -p $D
FB_FILTER=b32 timeout -k 10 240 ./tools/fwd_bench_l > $D/fwd_b32.txt 2>&1; rc=$?
echo "== fwd_b32 rc=$rc"; cat $D/fwd_b32.txt
exit $rc
