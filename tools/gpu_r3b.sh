#!/bin/bash
# Round-3 session B: forward-conv variants with the shared wide main loop
# (tools/fwd_bench_l, FB_LIGHT build) and the weight-gradient variants
# (tools/wg_bench). Stops at the first abnormal exit.
set -u
D=gpurun_out/r3b
mkdir -p $D
timeout -k 10 240 ./tools/fwd_bench_l > $D/fwd_bench_l.txt 2>&1; rc=$?
echo "== fwd_bench_l rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/fwd_bench_l.txt; exit $rc; }
timeout -k 10 240 ./tools/wg_bench > $D/wg_bench.txt 2>&1; rc=$?
echo "== wg_bench rc=$rc"; cat $D/wg_bench.txt
exit $rc
