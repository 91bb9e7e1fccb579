#!/bin/bash
# Round-4 session T: the stream-K 128x256 conv kernel (tools/fwd_bench.hip
# -DFB_SPREAD, "stream-K" rows; the error column covers the first and the
# last timed launch, i.e. the tile counters across replays).
set -u
D=gpurun_out/r4t
mkdir -p $D
FB_FILTER="P3 3x3" FB_VAR="128x256" timeout -k 10 200 tools/bin/fwd_bench_sk > $D/sk_p3.txt 2>&1; rc=$?
echo "== sk P3 rc=$rc"; cat $D/sk_p3.txt; [ $rc -eq 0 ] || exit $rc
FB_FILTER="P3 3x3" FB_VAR="128x256" FB_WARM=1 timeout -k 10 200 tools/bin/fwd_bench_sk > $D/sk_p3_warm.txt 2>&1; rc=$?
echo "== sk P3 warm rc=$rc"; cat $D/sk_p3_warm.txt; [ $rc -eq 0 ] || exit $rc
