#!/bin/bash
# Round-4 session A: the P4-path precision probe, the L2 -> LDS feed bench,
# then the new / changed GPU tests (world-2 DP step, SyncBN uneven shards,
# trained-model decode parity). Stops at the first abnormal exit.
set -u
D=gpurun_out/r4a
mkdir -p $D
export TMPDIR=/tmp
P4_PERTURB=3 timeout -k 10 900 python -u tools/probes/p4_chain.py 6 10000 > $D/p4_chain.txt 2>&1; rc=$?
echo "== p4_chain rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/p4_chain.txt; exit $rc; }
timeout -k 10 120 ./tools/lds_feed_bench > $D/lds_feed.txt 2>&1; rc=$?
echo "== lds_feed rc=$rc"; cat $D/lds_feed.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./tools/fwd_bench_t > $D/tile_bench.txt 2>&1; rc=$?
echo "== tile bench rc=$rc"; cat $D/tile_bench.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_syncbn.py tests/test_gpu_dp_step.py \
  "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32" \
  "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -15 $D/tests.txt; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
exit $rc
