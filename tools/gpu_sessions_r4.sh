#!/bin/bash
# Round-4 GPU sessions, one function per gpurun call (they were tools/gpu_r4a.sh
# .. gpu_r4t.sh). Run one as:  tools/gpu_sessions_r4.sh <a..t>
# Each stops at the first abnormal exit; outputs under gpurun_out/r4<x>.
# Kept as the record of how each profiles/r04/ file was produced; the bench
# binaries they name are built by the recipes in tools/README.md.
set -u

session_a() {
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
}

session_b() {
  # Round-4 session B: the P4-path probe with perturbed inputs (lr 0), the
  # trained-model decode parity tests. Stops at the first abnormal exit.
  set -u
  D=gpurun_out/r4b
  mkdir -p $D
  export TMPDIR=/tmp
  P4_PERTURB=4 timeout -k 10 900 python -u tools/probes/p4_chain.py 6 10000 > $D/p4_chain.txt 2>&1; rc=$?
  echo "== p4_chain rc=$rc"; grep -A8 "perturbed inputs" $D/p4_chain.txt; [ $rc -eq 0 ] || { tail -5 $D/p4_chain.txt; exit $rc; }
  timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread \
    "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32" \
    "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
    "tests/test_gpu_configs.py::test_c5_beam8_decode_matches_oracle_fp32" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "^image|passed|failed|Error" $D/tests.txt | head -30; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  exit $rc
}

session_c() {
  # Round-4 session C: the C2-model gradient parity at the 1e-5 bulk floor
  # (medians over three inputs), the peaked co-attention backward test, the
  # trained-model C5 decode parity. Stops at the first abnormal exit.
  set -u
  D=gpurun_out/r4c
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 1100 python -u -m pytest -x -v --timeout 1000 --timeout-method thread \
    "tests/test_gpu_kernels.py::test_spatial_softmax_peaked_bwd_vs_fp64" \
    "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
    "tests/test_gpu_model.py::test_train_step_parity_c2_model_fp32" -s > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "^image|passed|failed|Error|peaked|grad p90|grad max" $D/tests.txt | head -40; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  exit $rc
}

session_d() {
  # Round-4 session D: the whole -m gpu suite (fused encoder view projection,
  # DP / SyncBN / trained-decode / C2-parity tests), smoke(), a C2 step bench
  # and one profiled step (kernel count, breakdown). Stops at the first
  # abnormal exit.
  set -u
  D=gpurun_out/r4d
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 1000 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed" $D/tests.txt | tail -12; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  # 0 = green, 1 = assertion failures (read them afterwards); anything else
  # (a crash, a fault, a time limit) ends the session here
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1; rc=$?
  echo "== smoke rc=$rc"; tail -2 $D/smoke.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cat $D/bench_step.json | cut -c1-600; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(ls $D/step/*/step_kernel_trace.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -22 $D/step_breakdown.txt
  timeout -k 10 200 python tools/probes/headline_blas.py > $D/headline_blas.txt 2>&1; rc=$?
  echo "== headline blas rc=$rc"; cat $D/headline_blas.txt
}

session_f() {
  # Round-4 session F: LayerNorm-written dropout backward, consumer-summed
  # gradients (no autograd adds), batched wgrad read-modify-write, the 6-layer
  # trained decode at lr 1e-4: the targeted GPU tests, then a C2 step bench and
  # one profiled step. Stops at the first abnormal exit.
  set -u
  D=gpurun_out/r4f
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 1100 python -u -m pytest -m gpu -q --timeout 900 --timeout-method thread \
    tests/test_gpu_model.py tests/test_gpu_dp_step.py tests/test_gpu_kernels.py \
    "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
    "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -15; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-500 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -22 $D/step_breakdown.txt
}

session_h() {
  # Round-4 session H: grouped view attention / view LayerNorms, C5 warm-up schedule:
  set -u
  D=gpurun_out/r4h
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 1100 python -u -m pytest -m gpu -q --timeout 900 --timeout-method thread \
    tests/test_gpu_model.py tests/test_gpu_dp_step.py tests/test_gpu_kernels.py \
    "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" \
    "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -15; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-500 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -22 $D/step_breakdown.txt
}

session_i() {
  # Round-4 session I: the whole -m gpu suite after the launch-chain work
  # (grouped view attention / view LayerNorms, embedding dropout, step
  # targets kernel), then a C2 step bench and one profiled step.
  set -u
  D=gpurun_out/r4i
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -15; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-400 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -5 $D/step_breakdown.txt
  python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -40 $D/step_counts.txt
}

session_j() {
  # Round-4 session J: int32 step targets, P7 in the heads stage:
  # (grouped view attention / view LayerNorms, embedding dropout, step
  # targets kernel), then a C2 step bench and one profiled step.
  set -u
  D=gpurun_out/r4j
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -15; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-400 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -5 $D/step_breakdown.txt
  python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -40 $D/step_counts.txt
}

session_m() {
  # Round-4 session M: the transformer's Dense weight gradients deferred and
  # run as grouped whole-K tile launches at the backward's flush
  # (gemm_wg_jobs_kernel): targeted GPU tests, a C2 step bench, one profiled
  # step and the per-shape GEMM table of an eager step.
  set -u
  D=gpurun_out/r4m
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 600 --timeout-method thread \
    "tests/test_gpu_model.py::test_deferred_dense_wgrads_match_immediate" tests/test_gpu_model.py \
    tests/test_gpu_dp_step.py > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error|largest" $D/tests.txt | tail -12
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-300 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
  python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -25 $D/step_counts.txt
  rm -f gpurun_out/gemm.log
  FPNMT_GEMM_LOG=$D/gemm.log timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/gs -o gs -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-extra > $D/gs.log 2>&1; rc=$?
  echo "== gemm shapes rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/gemm_shapes.py $D/gemm.log $(find $D/gs -name "*kernel_trace.csv" | head -1) > $D/gemm_shapes.txt 2>&1; head -30 $D/gemm_shapes.txt
}

session_n() {
  # Round-4 session N: ffn1's LeakyReLU backward in ffn2's bwd-data epilogue
  # (fpnmt_gemm_act_in): the model tests, the C2 bench, one profiled step.
  set -u
  D=gpurun_out/r4n
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 600 --timeout-method thread \
    tests/test_gpu_model.py tests/test_gpu_dp_step.py "tests/test_gpu_configs.py::test_c2_logits_and_loss_parity_fp32" "tests/test_gpu_configs.py::test_c2_train_step_fp32_then_bf16" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -12
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 30 > $D/bench_step.json 2> $D/bench_step.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-300 $D/bench_step.json; [ $rc -eq 0 ] || { tail -20 $D/bench_step.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
  echo "== prof step rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
  python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -12 $D/step_counts.txt
}

session_o() {
  # Round-4 session O: the FFN-fusion test's bf16 bar (norm-wise over the
  # feature extractor), and the pipe kernel's spread-DMA variants
  # (tools/fwd_bench.hip -DFB_SPREAD, built beforehand into tools/bin).
  set -u
  D=gpurun_out/r4o
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_model.py::test_ffn_act_fused_matches" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  FB_FILTER=b32 timeout -k 10 300 tools/bin/fwd_bench_spread > $D/spread_b32.txt 2>&1; rc=$?
  echo "== spread b32 rc=$rc"; cat $D/spread_b32.txt; [ $rc -eq 0 ] || exit $rc
  FB_FILTER="P3 3x3" FB_WARM=1 timeout -k 10 300 tools/bin/fwd_bench_spread > $D/spread_p3_warm.txt 2>&1; rc=$?
  echo "== spread P3 warm rc=$rc"; cat $D/spread_p3_warm.txt; [ $rc -eq 0 ] || exit $rc
}

session_p() {
  # Round-4 session P: the FFN-fusion test (norm-wise FE bar), then a same-box
  # A/B of the spread-DMA pipe kernel in the dispatch: base (cfg 3 = 128x256
  # 2-stage), c3 (cfg 3 = 3-stage, DMA spread between k-steps, MFMA priority),
  # c34 (also cfg 4 = 64x64 4-stage spread).
  set -u
  D=gpurun_out/r4p
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_model.py::test_ffn_act_fused_matches" "tests/test_gpu_kernels.py" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  bash tools/ab_libs.sh 2 base c3 c34; rc=$?
  echo "== ab rc=$rc"; exit $rc
}

session_q() {
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
}

session_r() {
  # Round-4 session R: the ordered slab sum with its last round's loads in
  # flight together (predicated adds): the determinism / deferred-reduction
  # tests, then a same-box A/B against the previous build (c34).
  set -u
  D=gpurun_out/r4r
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread \
    tests/test_gpu_model.py -k "determin or deferred or graph" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  bash tools/ab_libs.sh 2 c34 slab8; rc=$?
  echo "== ab rc=$rc"; exit $rc
}

session_s() {
  # Round-4 session S: the EPI-0 pipe kernel's residual / act-mask rows
  # prefetched before its K loop: kernel + fused-epilogue model tests, then a
  # same-box A/B against the previous build (slab8).
  set -u
  D=gpurun_out/r4s
  mkdir -p $D
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_model.py -k "not c2_model and not parity_c2" > $D/tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $D/tests.txt | tail -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  bash tools/ab_libs.sh 2 slab8 rpre; rc=$?
  echo "== ab rc=$rc"; exit $rc
}

session_t() {
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
}

case "${1:-}" in
  a|b|c|d|f|h|i|j|m|n|o|p|q|r|s|t) "session_$1" ;;
  *) echo "usage: $0 <a|b|c|d|f|h|i|j|m|n|o|p|q|r|s|t>" >&2; exit 2 ;;
esac
