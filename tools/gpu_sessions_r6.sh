#!/bin/bash
# Round-6 GPU sessions, one function per gpurun call:
#   tools/gpu_sessions_r6.sh <name>
# Each stops at the first abnormal exit; outputs under gpurun_out/r6<name>.
set -u
export TMPDIR=/tmp

try() {  # try <dir> <seconds> <log name> <cmd...>: time-limited step; a test failure (rc 1) goes on, anything else stops
  local d=$1 t=$2 log=$3; shift 3
  timeout -k 10 "$t" "$@" > "$d/$log" 2>&1; local rc=$?
  echo "== $log rc=$rc"; tail -6 "$d/$log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}

run() {  # run <dir> <seconds> <log name> <cmd...>: time-limited step, stop the session on failure
  local d=$1 t=$2 log=$3; shift 3
  timeout -k 10 "$t" "$@" > "$d/$log" 2>&1; local rc=$?
  echo "== $log rc=$rc"; tail -6 "$d/$log"
  [ $rc -eq 0 ] || exit $rc
}

session_a() {
  # C4 on one box: the C4-model world-2 exchange test, the bf16-vs-oracle
  # bound at C2, the bench's N > 1 branch under a gloo rehearsal (two ranks,
  # one GPU, 64 images each), and the N = 1 bench line with the split-step leg
  D=gpurun_out/r6a; mkdir -p $D
  run $D 300 capi.txt python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_capi.py
  try $D 600 bf16_bound.txt python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_configs.py -k bf16_perf_path
  cp gpurun_out/parity.json $D/parity_bf16.json 2>/dev/null
  run $D 1000 dp_c4.txt python -u -m pytest -x -v -s --timeout 950 --timeout-method thread tests/test_gpu_dp_step.py -k c4_model
  cp gpurun_out/parity.json $D/parity_dp_c4.json 2>/dev/null
  FPNMT_DIST_BACKEND=gloo run $D 600 bench_world2_gloo.json python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --timeline $D/timeline2
  run $D 900 bench.json python bench.py
}

session_b() {
  # the loader-wave dispatch (cfgs 6 / 7 / 8): the whole -m gpu suite, the
  # default bench line, the step's kernel trace
  D=gpurun_out/r6b; mkdir -p $D
  run $D 300 wg_lw.txt tools/bin_r6/wg_bench_lw
  try $D 900 tests.txt python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  run $D 900 bench.json python bench.py
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
}

session_c() {
  # the loader-wave weight gradients (8 loaders on 128x256, 4 on the A_COL
  # 128x128 tiles) in the library, the short-row loader probe, the suite, bench
  D=gpurun_out/r6${R6TAG:-c}; mkdir -p $D
  try $D 900 tests.txt python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  run $D 900 bench.json python bench.py --no-cpu-baseline
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
}

session_i() {
  # kernel stats of the forward-only probes (headline R50-FPN b64, C3 R101-FPN
  # 512^2 b64) on the loader-wave library, and the 1x1 / 3x3 shape sweep
  D=gpurun_out/r6i; mkdir -p $D
  run $D 300 prof_head.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/head -o head -- python3 bench.py --headline-only
  run $D 300 prof_c3.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/c3 -o c3 -- python3 bench.py --c3-only
  run $D 300 c3_shapes.txt env FB_FILTER=c3 tools/bin_r6/fwd_bench_lw
}

session_fin() {
  # round-6 evidence (gpurun_out/r6fin): the whole -m gpu suite, smoke(), the
  # kernel stats of the step / roofline probe / headline / C3, the roofline
  # kernel's FETCH / WRITE passes -> pmc/roofline_pmc.json, the default bench
  # line (which attaches that traffic)
  D=gpurun_out/r6${R6TAG:-fin}; rm -rf $D; mkdir -p $D
  run $D 1300 tests.txt python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  run $D 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
  for probe in step roof head c3; do
    case $probe in
      step) args="--steps 5 --warmup 2 --no-cpu-baseline --no-extra" ;;
      roof) args="--roofline-only" ;;
      head) args="--headline-only" ;;
      c3) args="--c3-only" ;;
    esac
    run $D 300 prof_$probe.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/$probe -o $probe -- python3 bench.py $args
  done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D/roof_$c -o pmc -- python3 bench.py --roofline-only > $D/roof_$c.log 2>&1; rc=$?
    echo "== roof pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  ff=$(find $D/roof_FETCH_SIZE -name "*counter_collection.csv" | head -1)
  fw=$(find $D/roof_WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python tools/pmc_traffic.py "$ff" "$fw" "gemm_pipe_lw_kernel<128, 256, 1, 8, 2, 4, 3, 112>" 26869760 > $D/roofline_pmc_raw.json && \
  python - "$D" <<'PY'
import json, sys
d = sys.argv[1]
r = json.load(open(d + "/roofline_pmc_raw.json"))
assert r["launches"] > 0, r
r["kernel"] = "gemm_pipe_lw_kernel<128,256,1,8,A_IM2COL,4,3,112>"
r["launch"] = "conv3x3 256->256 on 32x28x28, M=25088 N=256 K=2304"
r["measured"] = "round 6 (final), tools/gpu_sessions_r6.sh fin: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --roofline-only (gpurun_out/r6fin)"
json.dump(r, open("pmc/roofline_pmc.json", "w"), indent=1)
json.dump(r, open(d + "/roofline_pmc.json", "w"), indent=1)
print("traffic", r["hbm_bytes_per_launch"], "reread", r["reread_factor"])
PY
  rc=$?; echo "== pmc json rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-400 $D/bench.json; [ $rc -eq 0 ] || { tail -20 $D/bench.err; exit $rc; }
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
  python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -1 $D/step_counts.txt
}

session_fin2() {
  # the headline's and the step's PMC passes (MFMA busy, HBM bytes)
  D=gpurun_out/r6${R6TAG:-fin}; mkdir -p $D
  i=0
  for grp in "SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_MFMA,GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $D/headpmc/pmc$i -o pmc -- python3 bench.py --headline-only > $D/headpmc$i.log 2>&1; rc=$?
    echo "== head pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/steppmc/pmc$i -o pmc -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extra > $D/steppmc$i.log 2>&1; rc=$?
    echo "== step pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}

session_k() {
  # the beam step / decode attention rework: decode tests, C5 probe x2, suite, bench
  D=gpurun_out/r6${R6TAG:-k}; mkdir -p $D
  run $D 600 decode_tests.txt python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_decode.py
  run $D 300 c5a.json python bench.py --c5-only
  run $D 300 c5b.json python bench.py --c5-only
  run $D 300 prof_c5.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/c5 -o c5 -- python3 bench.py --c5-only
  try $D 900 tests.txt python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  run $D 900 bench.json python bench.py --no-cpu-baseline
}

session_d() {
  # decode-only iteration: decode tests, C5 probe x2, C5 kernel stats
  D=gpurun_out/r6${R6TAG:-d}; mkdir -p $D
  run $D 600 decode_tests.txt python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_decode.py
  run $D 300 c5a.json python bench.py --c5-only
  run $D 300 c5b.json python bench.py --c5-only
  run $D 300 prof_c5.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/c5 -o c5 -- python3 bench.py --c5-only
  [ -x tools/bin_r6/fwd_bench_lw2 ] && run $D 400 lw2.txt tools/bin_r6/fwd_bench_lw2
  true
}

session_e() {
  # decode-attention variants (tools/dec_attn_bench), decode tests, C5 x2
  D=gpurun_out/r6${R6TAG:-e}; mkdir -p $D
  run $D 120 dec_attn.txt tools/bin_r6/dec_attn_bench
  run $D 600 decode_tests.txt python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_decode.py
  run $D 300 c5a.json python bench.py --c5-only
  run $D 300 c5b.json python bench.py --c5-only
}

session_tests() {
  # the whole -m gpu suite
  D=gpurun_out/r6tests; mkdir -p $D
  run $D 1300 tests.txt python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
}

session_m() {
  rm -rf gpurun_out/r6m
  # the wide conv class's tile by per-CU L2 -> LDS bytes (cfg 6 128x256,
  # cfg 10 224x128, cfg 11 208x128; FPNMT_WIDE_CFG forces): conv tests,
  # roofline probe and headline A/B, kernel stats, bench (auto rule)
  D=gpurun_out/r6${R6TAG:-m}; mkdir -p $D
  run $D 600 conv_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "conv"
  for i in 1 2; do
    for c in 6 10 11; do
      FPNMT_WIDE_CFG=$c run $D 200 roof_c${c}_$i.json python bench.py --roofline-only
    done
  done
  for c in 6 10 11; do
    FPNMT_WIDE_CFG=$c run $D 200 head_c$c.json python bench.py --headline-only
  done
  run $D 300 prof_roof.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/roof -o roof -- python3 bench.py --roofline-only
  FPNMT_WIDE_CFG=6 run $D 300 prof_roof6.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/roof6 -o roof6 -- python3 bench.py --roofline-only
  run $D 600 bench.json python bench.py --no-cpu-baseline
}

session_f() {
  # the bias column sums folded into the weight-gradient kernel: the fold test,
  # the deferred / determinism / grouped tests, the C2 parity tests, bench, step trace
  D=gpurun_out/r6${R6TAG:-f}; rm -rf $D; mkdir -p $D
  try $D 600 fold_tests.txt python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "bias or grouped or wide_tiles or deferred"
  try $D 900 model_tests.txt python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_model.py
  run $D 600 bench.json python bench.py --no-cpu-baseline
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -20 $D/step_breakdown.txt
}

session_r() {
  # the roofline probe timed from a captured graph of its 20 launches: probe x2,
  # its kernel stats, the default bench line
  D=gpurun_out/r6${R6TAG:-r}; rm -rf $D; mkdir -p $D
  run $D 200 roof1.json python bench.py --roofline-only
  run $D 200 roof2.json python bench.py --roofline-only
  run $D 300 prof_roof.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/roof -o roof -- python3 bench.py --roofline-only
  run $D 600 bench.json python bench.py
  FPNMT_GEMM_LOG=$D/gemm.log run $D 300 gemm_log.txt python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra
}

session_s() {
  # strided 1x1 bwd-data on the pipe kernels + scatter pass: conv tests, model
  # tests, bench, step trace
  D=gpurun_out/r6${R6TAG:-s}; rm -rf $D; mkdir -p $D
  try $D 600 conv_tests.txt python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "conv"
  try $D 900 model_tests.txt python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_model.py
  run $D 600 bench.json python bench.py --no-cpu-baseline
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
}

session_t() {
  # tall row GEMMs on the conv pipe tiles: GEMM / model tests, bench, step trace
  D=gpurun_out/r6${R6TAG:-t}; rm -rf $D; mkdir -p $D
  try $D 600 gemm_tests.txt python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or dense or linear or attention"
  try $D 900 model_tests.txt python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_model.py
  run $D 600 bench.json python bench.py --no-cpu-baseline --no-extra
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
}

session_last() {
  # the committed tree: the whole -m gpu suite, smoke(), the default bench line
  D=gpurun_out/r6${R6TAG:-last}; rm -rf $D; mkdir -p $D
  run $D 1300 tests.txt python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread
  run $D 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
  run $D 900 bench.json python bench.py
}

session_u() {
  # the 128x128 loader tile at the 112-row M step (cfg 11) against cfg 7
  D=gpurun_out/r6${R6TAG:-u}; rm -rf $D; mkdir -p $D
  run $D 600 conv_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "conv"
  for i in 1 2; do
    FPNMT_WIDE_CFG=6 run $D 200 head_c6_$i.json python bench.py --headline-only
    run $D 200 head_auto_$i.json python bench.py --headline-only
  done
  FPNMT_WIDE_CFG=6 run $D 300 c3_c6.json python bench.py --c3-only
  run $D 300 c3_auto.json python bench.py --c3-only
  run $D 300 prof_head.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/head -o head -- python3 bench.py --headline-only
  run $D 600 bench.json python bench.py --no-cpu-baseline --no-extra
}

"session_$1"
