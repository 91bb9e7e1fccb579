#!/bin/bash
# Round-5 GPU sessions, one function per gpurun call:
#   tools/gpu_sessions_r5.sh <name>
# Each stops at the first abnormal exit; outputs under gpurun_out/r5<name>.
set -u
export TMPDIR=/tmp

run() {  # run <dir> <seconds> <log name> <cmd...>: time-limited step, stop the session on failure
  local d=$1 t=$2 log=$3; shift 3
  timeout -k 10 "$t" "$@" > "$d/$log" 2>&1; local rc=$?
  echo "== $log rc=$rc"; tail -6 "$d/$log"
  [ $rc -eq 0 ] || exit $rc
}

session_a() {
  # image-conditioned memorisation probe; the DP exchange tests (async gloo
  # worker, delayed async == sync, timeline)
  D=gpurun_out/r5a; mkdir -p $D
  run $D 600 train_cond.txt python -u tools/probes/train_cond.py
  run $D 900 dp_tests.txt python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_dp_step.py
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
}

session_b() {
  # the ping-pong conv kernel (gemm_pp.h) against the shipped pipe tiles on the
  # forward shapes: cold caches, then the C2 P3 conv warm
  D=gpurun_out/r5b; mkdir -p $D
  run $D 300 pp_cold.txt tools/bin_r5/fwd_bench_pp
  run $D 120 pp_p3_warm.txt env FB_FILTER="P3 3x3" FB_WARM=1 tools/bin_r5/fwd_bench_pp
  cat $D/pp_cold.txt
}

session_c() {
  # the 16x16x32 pipe tiles + widened epilogue stores (fwd_bench), the 2-layer
  # conditioning sweep, then the whole GPU suite on the rebuilt library
  D=gpurun_out/r5c; mkdir -p $D
  run $D 400 mf16_cold.txt tools/bin_r5/fwd_bench_pp
  run $D 400 train_cond_2L.txt python -u tools/probes/train_cond.py 2L
  run $D 900 gpu_tests.txt python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
}

session_d() {
  # the fused identity bottleneck (tests first: a new kernel), its timing and
  # the headline with / without it, the 2-layer conditioning sweep, then the
  # whole GPU suite on the MF 16 / widened-epilogue library
  D=gpurun_out/r5d; mkdir -p $D
  run $D 300 bottleneck_tests.txt python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bottleneck.py
  run $D 300 bottleneck_bench.txt python -u tools/probes/bottleneck_bench.py
  run $D 400 train_cond_2L.txt python -u tools/probes/train_cond.py 2L
  run $D 900 gpu_tests.txt python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  run $D 600 bench.json python bench.py
}

session_fin() {
  # round-5 evidence (gpurun_out/r5fin): the whole -m gpu suite, smoke(),
  # kernel stats of the C2 step / roofline probe / headline, the roofline
  # kernel's FETCH / WRITE passes -> pmc/roofline_pmc.json, the default bench
  # line (which attaches that traffic), the headline's and the step's PMC
  # passes (MFMA busy, HBM bytes) -> the top-kernel tables
  D=gpurun_out/r5fin; mkdir -p $D
  run $D 1300 tests.txt python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
  run $D 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
  for probe in step roof head; do
    case $probe in
      step) args="--steps 5 --warmup 2 --no-cpu-baseline --no-extra" ;;
      roof) args="--roofline-only" ;;
      head) args="--headline-only" ;;
    esac
    run $D 300 prof_$probe.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/$probe -o $probe -- python3 bench.py $args
  done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D/roof_$c -o pmc -- python3 bench.py --roofline-only > $D/roof_$c.log 2>&1; rc=$?
    echo "== roof pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  ff=$(find $D/roof_FETCH_SIZE -name "*counter_collection.csv" | head -1)
  fw=$(find $D/roof_WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python tools/pmc_traffic.py "$ff" "$fw" "gemm_pipe_kernel<128, 256, 2, 4, 2, 512, 3, 1, 64, 2, 16>" 26869760 > $D/roofline_pmc_raw.json && \
  python - "$D" <<'PY'
import json, sys
d = sys.argv[1]
r = json.load(open(d + "/roofline_pmc_raw.json"))
assert r["launches"] > 0, r
r["kernel"] = "gemm_pipe_kernel<128,256,2,4,A_IM2COL,512,3,1,64,2,16>"
r["launch"] = "conv3x3 256->256 on 32x28x28, M=25088 N=256 K=2304"
r["measured"] = "round 5 (final), tools/gpu_sessions_r5.sh fin: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --roofline-only (gpurun_out/r5fin)"
json.dump(r, open("pmc/roofline_pmc.json", "w"), indent=1)
json.dump(r, open(d + "/roofline_pmc.json", "w"), indent=1)
print("traffic", r["hbm_bytes_per_launch"], "reread", r["reread_factor"])
PY
  rc=$?; echo "== pmc json rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err; rc=$?
  echo "== bench rc=$rc"; cut -c1-400 $D/bench.json; [ $rc -eq 0 ] || { tail -20 $D/bench.err; exit $rc; }
}

session_fin2() {
  # the second half of the round-5 evidence (one gpurun call holds at most
  # 20 minutes): the headline's and the step's PMC passes, the breakdowns
  D=gpurun_out/r5fin; mkdir -p $D
  i=0
  for grp in "SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_MFMA,GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $D/headpmc/pmc$i -o pmc -- python3 bench.py --headline-only > $D/headpmc$i.log 2>&1; rc=$?
    echo "== head pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/steppmc/pmc$i -o pmc -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extra > $D/steppmc$i.log 2>&1; rc=$?
    echo "== step pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
  python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -1 $D/step_counts.txt
}

session_e() {
  # the fused bottleneck on a 3-slot DMA ring (two units in flight), the
  # image-conditioned decode tests
  D=gpurun_out/r5e; mkdir -p $D
  run $D 300 bottleneck_tests.txt python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bottleneck.py
  run $D 300 bottleneck_bench.txt python -u tools/probes/bottleneck_bench.py
  run $D 600 decode_tests.txt python -u -m pytest -x -v --timeout 500 --timeout-method thread "tests/test_gpu_configs.py::test_c5_beam8_trained_decode_matches_oracle_fp32" "tests/test_gpu_configs.py::test_greedy_trained_decode_matches_oracle_fp32"
  cp gpurun_out/parity.json $D/parity.json 2>/dev/null
}

session_f() {
  # fused bottleneck timing probes (tools/bn_bench.hip BN_PROBE 0 / 1 / 3),
  # the library form with the biases staged in LDS (tests + probe)
  D=gpurun_out/r5${TAG:-f}; mkdir -p $D
  for pr in 0 3; do run $D 120 bn_probe$pr.txt tools/bin_r5/bn_bench$pr; done
  run $D 300 bottleneck_tests.txt python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bottleneck.py
  run $D 300 bottleneck_bench.txt python -u tools/probes/bottleneck_bench.py
}

session_g() {
  # segmented deferred colsum jobs (no flush per head level), the 64-wide /
  # short-K weight-gradient tiles: kernel + deferred-reduction tests, the
  # step's kernel trace, the default bench line
  D=gpurun_out/r5${TAG:-g}; mkdir -p $D
  run $D 600 kernel_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py
  run $D 600 defer_tests.txt python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_model.py -k "deferred or bitwise or grad"
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
  run $D 600 bench.json python bench.py
}

session_h() {
  # the transformer's optimizer part beside the feature extractor's backward
  # (config.early_update): bitwise test + the deferred / model tests, the
  # step with it off / on (same box), the step's kernel trace
  D=gpurun_out/r5${TAG:-h}; mkdir -p $D
  run $D 600 early_tests.txt python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_model.py -k "early_update or deferred or bitwise"
  for e in off on off on; do
    run $D 300 bench_early_$e.json python bench.py --no-cpu-baseline --no-extra --steps 20 --early-update $e
    echo "early=$e $(python -c "import json;print(json.loads(open('$D/bench_early_$e.json').read().strip().splitlines()[-1])['ms_per_step'])")" >> $D/ab.txt
  done
  cat $D/ab.txt
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
}

session_hi() {
  # session h again (the early part on 64 persistent LDS-free workgroups), then i
  session_h
  session_i
}

session_j() {
  # the decoder's short-row GEMMs on 64x32 MF 16 tiles (N <= 1536): kernel,
  # model and decode tests, the default bench line, the step's kernel trace
  D=gpurun_out/r5${TAG:-j}; mkdir -p $D
  run $D 600 kernel_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py
  run $D 900 model_tests.txt python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_model.py -k "deferred or bitwise or early or drop or graph or greedy"
  run $D 600 bench.json python bench.py
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
}

session_k() {
  # the stem's weight gradient as its own kernel (conv_stem.hip): its test
  # first, then the kernel / model tests, the bench line, the step trace
  D=gpurun_out/r5${TAG:-k}; mkdir -p $D
  run $D 300 stem_tests.txt python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k stem_bwd_filter
  run $D 600 kernel_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py
  run $D 900 model_tests.txt python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_model.py -k "deferred or bitwise or graph"
  run $D 600 bench.json python bench.py
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
}

session_l() {
  # stem weight-gradient kernel v2 (register prefetch, wave-private T rows, two
  # blocks per CU): its test, the step trace, the bench line
  D=gpurun_out/r5${TAG:-l2}; mkdir -p $D
  run $D 300 stem_tests.txt python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k stem_bwd_filter
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt; grep stem_ $D/step_breakdown.txt
  run $D 600 bench.json python bench.py --no-cpu-baseline --no-extra --steps 20
}

session_m() {
  # the halo-staged 3x3 weight-gradient kernel (tools/wg_halo.h) against the
  # shipped LDS-DMA tiles (tools/wg_bench.hip -DWB_HALO)
  D=gpurun_out/r5${TAG:-m}; mkdir -p $D
  run $D 240 wg_halo.txt tools/bin_r5/wg_bench_halo
  cat $D/wg_halo.txt
}

session_n() {
  # confirmation of the tree to be committed: kernel tests, the bench line
  D=gpurun_out/r5${TAG:-n}; mkdir -p $D
  run $D 600 kernel_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py
  run $D 600 bench.json python bench.py
}

session_o() {
  # the consumers' bwd-data / max-pool backward with the producer's ReLU'
  # (fuse_input_act): its test, the fused-path model tests, the kernel tests,
  # the step trace, the bench line
  D=gpurun_out/r5${TAG:-o}; mkdir -p $D
  run $D 400 input_act_tests.txt python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "input_act or block_act or conv_chains or identity_residual or zero_grad_overlap or early_update or graph"
  run $D 400 dp_tests.txt python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp_step.py
  run $D 600 kernel_tests.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py
  run $D 300 prof_step.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
  f=$(find $D/step -name "*kernel_trace.csv" | head -1)
  python tools/step_breakdown.py "$f" 40 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
  run $D 600 bench.json python bench.py --no-cpu-baseline --no-extra --steps 20
}

session_p() {
  # which act_bwd passes remain (tools/probes/act_bwd_shapes.py, the calling
  # Function and layer), then session o
  D=gpurun_out/r5${TAG:-p}; mkdir -p $D
  run $D 300 act_bwd_sites.txt python -u tools/probes/act_bwd_shapes.py
  session_o
}

session_r() {
  # A/B on one box: the gradient arena's fill inline (0) / on a side stream
  # beside the forward (64, 256 workgroups), alternating; then the pool tests
  D=gpurun_out/r5${TAG:-r}; mkdir -p $D
  run $D 300 pool_tests.txt python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k maxpool
  for z in 0 64 0 64 256 0; do
    run $D 300 bench_z$z.json python bench.py --no-cpu-baseline --no-extra --steps 30 --zero-grad-grid $z
    echo "zero_grid=$z $(python -c "import json;print(json.loads(open('$D/bench_z$z.json').read().strip().splitlines()[-1])['ms_per_step'])")" >> $D/ab.txt
  done
  cat $D/ab.txt
}

session_t() {
  # AMSGrad with plain (cached) loads instead of non-temporal ones
  # (var/libfpnmt_plainld.so: optim.hip built with the ld lambda returning *a,
  # linked with the other objects; not kept) against the in-tree library:
  # kernel stats of a short step run each, then alternating benches
  # (profiles/r05/adam_loads_ab_r5t.txt: negative)
  D=gpurun_out/r5${TAG:-t}; mkdir -p $D
  T=fpn-mt-image-captioning_amd/fpnmt/libfpnmt.so
  cp $T var/libfpnmt_base.so
  for v in base plain base plain; do
    cp var/libfpnmt_$([ $v = plain ] && echo plainld || echo base).so $T  # the box's scratch copy only
    run $D 300 prof_$v.log rocprofv3 --kernel-trace --stats --output-format csv -d $D/st_$v -o st -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra
    f=$(find $D/st_$v -name "*kernel_stats.csv" | head -1)
    echo "$v $(grep amsgrad $f | cut -c1-200)" >> $D/ab.txt
    run $D 300 bench_$v.json python bench.py --no-cpu-baseline --no-extra --steps 30
    echo "$v $(python -c "import json;print(json.loads(open('$D/bench_$v.json').read().strip().splitlines()[-1])['ms_per_step'])")" >> $D/ab.txt
  done
  cp var/libfpnmt_base.so $T
  cat $D/ab.txt
}

session_i() {
  # the decoder's short-row GEMMs (M = 992) on the pipe kernel's tile / MFMA
  # variants (tools/small_bench.hip -DSB_PIPE, graph replay)
  D=gpurun_out/r5${TAG:-i}; mkdir -p $D
  run $D 300 small_pipe.txt tools/bin_r5/small_bench_pipe
  cat $D/small_pipe.txt
}

case "${1:-}" in
  a|b|c|d|e|f|g|h|i|hi|j|k|l|m|n|o|p|r|t|fin|fin2) "session_$1" ;;
  *) echo "usage: $0 <a|b|c|d|e|f|g|h|i|hi|j|k|l|m|n|o|p|r|t|fin|fin2>" >&2; exit 2 ;;
esac
