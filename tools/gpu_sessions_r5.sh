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

case "${1:-}" in
  a|b|c|d) "session_$1" ;;
  *) echo "usage: $0 <a|b|c|d>" >&2; exit 2 ;;
esac
