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

case "${1:-}" in
  a) "session_$1" ;;
  *) echo "usage: $0 <a>" >&2; exit 2 ;;
esac
