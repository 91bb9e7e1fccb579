#!/bin/bash
# Runs the GPU test files one after another; stops at the first run that did
# not end in a normal pass/fail (pytest rc 0/1), e.g. a fault or a timeout.
mkdir -p gpurun_out
for f in "$@"; do
  name=$(basename "$f" .py)
  timeout -k 10 900 python -m pytest "$f" -q -x -m gpu -s > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $f rc=$rc"; tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
done
