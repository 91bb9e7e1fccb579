#!/bin/bash
# Final-tree check: the whole -m gpu suite, smoke(), the default bench line.
set -u
D=gpurun_out/r3q
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1; rc=$?
echo "== smoke rc=$rc"; tail -2 $D/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err; rc=$?
echo "== bench rc=$rc"; cut -c1-300 $D/bench.json; exit $rc
