#!/bin/bash
# Round-3 session D: full GPU suite, then a same-box A/B of the in-tree
# library against abbase/libfpnmt_base.so (swapped in place; restored).
set -u
D=gpurun_out/r3d
mkdir -p $D
L=fpn-mt-image-captioning_amd/fpnmt/libfpnmt.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -4 $D/tests.txt; [ $rc -le 1 ] || exit $rc
cp $L /tmp/new.so
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then cp abbase/libfpnmt_base.so $L; else cp /tmp/new.so $L; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $D/ab.json 2>$D/ab.err || { cp /tmp/new.so $L; tail -5 $D/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$D/ab.json'));print('[$lib]', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
cp /tmp/new.so $L
timeout -k 10 200 python bench.py --headline-only > $D/headline.json 2>$D/headline.err; rc=$?
echo "== headline rc=$rc"; cut -c1-400 $D/headline.json
exit $rc
