#!/bin/bash
# Round-3 session A: forward-conv kernel variants (tools/fwd_bench), the fused
# optimizer-prep test, the C2 step kernel trace, a fused-prep A/B, and the
# FE-backward fp32 precision probe. Stops at the first abnormal exit.
set -u
D=gpurun_out/r3a
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 ./tools/fwd_bench > $D/fwd_bench.txt 2>&1; rc=$?
echo "== fwd_bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/fwd_bench.txt; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -k "fused_optimizer_prep or bitwise_deterministic" -x -q --timeout 300 --timeout-method thread > $D/prep_test.txt 2>&1; rc=$?
echo "== prep test rc=$rc"; tail -3 $D/prep_test.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/step -o step -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $D/prof_step.log 2>&1; rc=$?
echo "== prof step rc=$rc"; tail -1 $D/prof_step.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for f in "--fuse-prep off" "--fuse-prep on" "--fuse-prep off" "--fuse-prep on"; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra $f > $D/ab.json 2>$D/ab.err || { tail -5 $D/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$D/ab.json'));print('[$f]', d['ms_per_step'])"
done
timeout -k 10 500 python -u tools/probes/fe_bwd.py 6 10000 > $D/fe_bwd.txt 2>&1; rc=$?
echo "== fe_bwd rc=$rc"; tail -40 $D/fe_bwd.txt
exit $rc
