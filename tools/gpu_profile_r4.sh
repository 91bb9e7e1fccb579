#!/bin/bash
# Round-4 end evidence (outputs in gpurun_out/${1:-r4z}/): the whole -m gpu suite,
# smoke(), the default bench line, rocprofv3 kernel stats of the C2 step /
# roofline probe / R50-FPN headline, the roofline kernel's FETCH / WRITE
# passes and the headline forward's PMC passes (MFMA busy, HBM fetch, HBM
# write; one counter group per run). Stops at the first abnormal exit.
set -u
D=gpurun_out/${1:-r4z}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1300 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed" $D/tests.txt | tail -8; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1; rc=$?
echo "== smoke rc=$rc"; tail -2 $D/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $D/bench.json 2> $D/bench.err; rc=$?
echo "== bench rc=$rc"; cut -c1-300 $D/bench.json; [ $rc -eq 0 ] || { tail -20 $D/bench.err; exit $rc; }
for probe in step roof head; do
  case $probe in
    step) args="--steps 5 --warmup 2 --no-cpu-baseline --no-extra" ;;
    roof) args="--roofline-only" ;;
    head) args="--headline-only" ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$probe -o $probe -- python3 bench.py $args > $D/prof_$probe.log 2>&1; rc=$?
  echo "== prof $probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D/roof_$c -o pmc -- python3 bench.py --roofline-only > $D/roof_$c.log 2>&1; rc=$?
  echo "== roof pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_MFMA,GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $D/headpmc/pmc$i -o pmc -- python3 bench.py --headline-only > $D/headpmc$i.log 2>&1; rc=$?
  echo "== head pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -1 $D/step_counts.txt
