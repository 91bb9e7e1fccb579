#!/bin/bash
# Round-4 final evidence (outputs in gpurun_out/r4fin/): the whole -m gpu
# suite, smoke(), rocprofv3 kernel stats of the C2 step / roofline probe /
# R50-FPN headline, the roofline kernel's FETCH / WRITE passes turned into
# pmc/roofline_pmc.json (in the box's tree, copied back under gpurun_out),
# then the default bench line (which attaches that traffic), then the
# headline forward's PMC passes. Stops at the first abnormal exit.
set -u
D=gpurun_out/r4fin
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1300 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed" $D/tests.txt | tail -8; cp gpurun_out/parity.json $D/parity.json 2>/dev/null
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1; rc=$?
echo "== smoke rc=$rc"; tail -2 $D/smoke.txt; [ $rc -eq 0 ] || exit $rc
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
ff=$(find $D/roof_FETCH_SIZE -name "*counter_collection.csv" | head -1)
fw=$(find $D/roof_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py "$ff" "$fw" "gemm_pipe_kernel<128, 256, 2, 4, 2, 512, 3, 1, 64, 2>" 26869760 > $D/roofline_pmc_raw.json && \
python - "$D" <<'PY'
import json, sys
d = sys.argv[1]
r = json.load(open(d + "/roofline_pmc_raw.json"))
assert r["launches"] > 0, r
r["kernel"] = "gemm_pipe_kernel<128,256,2,4,A_IM2COL,512,3,1,64,2>"
r["launch"] = "conv3x3 256->256 on 32x28x28, M=25088 N=256 K=2304"
r["measured"] = "round 4 (final), tools/gpu_final_r4.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --roofline-only (gpurun_out/r4fin)"
json.dump(r, open("pmc/roofline_pmc.json", "w"), indent=1)
json.dump(r, open(d + "/roofline_pmc.json", "w"), indent=1)
print("traffic", r["hbm_bytes_per_launch"], "reread", r["reread_factor"])
PY
rc=$?; echo "== pmc json rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $D/bench.json 2> $D/bench.err; rc=$?
echo "== bench rc=$rc"; cut -c1-400 $D/bench.json; [ $rc -eq 0 ] || { tail -20 $D/bench.err; exit $rc; }
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_MFMA,GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $D/headpmc/pmc$i -o pmc -- python3 bench.py --headline-only > $D/headpmc$i.log 2>&1; rc=$?
  echo "== head pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
f=$(find $D/step -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$f" 30 > $D/step_breakdown.txt 2>&1; head -3 $D/step_breakdown.txt
python tools/step_counts.py "$f" > $D/step_counts.txt 2>&1; head -1 $D/step_counts.txt
