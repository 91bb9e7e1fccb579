#!/bin/bash
# Round-end evidence for profiles/<round>/: the default bench line (CPU
# baseline + extras), rocprofv3 kernel stats of the C2 step / roofline probe /
# R50-FPN headline / C3 probe (one stats file each), the C2 step's PMC passes
# (tools/gpu_step_pmc.sh) and the roofline kernel's FETCH / WRITE passes.
# Stops at the first abnormal exit. Outputs in gpurun_out/<round>f/.
set -u
R=${ROUND:-r02}
D=gpurun_out/${R}f
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err; rc=$?
echo "== bench rc=$rc"; cut -c1-400 $D/bench.json; [ $rc -eq 0 ] || { tail -20 $D/bench.err; exit $rc; }
for probe in step roof head c3; do
  case $probe in
    step) args="--steps 5 --warmup 2 --no-cpu-baseline --no-extra" ;;
    roof) args="--roofline-only" ;;
    head) args="--headline-only" ;;
    c3) args="--c3-only" ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$probe -o $probe -- python3 bench.py $args > $D/prof_$probe.log 2>&1; rc=$?
  echo "== prof $probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D/roof_$c -o pmc -- python3 bench.py --roofline-only > $D/roof_$c.log 2>&1; rc=$?
  echo "== roof pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
TAG=${R}f/steppmc bash tools/gpu_step_pmc.sh
