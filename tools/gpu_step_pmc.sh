#!/bin/bash
# C2 training step: kernel trace + PMC passes (MFMA busy / wave states, HBM
# fetch, HBM write), one counter group per rocprofv3 run.
set -u
D=gpurun_out/${TAG:-steppmc}
mkdir -p $D
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o trace -- $CMD > $D/trace.log 2>&1; rc=$?
echo "== trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_MFMA,GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o pmc -- $CMD > $D/pmc$i.log 2>&1; rc=$?
  echo "== pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
