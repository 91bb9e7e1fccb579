#!/bin/bash
# rocprofv3 kernel stats + PMC passes of tools/probes/n1_probe.py
set -u
D=gpurun_out/n1p
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/tr -o tr -- python3 tools/probes/n1_probe.py > $D/tr.log 2>&1 || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum,TCC_MISS_sum" "SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o pmc -- python3 tools/probes/n1_probe.py > $D/pmc$i.log 2>&1 || exit $?
done
echo done
