#!/bin/bash
# conv_bench timing + rocprofv3 PMC passes (one counter group per run).
set -u
D=gpurun_out/${TAG:-convpmc}
mkdir -p $D
export TMPDIR=/tmp
ONLY=${ONLY:-}
timeout -k 10 200 python tools/conv_bench.py --check ${ONLY:+--only $ONLY} > $D/bench.txt 2>&1; rc=$?
echo "== bench rc=$rc"; cat $D/bench.txt; [ $rc -eq 0 ] || exit $rc
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_MFMA,SQ_INSTS_VALU,GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_SALU,SQ_ACTIVE_INST_VALU,SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $D/pmc$i -o pmc -- python3 tools/conv_bench.py --iters 3 ${ONLY:+--only $ONLY} > $D/pmc$i.log 2>&1; rc=$?
  echo "== pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
