#!/bin/bash
# Same-box A/B of dispatch tuning knobs (FPNMT_TUNE_*, csrc/gemm_dispatch.h)
# on the C2 step: two interleaved rounds per setting.
set -u
D=gpurun_out/r3n
mkdir -p $D
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $D/$name.json 2>$D/$name.err || { tail -5 $D/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$D/$name.json'));print('[$name]', d['ms_per_step'], d['loss'])"
}
for r in 1 2; do
  run def X=0
  run rs2 FPNMT_TUNE_ROW_SPLIT=2
  run wg256 FPNMT_TUNE_WG_TARGET=256
  run wg384 FPNMT_TUNE_WG_TARGET=384
  run rc2 FPNMT_TUNE_ROW_CFG=2
  run rc1 FPNMT_TUNE_ROW_CFG=1
done
