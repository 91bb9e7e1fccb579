#!/bin/bash
# Deep LDS rings (8 / 6 stages, cfg 7 / 8) for the short-row pipe GEMMs
# against the 4-stage default: same K order per block, so the loss must match
# bit for bit; two interleaved rounds.
set -u
D=gpurun_out/r3p
mkdir -p $D
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $D/$name.json 2>$D/$name.err || { tail -5 $D/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$D/$name.json'));print('[$name]', d['ms_per_step'], repr(d['loss']))"
}
for r in 1 2; do
  run def X=0
  run rc7 FPNMT_TUNE_ROW_CFG=7
  run rc8 FPNMT_TUNE_ROW_CFG=8
done
for c in 7 8; do
  FPNMT_TUNE_ROW_CFG=$c timeout -k 10 200 python bench.py --c5-only > $D/c5_$c.json 2>$D/c5_$c.err || { tail -5 $D/c5_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$D/c5_$c.json'));print('[c5 cfg $c]', d['c5_decode']['ms'])"
done
timeout -k 10 200 python bench.py --c5-only > $D/c5_def.json 2>$D/c5_def.err && python -c "import json;d=json.load(open('$D/c5_def.json'));print('[c5 def]', d['c5_decode']['ms'])"
