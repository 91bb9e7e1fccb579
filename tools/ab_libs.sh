#!/bin/bash
# Same-box A/B of library builds: tools/abj/lib_<name>.so copied over the
# in-tree libfpnmt.so of the GPU box's tree copy (bench.py measures only the
# in-tree build), C2 step, the variants alternating for R rounds; the in-tree
# build is restored at the end.  usage: ab_libs.sh <rounds> <name>...
LIB=fpn-mt-image-captioning_amd/fpnmt/libfpnmt.so
D=gpurun_out/abl
mkdir -p $D
cp $LIB $D/lib_intree.so
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    cp tools/abj/lib_$v.so $LIB
    timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extra > $D/run.json 2>$D/run.err || { tail -5 $D/run.err; cp $D/lib_intree.so $LIB; exit 1; }
    python -c "import json;d=json.load(open('$D/run.json'));print('[$v]', d['ms_per_step'], d['roofline']['achieved'], d['loss'])" | tee -a $D/ab.txt
  done
done
cp $D/lib_intree.so $LIB
