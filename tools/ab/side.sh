set -u
mkdir -p gpurun_out/s1
for i in 1 2; do
for v in off dense all; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 --side-wgrad $v > gpurun_out/s1/b_${v}_$i.json 2>gpurun_out/s1/b_${v}_$i.err || exit 1
done
done
python -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/s1/*.json')):
    d=json.load(open(f)); print(f, d['ms_per_step'])"
