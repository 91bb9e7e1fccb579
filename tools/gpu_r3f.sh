#!/bin/bash
# Round-3 session F: the input-pipeline and C2-size gradient tests, the input
# probe, then the round's evidence (tools/gpu_profile_round.sh -> gpurun_out/r03f).
set -u
D=gpurun_out/r3f
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_input_pipeline.py tests/test_gpu_model.py -m gpu -x -q --timeout 500 --timeout-method thread \
  -k "resize or batch_loader or coco_images or c2_model" > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --input-only > $D/input.json 2>$D/input.err; rc=$?
echo "== input rc=$rc"; cut -c1-400 $D/input.json; [ $rc -eq 0 ] || exit $rc
ROUND=r03 bash tools/gpu_profile_round.sh
