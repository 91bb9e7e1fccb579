#!/bin/bash
# Round-3 session E: full GPU suite (the C2 fp32-gradient test deselected;
# its diagnosis runs below), the input-pipeline probe (resize kernel), and
# the gradient-boundary / FE-backward precision probes.
set -u
D=gpurun_out/r3e
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_model.py::test_train_step_parity_c2_model_fp32 > $D/tests.txt 2>&1; rc=$?
echo "== tests rc=$rc"; tail -3 $D/tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --input-only > $D/input.json 2>$D/input.err; rc=$?
echo "== input rc=$rc"; cut -c1-700 $D/input.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tests/probe_grad_boundary.py 6 10000 224 > $D/grad_boundary.txt 2>&1; rc=$?
echo "== grad boundary rc=$rc"; grep -v Warning $D/grad_boundary.txt | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probes/fe_bwd.py 6 10000 > $D/fe_bwd.txt 2>&1; rc=$?
echo "== fe_bwd rc=$rc"; tail -14 $D/fe_bwd.txt
exit $rc
