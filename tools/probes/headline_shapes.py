"""Per-GEMM-shape times of the ResNet-50-FPN forward (batch 64, 224^2, bf16):
run eagerly twice under rocprofv3 with FPNMT_GEMM_LOG, then
python tools/gemm_shapes.py <log> <trace> 60 --last-half"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from models.retinanet import FeatureExtractor  # noqa: E402

fpnmt.set_precision("bf16")
b = int(sys.argv[1]) if len(sys.argv) > 1 else 64
fe = FeatureExtractor(backbone="resnet50", init=Init(torch.Generator().manual_seed(3))).cuda()
x = (torch.rand(b, 224, 224, 3, device="cuda") * 2 - 1).to(torch.bfloat16)
with torch.no_grad():
    for _ in range(2):
        fe.retinanet_model.pyramid(x)
torch.cuda.synchronize()
print("ok")
