"""Warm vs cold timing of the M=32 encoder GEMMs (small kernel): 200 launches
of x(32x512) @ W^T(512x512) with the same W (warm) and with 64 different Ws
(cold-ish), under rocprofv3 --kernel-trace --stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt.layers import Dense  # noqa: E402

fpnmt.set_precision("bf16")
torch.manual_seed(0)
x = torch.randn(32, 512, device="cuda").to(torch.bfloat16)
layers = [Dense(512, 512).cuda() for _ in range(64)]
with torch.no_grad():
    for _ in range(3):
        for L in layers:
            L(x)
    torch.cuda.synchronize()
    for _ in range(200):
        layers[0](x)
    torch.cuda.synchronize()
    for r in range(3):
        for L in layers:
            L(x)
    torch.cuda.synchronize()
print("ok")
