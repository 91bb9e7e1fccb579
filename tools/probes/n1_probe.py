"""Single-filter (k=1) conv kernels at the C2 shapes (regression head 256 -> 1,
3x3 'same', batch 32, pyramid levels of a 224 image), 20 launches of each
pass plus a torch clone of the inputs as a bandwidth yardstick; run under
rocprofv3 --kernel-trace --stats (and --pmc passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import _lib as L, ops  # noqa: E402
from fpnmt.layers import Conv2D  # noqa: E402

fpnmt.set_precision("bf16")
dt = torch.bfloat16
layer = Conv2D(256, 1, 3, padding="same").cuda()
shapes = [(32, 28, 28), (32, 14, 14), (32, 7, 7), (32, 3, 3), (32, 1, 1)]
xs = [torch.randn(*s, 256, device="cuda").clamp_min(0).to(dt) for s in shapes]
dzs = [torch.randn(*s, 1, device="cuda").to(dt) for s in shapes]
s = L.stream_ptr()
layer.kernel.grad = torch.zeros_like(layer.kernel)
for _ in range(20):
    ops._grouped_fwd(layer, xs)
for _ in range(20):
    ops._grouped_bwd_data(layer, xs, dzs, s, act_in=L.ACT_RELU)
for _ in range(20):
    ops._grouped_bwd_filter(layer, xs, dzs, s)
for _ in range(20):
    [x.clone() for x in xs[:1]]
torch.cuda.synchronize()
print("ok", sum(x.numel() * 2 for x in xs) / 1e6, "MB of input")
