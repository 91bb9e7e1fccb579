"""Repeat the FE level forward/backward (tests/test_gpu_parts.py setup) and
report parameters whose gradients vary between runs by more than fp32
summation-order noise (hunting an intermittent wrong result)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from test_gpu_parts import _setup  # noqa: E402

fe, sd = _setup()
g = torch.Generator().manual_seed(2)
f = torch.randn(2, 28, 28, 256, generator=g)
w = None
runs = []
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    fe.zero_grad(set_to_none=True)
    fd = f.cuda().requires_grad_(True)
    out = fe.level(fd)
    if w is None:
        w = torch.randn(out.shape, generator=g).cuda()
    (out * w).sum().backward()
    torch.cuda.synchronize()
    gr = {n: p.grad.detach().clone() for n, p in fe.named_parameters() if p.grad is not None}
    gr["<input>"] = fd.grad.detach().clone()
    gr["<out>"] = out.detach().float().clone()
    runs.append(gr)
base = runs[0]
bad = 0
for i, r in enumerate(runs[1:], 1):
    for n, t in r.items():
        mx = float(base[n].abs().max())
        e = float((t - base[n]).abs().max())
        if e > 1e-4 * mx + 1e-6:
            bad += 1
            print(f"run {i}: {n} differs: {e:.3e} (max {mx:.3e})")
print("runs", len(runs), "bad", bad)
