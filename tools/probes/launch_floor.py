"""Per-kernel cost floor inside a hipGraph on this box: N back-to-back tiny
kernels (fpnmt_add of 2048 bf16, an M=32 512x512 Dense, torch fill_) captured
in one graph and replayed; prints us per kernel (wall / N)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import _lib as L  # noqa: E402
from fpnmt.layers import Dense  # noqa: E402

fpnmt.set_precision("bf16")
N = 500
a = torch.randn(2048, device="cuda").to(torch.bfloat16)
b = torch.randn(2048, device="cuda").to(torch.bfloat16)
o = torch.empty_like(a)
x = torch.randn(32, 512, device="cuda").to(torch.bfloat16)
dense = Dense(512, 512).cuda()
f = torch.empty(2048, device="cuda")


def add():
    for _ in range(N):
        L.call("fpnmt_add", L.BF16, 2048, L.ptr(a), L.ptr(b), L.ptr(o), L.stream_ptr())


def small():
    with torch.no_grad():
        for _ in range(N):
            dense(x)


def fill():
    for _ in range(N):
        f.fill_(1.0)


s = torch.cuda.Stream()
for name, fn in (("fpnmt_add 2048", add), ("dense M=32 512x512", small), ("torch fill_ 2048", fill)):
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:24s} graph: {e0.elapsed_time(e1) * 1e3 / (5 * N):6.2f} us/kernel", flush=True)
