"""Known-good reference on the same box: torch.matmul (hipBLASLt) on the
implicit-GEMM shapes of tools/conv_bench.py (M x K @ K x N, bf16), i.e. what a
vendor GEMM reaches when im2col is free."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import torch
from conv_bench import SHAPES
for name, (n, h, w, c, k, r, st, res, act) in SHAPES.items():
    ho, wo = -(-h // st), -(-w // st)
    M, K, N = n * ho * wo, r * r * c, k
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    fl = 2.0 * M * N * K
    print(f"{name:10s} M={M:7d} N={N:5d} K={K:5d}  {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF/s ({fl/ms/1e9/25:5.1f}%)", flush=True)
