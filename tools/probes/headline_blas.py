"""Known-good reference on the same box for the R50-FPN forward's GEMM shapes
at batch 64 (and the C2 dominant conv): torch.matmul (hipBLASLt) on
(M x K) @ (K x N) bf16 — what a vendor GEMM reaches when the im2col gather
and the epilogue are free. Prints us and TFLOP/s per shape next to the
HBM-floor time of the GEMM's own operands.
  python tools/probes/headline_blas.py"""
import torch

SHAPES = [  # name, M, N, K
    ("r2_a 1x1 256->64", 200704, 64, 256), ("r2_b 3x3 64->64", 200704, 64, 576),
    ("r2_c 1x1 64->256", 200704, 256, 64), ("r3_a 1x1 512->128", 50176, 128, 512),
    ("r3_b 3x3 128->128", 50176, 128, 1152), ("r3_c 1x1 128->512", 50176, 512, 128),
    ("r3_sc 1x1 256->512", 50176, 512, 256), ("r4_a 1x1 1024->256", 12544, 256, 1024),
    ("r4_b 3x3 256->256", 12544, 256, 2304), ("r4_c 1x1 256->1024", 12544, 1024, 256),
    ("r4_sc 1x1 512->1024", 12544, 1024, 512), ("r5_a 1x1 2048->512", 3136, 512, 2048),
    ("r5_b 3x3 512->512", 3136, 512, 4608), ("r5_c 1x1 512->2048", 3136, 2048, 512),
    ("r5_sc 1x1 1024->2048", 3136, 2048, 1024), ("lat3 1x1 512->256", 50176, 256, 512),
    ("P3 3x3 256->256 b64", 50176, 256, 2304), ("P4 3x3 256->256 b64", 12544, 256, 2304),
    ("C2 P3 3x3 256->256 b32", 25088, 256, 2304),
]


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, m, n, k in SHAPES:
        a = (torch.rand(m, k, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(k, n, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
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
        fl = 2.0 * m * n * k
        floor_us = 2.0 * (m * k + k * n + m * n) / 6.3e12 * 1e6
        print(f"{name:26s} M={m:7d} N={n:5d} K={k:5d}  {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s "
              f"({fl / ms / 1e9 / 25:5.1f}% of 2.5 PF)  hbm-floor {floor_us:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
