"""Time fpnmt_gemm on the row-major GEMM shapes of the C2 step (bf16) through
the C-ABI, HIP events on the launching stream, random operands.
python tools/probes/gemm_bench.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fpnmt import _lib as L  # noqa: E402

# (label, M, N, K, a_trans, b_trans, accumulate(2 = fp32 atomic C), batch)
SHAPES = [
    ("ffn2 fwd dec", 992, 512, 2048, 0, 0, 0, 1),
    ("ffn2 dgrad-ish", 992, 512, 1536, 0, 0, 0, 1),
    ("vocab dgrad", 992, 512, 10000, 0, 0, 0, 1),
    ("proj dec", 992, 512, 512, 0, 0, 0, 1),
    ("ffn1 dec", 992, 2048, 512, 0, 0, 0, 1),
    ("enc proj M32", 32, 512, 512, 0, 0, 0, 1),
    ("enc ffn2 M32", 32, 512, 2048, 0, 0, 0, 1),
    ("enc ffn1 M32", 32, 2048, 512, 0, 0, 0, 1),
    ("view kv", 288, 512, 6144, 0, 0, 0, 1),
    ("wgrad M32", 512, 512, 32, 1, 1, 2, 1),
    ("wgrad dec", 512, 512, 992, 1, 1, 2, 1),
    ("wgrad ffn", 2048, 512, 992, 1, 1, 2, 1),
    ("wgrad ffn1", 512, 2048, 992, 1, 1, 2, 1),
]


def run(label, m, n, k, ta, tb, acc, batch, iters):
    dt = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(m + n + k)
    A = (torch.rand(batch, k, m, generator=g) * 2 - 1).to(dt).cuda() if ta else \
        (torch.rand(batch, m, k, generator=g) * 2 - 1).to(dt).cuda()
    B = (torch.rand(batch, k, n, generator=g) * 2 - 1).to(dt).cuda() if tb else \
        (torch.rand(batch, n, k, generator=g) * 2 - 1).to(dt).cuda()
    c_f32 = 1 if acc == 2 else 0
    C = torch.zeros(batch, m, n, dtype=torch.float32 if c_f32 else dt, device="cuda")
    d = L.GemmDesc()
    d.m, d.n, d.k, d.batch, d.batch_inner, d.dtype = m, n, k, batch, 1, L.BF16
    d.a_trans, d.b_trans = ta, tb
    d.lda = m if ta else k
    d.ldb = n if tb else k
    d.ldc = d.ldr = n
    d.a_so, d.b_so, d.c_so = A[0].numel(), B[0].numel(), C[0].numel()
    d.alpha, d.act, d.act_alpha, d.accumulate, d.c_f32, d.split_k = 1.0, 0, 0.0, acc, c_f32, 0 if acc == 2 else 1
    args = (d, A.data_ptr(), B.data_ptr(), C.data_ptr(), None, None, None)
    s = L.stream_ptr()
    for _ in range(5):
        L.call("fpnmt_gemm", *args, s)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        L.call("fpnmt_gemm", *args, s)
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    ref = torch.einsum("bkm,bkn->bmn" if ta else "bmk,bkn->bmn", A.float(),
                       B.float() if tb else B.float().transpose(1, 2))
    if acc == 2:
        C.zero_()
        L.call("fpnmt_gemm", *args, s)
    else:
        L.call("fpnmt_gemm", *args, s)
    torch.cuda.synchronize()
    err = float((C.float() - ref).abs().max()) / max(1.0, float(ref.abs().max()))
    tf = 2.0 * m * n * k * batch / (us * 1e-6) / 1e12
    print(f"{label:16s} M={m:5d} N={n:5d} K={k:6d} b={batch} acc={acc}: {us:8.2f} us {tf:7.1f} TF  relerr {err:.1e}",
          flush=True)


if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for sh in SHAPES:
        if only is None or any(o in sh[0] for o in only):
            run(*sh, iters)
