import math, sys, os
sys.path[:0] = [os.path.join(os.getcwd(), "fpn-mt-image-captioning_amd"), os.getcwd()]
import torch
import fpnmt
from fpnmt import ops
from oracle import ref_cpu as R
DEV = "cuda"
fpnmt.set_precision("bf16")
for (B, H, Lq, Lk, D, mk) in [(4, 8, 31, 31, 64, "causal"), (2, 8, 13, 17, 64, None), (1, 1, 32, 32, 64, None)]:
    torch.manual_seed(0)
    dt = torch.bfloat16
    q = torch.randn(B, Lq, H * D, device=DEV).to(dt).requires_grad_(True)
    k = torch.randn(B, Lk, H * D, device=DEV).to(dt).requires_grad_(True)
    v = torch.randn(B, Lk, H * D, device=DEV).to(dt).requires_grad_(True)
    mask = None
    if mk == "causal":
        tok = torch.randint(1, 50, (B, Lq), device=DEV)
        mask = R.create_masks(tok.cpu()).to(DEV)
    out, w = ops.AttentionFn.apply(q, k, v, mask, H, 1.0 / math.sqrt(D))
    qr, kr, vr = [t.detach().float().requires_grad_(True) for t in (q, k, v)]
    sp = lambda x: x.reshape(B, -1, H, D).permute(0, 2, 1, 3)
    o_r, w_r = R.scaled_dot_product_attention(sp(qr), sp(kr), sp(vr), mask)
    o_r = o_r.permute(0, 2, 1, 3).reshape(B, Lq, H * D)
    g = torch.randn_like(o_r)
    out.backward(g.to(dt)); o_r.backward(g)
    torch.cuda.synchronize()
    print((B, H, Lq, Lk, mk), "out", float((out.float() - o_r).abs().max()), "w", float((w.float() - w_r).abs().max()))
    for nm, a, b in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        e = (a.float() - b).abs()
        idx = (e == e.max()).nonzero()[0].tolist()
        print(" ", nm, float(e.max()), "at", idx, "got", float(a.float()[tuple(idx)]), "ref", float(b[tuple(idx)]),
              "rows bad:", sorted(set((e.amax(-1) > 0.1).nonzero()[:, 1].tolist()))[:40])
