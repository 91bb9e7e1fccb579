"""Generates tests/golden/golden_small.json from the CPU oracle (oracle/ref_cpu.py)
with fixed seeds. The reference itself (TensorFlow) cannot run here, so these
vectors pin the oracle against regressions and feed the GPU parity tests;
they are NOT reference-generated (parity unpinned vs TF).
Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402


def r(t):
    return [round(float(v), 7) for v in t.reshape(-1)] if t.dim() == 0 else t.tolist()


def main():
    g = torch.Generator().manual_seed(20240)
    out = {"coattention": [], "sdpa": [], "fpn": [], "xent": []}
    for (n, h, w, c) in [(1, 7, 7, 3), (2, 3, 4, 5)]:
        s = torch.randn(n, h, w, 1, generator=g)
        hs = torch.randn(n, h, w, c, generator=g)
        out["coattention"].append({"score": s.tolist(), "hs": hs.tolist(), "out": R.coattention(s, hs).tolist()})
    for (b, hh, lq, lk, d, masked) in [(1, 2, 5, 5, 4, True), (2, 1, 1, 6, 8, False), (1, 1, 3, 0, 4, False)]:
        q = torch.randn(b, hh, lq, d, generator=g)
        k = torch.randn(b, hh, lk, d, generator=g)
        v = torch.randn(b, hh, lk, d, generator=g)
        mask = None
        if masked:
            tok = torch.tensor([[2, 9, 4, 3, 0]])
            mask = R.create_masks(tok)
        o, wts = R.scaled_dot_product_attention(q, k, v, mask)
        out["sdpa"].append({"q": q.tolist(), "k": k.tolist(), "v": v.tolist(), "kshape": list(k.shape),
                            "mask": None if mask is None else mask.tolist(), "out": o.tolist(), "w": wts.tolist()})
    for (h5, h4, h3) in [(2, 4, 8), (4, 7, 13)]:
        l5 = torch.randn(1, h5, h5, 2, generator=g)
        l4 = torch.randn(1, h4, h4, 2, generator=g)
        l3 = torch.randn(1, h3, h3, 2, generator=g)
        p4 = R.upsample_like(l5, l4) + l4
        p3 = R.upsample_like(p4, l3) + l3
        out["fpn"].append({"l5": l5.tolist(), "l4": l4.tolist(), "l3": l3.tolist(), "p3": p3.tolist()})
    lg = torch.randn(2, 5, 11, generator=g) * 2
    lab = torch.tensor([[3, 4, 1, 0, 0], [2, 10, 7, 7, 3]])
    out["xent"].append({"logits": lg.tolist(), "labels": lab.tolist(), "loss": float(R.masked_loss(lab, lg))})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_small.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
