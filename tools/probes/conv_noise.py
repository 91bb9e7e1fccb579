"""Captured conv forward+backward replayed after eager allocation noise vs an
eager run, per conv kind (which one reads memory outside its graph pool?)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import ops  # noqa: E402
from fpnmt.layers import Conv2D  # noqa: E402
from fpnmt.train import capture_sequence  # noqa: E402

fpnmt.set_precision("fp32")
CASES = {
    "1x1s2": dict(cin=256, cout=128, k=1, s=2, pad="valid", act="relu", bn=True, h=56),
    "1x1s2-lin": dict(cin=256, cout=512, k=1, s=2, pad="valid", act=None, bn=True, h=56),
    "1x1s1-res": dict(cin=64, cout=256, k=1, s=1, pad="valid", act="relu", bn=True, h=56, res=True),
    "3x3": dict(cin=64, cout=64, k=3, s=1, pad=(1, 1, 1, 1), act="relu", bn=True, h=56),
}
for name, c in CASES.items():
    torch.manual_seed(0)
    layer = Conv2D(c["cin"], c["cout"], c["k"], strides=c["s"], padding=c["pad"], activation=c["act"],
                   use_bias=not c["bn"], frozen_bn=c["bn"]).cuda()
    x = torch.randn(2, c["h"], c["h"], c["cin"], device="cuda").requires_grad_(True)
    out = {}

    def run():
        layer.kernel.grad = None
        x.grad = None
        res = None
        if c.get("res"):
            res = torch.ones(2, c["h"], c["h"], c["cout"], device="cuda")
        y = layer(x, residual=res) if res is not None else layer(x)
        if c.get("pool"):
            y = ops.max_pool2d_same(y, 3, 2)
        (y * y).sum().backward()
        out["dx"] = x.grad.clone()
        out["dw"] = layer.kernel.grad.clone()

    run()
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in out.items()}
    gr = capture_sequence([run])[0]
    errs = []
    for i in range(3):
        junk = [torch.full((1 << 26,), 1e30, device="cuda") for _ in range(8)]
        torch.cuda.synchronize()
        del junk
        gr.replay()
        torch.cuda.synchronize()
        errs.append(max(float((out[k] - ref[k]).abs().max()) / max(1.0, float(ref[k].abs().max())) for k in ref))
    print(name, ["%.2e" % e for e in errs], flush=True)
