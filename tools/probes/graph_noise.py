"""Does a captured graph reference memory outside its pool? Capture a piece of
the model, replay it with eager allocation noise in between, compare with an
eager run. usage: graph_noise.py {fe,fwd,fwdbwd}"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from fpnmt.train import capture_sequence  # noqa: E402
from models.transformer import Transformer, create_masks  # noqa: E402

fpnmt.set_precision("fp32")
part = sys.argv[1]
torch.manual_seed(0)
m = Transformer(1, 512, 8, 2048, 196, 300, 0.0, max_seq_len=32, init=Init(torch.Generator().manual_seed(12))).cuda()
g = torch.Generator().manual_seed(6)
img = (torch.rand(2, 224, 224, 3, generator=g) * 2 - 1).cuda()
tok = torch.randint(4, 300, (2, 32), generator=g)
tok[:, 0] = 2
tok = tok.to(torch.int32).cuda()
tar = tok[:, :-1]
out = {}


def run():
    if part == "fe":
        with torch.no_grad():
            out["y"] = m.encoder.feature_extractor(img)[0]
    elif part == "fwd":
        with torch.no_grad():
            out["y"], _ = m(img, tar, True, create_masks(tar))
    else:  # forward + backward
        for p in m.parameters():
            p.grad = None
        lg, _ = m(img, tar, True, create_masks(tar))
        lg.float().sum().backward()
        out["y"] = m.final_layer.kernel.grad.clone()


run()
torch.cuda.synchronize()
ref = out["y"].clone()
gr = capture_sequence([run])[0]
for i in range(3):
    junk = [torch.full((1 << 26,), 1e30, device="cuda") for _ in range(16)]
    torch.cuda.synchronize()
    del junk
    gr.replay()
    torch.cuda.synchronize()
    print(part, i, "max |graph - eager| =", float((out["y"] - ref).abs().max()), "|ref|", float(ref.abs().max()),
          flush=True)
