"""TrainEngine graph replay with eager allocation noise between steps vs an
eager engine: per step, which parameter segments / state diverge."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from fpnmt.train import TrainEngine  # noqa: E402
from models.transformer import Transformer  # noqa: E402

fpnmt.set_precision("fp32")


def build():
    torch.manual_seed(0)
    return Transformer(1, 512, 8, 2048, 196, 300, 0.0, max_seq_len=32,
                       init=Init(torch.Generator().manual_seed(12))).cuda()


g = torch.Generator().manual_seed(6)
img = (torch.rand(2, 224, 224, 3, generator=g) * 2 - 1).cuda()
tok = torch.randint(4, 300, (2, 32), generator=g)
tok[:, 0] = 2
tok = tok.to(torch.int32).cuda()
E = TrainEngine(build(), 1e-6, use_graph=False)
G = TrainEngine(build(), 1e-6, use_graph=True)
for i in range(4):
    le = float(E.step(img, tok))
    if i:
        junk = [torch.full((1 << 26,), 1e30, device="cuda") for _ in range(16)]
        torch.cuda.synchronize()
        del junk
    lg = float(G.step(img, tok))
    torch.cuda.synchronize()
    print(f"step {i}: loss E {le:.7f} G {lg:.7f}", flush=True)
    for nme in ("flat", "grad", "m", "v", "vhat", "step", "sumsq"):
        a, b = getattr(E.arena, nme), getattr(G.arena, nme)
        d = (a.double() - b.double()).abs()
        print(f"   {nme}: max|E-G| {float(d.max()):.3e} (|E| {float(a.double().abs().max()):.3e}) "
              f"nonfinite G {int((~torch.isfinite(b.double())).sum())}", flush=True)
    segs = []
    for n, o, p in zip(G.arena.names, G.arena.offsets, G.arena.params):
        ge, gg = E.arena.grad[o:o + p.numel()], G.arena.grad[o:o + p.numel()]
        segs.append((float((ge - gg).abs().max()) / max(float(ge.abs().max()), 1e-30), n))
    segs.sort(reverse=True)
    print("   worst grad segs:", [(f"{e:.2e}", n) for e, n in segs[:4]], flush=True)
