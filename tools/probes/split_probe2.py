"""Split-backward graphs: which capture structure breaks? Variants of
TrainEngine._capture for the split step, fixed seeds, losses over 6 steps."""
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
variant = sys.argv[1]


def build():
    torch.manual_seed(0)
    return Transformer(1, 512, 8, 2048, 196, 300, 0.0, max_seq_len=32,
                       init=Init(torch.Generator().manual_seed(12))).cuda()


def capture_merged12(self, img, tok):
    s_img, s_tok = img.detach().clone(), tok.detach().clone()
    torch.cuda.synchronize()
    pool = torch.cuda.graph_pool_handle()
    g1, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, pool=pool):
        s_loss = self._fwd_bwd_split(s_img, s_tok).detach()
        self._bwd_fe()
    with torch.cuda.graph(g3, pool=pool):
        self._update()
    self.graphs = (g1, torch.cuda.CUDAGraph(), g3)
    self.static = (s_img, s_tok, s_loss)


def capture_nopool(self, img, tok):
    s_img, s_tok = img.detach().clone(), tok.detach().clone()
    torch.cuda.synchronize()
    g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        s_loss = self._fwd_bwd_split(s_img, s_tok).detach()
    with torch.cuda.graph(g2):
        self._bwd_fe()
    with torch.cuda.graph(g3):
        self._update()
    self.graphs = (g1, g2, g3)
    self.static = (s_img, s_tok, s_loss)


g = torch.Generator().manual_seed(6)
img = (torch.rand(2, 224, 224, 3, generator=g) * 2 - 1).cuda()
tok = torch.randint(4, 300, (2, 32), generator=g)
tok[:, 0] = 2
tok = tok.to(torch.int32).cuda()
if variant == "merged12":
    TrainEngine._capture = capture_merged12
    TrainEngine._empty_g2 = True
elif variant == "nopool":
    TrainEngine._capture = capture_nopool
pre = None
if variant.startswith("after-"):  # another engine first (kept alive), then the split graph engine
    pre_kind = variant[len("after-"):]
    pm = build()
    pre = TrainEngine(pm, 1e-6, use_graph=pre_kind != "eager", split_backward=pre_kind == "split")
    print("pre", ["%.7f" % float(pre.step(img, tok)) for _ in range(3)], flush=True)
    variant = "split"
kw = dict(use_graph=True) if variant == "single" else dict(use_graph=variant != "eager", split_backward=True)
m = build()
e = TrainEngine(m, 1e-6, **kw)
losses = [float(e.step(img, tok)) for _ in range(6)]
print(variant, ["%.7f" % x for x in losses], flush=True)
