"""Split graph engine B: what between its replays breaks it?
variants: interleave (A single-graph replays between B's), prep (eager
prepare_all(B) between B's steps), copy (B's arena state copied from an
identical clone of itself between steps), sync (the GPU test's full sync)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import layers as flayers  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from fpnmt.train import TrainEngine  # noqa: E402
from models.transformer import Transformer  # noqa: E402

fpnmt.set_precision("fp32")
variant = sys.argv[1]
capmode = sys.argv[2] if len(sys.argv) > 2 else "default"


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


def capture_merged(self, img, tok):
    s_img, s_tok = img.detach().clone(), tok.detach().clone()
    torch.cuda.synchronize()
    pool = torch.cuda.graph_pool_handle()
    g1, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, pool=pool):
        s_loss = self._fwd_bwd_split(s_img, s_tok).detach()
        self._bwd_fe()
    with torch.cuda.graph(g3, pool=pool):
        self._update()

    class _Nop:
        def replay(self):
            pass
    self.graphs = (g1, _Nop(), g3)
    self.static = (s_img, s_tok, s_loss)


def capture_manual(self, img, tok):
    """three graphs via capture_begin/capture_end on one side stream: no
    gc.collect / empty_cache between the captures"""
    s_img, s_tok = img.detach().clone(), tok.detach().clone()
    torch.cuda.synchronize()
    pool = torch.cuda.graph_pool_handle()
    st = torch.cuda.Stream()
    g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        g1.capture_begin(pool=pool)
        s_loss = self._fwd_bwd_split(s_img, s_tok).detach()
        g1.capture_end()
        g2.capture_begin(pool=pool)
        self._bwd_fe()
        g2.capture_end()
        g3.capture_begin(pool=pool)
        self._update()
        g3.capture_end()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    self.graphs = (g1, g2, g3)
    self.static = (s_img, s_tok, s_loss)


_orig = TrainEngine._capture


def _pick(fn):
    def cap(self, img, tok):
        return fn(self, img, tok) if self.split else _orig(self, img, tok)
    return cap


if capmode == "nopool":
    TrainEngine._capture = _pick(capture_nopool)
elif capmode == "manual":
    TrainEngine._capture = _pick(capture_manual)
elif capmode == "merged":
    TrainEngine._capture = _pick(capture_merged)


def build():
    torch.manual_seed(0)
    return Transformer(1, 512, 8, 2048, 196, 300, 0.0, max_seq_len=32,
                       init=Init(torch.Generator().manual_seed(12))).cuda()


g = torch.Generator().manual_seed(6)
img = (torch.rand(2, 224, 224, 3, generator=g) * 2 - 1).cuda()
tok = torch.randint(4, 300, (2, 32), generator=g)
tok[:, 0] = 2
tok = tok.to(torch.int32).cuda()
if variant == "rev":
    B = TrainEngine(build(), 1e-6, use_graph=True, split_backward=True)
    A = TrainEngine(build(), 1e-6, use_graph=True)
else:
    A = TrainEngine(build(), 1e-6, use_graph=variant != "inter-eager", split_backward=variant == "inter-split") \
        if variant in ("interleave", "sync", "inter-sync", "inter-single", "inter-split", "inter-eager") else None
    B = TrainEngine(build(), 1e-6, use_graph=True, split_backward=variant not in ("inter-single", "noise-single"))
la, lb = [], []
for i in range(6):
    if A is not None:
        la.append(float(A.step(img, tok)))
        if variant == "inter-sync":
            torch.cuda.synchronize()
    if variant == "sync" and i:
        with torch.no_grad():
            for nme in ("flat", "m", "v", "vhat", "step"):
                getattr(B.arena, nme).copy_(getattr(A.arena, nme))
    if variant in ("prep", "sync") and i:
        flayers.prepare_all(B.model)
    if variant in ("noise", "noise-single") and i:
        junk = [torch.full((1 << 26,), 1e30, device="cuda") for _ in range(16)]  # 4 GiB of eager allocations
        torch.cuda.synchronize()
        del junk
    if variant == "noise-empty" and i:
        junk = [torch.full((1 << 26,), 1e30, device="cuda") for _ in range(16)]
        torch.cuda.synchronize()
        del junk
        torch.cuda.empty_cache()
    if variant == "copy" and i:
        with torch.no_grad():
            for nme in ("flat", "m", "v", "vhat", "step"):
                t = getattr(B.arena, nme)
                t.copy_(t.clone())
    lb.append(float(B.step(img, tok)))
print(variant, "A", ["%.7f" % x for x in la], flush=True)
print(variant, "B", ["%.7f" % x for x in lb], flush=True)
