"""The training step of the reference (utils/pipeline.py:64-80) as a
hipGraph-replayed MI355X step.

step(img, caption_token):
  tar_inp = tok[:, :-1]; tar_real = tok[:, 1:]            (pipeline.py:66-67)
  mask = create_masks(tar_inp)                              (pipeline.py:69)
  logits = transformer(img, tar_inp, True, mask)            (pipeline.py:72)
  loss = masked CE mean over B*T                            (pipeline.py:50-57,75)
  grads -> [RCCL all-reduce] -> clip_by_norm per tensor -> AMSGrad   (pipeline.py:77-78)
  refresh the bf16/fp32 compute copies of the weights

The first call runs eagerly (warms the autograd engine and the allocator);
the second call captures the whole step into a hipGraph (torch.cuda.CUDAGraph
drives hipGraph on ROCm) and every later call only copies the new batch into
the static input buffers and replays. With world > 1 the step is two graphs
(forward+backward, optimizer) around the bucketed gradient all-reduce.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import dist as fdist
from . import layers as flayers
from . import ops
from .arena import ParamArena
from .layers import group_param_order


class TrainEngine:
    def __init__(self, transformer, schedule, beta1=0.9, beta2=0.98, eps=1e-9, clipnorm=1.0, use_graph=True,
                 group=None, bucket_bytes=fdist.DEFAULT_BUCKET_BYTES):
        from models.transformer import create_masks  # noqa: F401 (ensures import path)
        self.model = transformer
        self.schedule = schedule
        self.adam = dict(beta1=beta1, beta2=beta2, eps=eps, clipnorm=clipnorm)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_bytes = bucket_bytes
        dev = next(transformer.parameters()).device
        emb = transformer.decoder.embedding.embeddings
        named = [(n, p) for n, p in transformer.named_parameters() if p.requires_grad]
        named = group_param_order(transformer, named)  # grouped projections: contiguous blocks
        emb_name = [n for n, p in named if p is emb][0]
        self.arena = ParamArena(named, dev, sparse_names=[emb_name])
        transformer.decoder.embedding.sumsq_slot = self.arena.sumsq_slot(emb)
        self.emb_seg = self.arena.seg_of(emb)
        ops.runtime.seed_tensor = self.arena.step
        if self.world > 1:
            # identical initial weights on every rank
            dist.broadcast(self.arena.flat, 0, group=group)
        flayers.invalidate_weights()
        self.dtype = None
        self.use_graph = use_graph
        self.calls = 0
        self.graphs = None
        self.static = None

    # ------------------------------------------------------------ pieces
    def _fwd_bwd(self, img, tok):
        from models.transformer import create_masks
        self.arena.zero_grad()
        tar_inp = tok[:, :-1]
        tar_real = tok[:, 1:]
        mask = create_masks(tar_inp)
        logits, _ = self.model(img, tar_inp, True, mask)
        loss = ops.MaskedXentFn.apply(logits, tar_real)
        loss.backward()
        return loss

    def _exchange(self):
        if self.world > 1:
            fdist.allreduce_flat(self.arena.grad, self.bucket_bytes, self.group,
                                 extra=[self.arena.sumsq[self.emb_seg:self.emb_seg + 1]])

    def _update(self):
        self.arena.amsgrad_step(self.schedule, grad_scale=1.0 / self.world, **self.adam)
        flayers.prepare_all(self.model)

    def _eager(self, img, tok):
        loss = self._fwd_bwd(img, tok)
        self._exchange()
        self._update()
        return loss.detach()

    # -------------------------------------------------------------- step
    def step(self, img, tok):
        """One training step; returns the (device) loss of this batch."""
        self.calls += 1
        if not self.use_graph or self.calls == 1:
            import fpnmt
            flayers.prepare_all(self.model, fpnmt.compute_dtype())
            return self._eager(img, tok)
        if self.graphs is None:
            self._capture(img, tok)
        self.static[0].copy_(img)
        self.static[1].copy_(tok)
        g_fb, g_up = self.graphs
        g_fb.replay()
        if g_up is not None:
            self._exchange()
            g_up.replay()
        return self.static[2]

    def _capture(self, img, tok):
        s_img = img.detach().clone()
        s_tok = tok.detach().clone()
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        if self.world == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                loss = self._fwd_bwd(s_img, s_tok)
                self._update()
                s_loss = loss.detach()
            self.graphs = (g, None)
        else:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, pool=pool):
                s_loss = self._fwd_bwd(s_img, s_tok).detach()
            with torch.cuda.graph(g2, pool=pool):
                self._update()
            self.graphs = (g1, g2)
        self.static = (s_img, s_tok, s_loss)
