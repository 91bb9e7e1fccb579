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
the static input buffers and replays.

With world > 1 (or split_backward=True) the step is three graphs:
  G1  forward + loss + the transformer's backward (stops at the feature
      extractor's five level outputs, which enter the encoder as leaves)
  G2  the feature extractor's backward (backbone, FPN, shared heads)
  G3  clip + AMSGrad + compute-copy refresh
and the gradient arena is ordered transformer-first, so the RCCL all-reduce
of the transformer's gradients (~73 M of the 105 M parameters at C2) is
issued right after G1 and runs on RCCL's stream while G2 computes; the
feature extractor's gradients follow G2; G3 waits for both.
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
                 group=None, bucket_bytes=fdist.DEFAULT_BUCKET_BYTES, split_backward=None):
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
        self.split = (self.world > 1) if split_backward is None else bool(split_backward)
        fe_prefix = "encoder.feature_extractor."
        # transformer parameters first, the feature extractor's last (stable:
        # DenseGroups live in the transformer and stay contiguous)
        named = [x for x in named if not x[0].startswith(fe_prefix)] + [x for x in named if x[0].startswith(fe_prefix)]
        emb_name = [n for n, p in named if p is emb][0]
        self.arena = ParamArena(named, dev, sparse_names=[emb_name])
        fe_idx = [i for i, n in enumerate(self.arena.names) if n.startswith(fe_prefix)]
        self.split_at = self.arena.offsets[fe_idx[0]] if fe_idx else self.arena.total
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

    def _fwd_bwd_split(self, img, tok):
        """G1: forward + loss + backward down to the feature-extractor outputs."""
        from models.transformer import create_masks
        self.arena.zero_grad()
        m = self.model
        tar_inp = tok[:, :-1]
        tar_real = tok[:, 1:]
        mask = create_masks(tar_inp)
        feats = m.encoder.feature_extractor(img)
        leaves = [f.detach().requires_grad_(f.requires_grad) for f in feats]
        enc = m.encoder.from_features(leaves, True, None)
        dec, _ = m.decoder(tar_inp, enc, True, mask, None)
        logits = m.final_layer(dec)
        loss = ops.MaskedXentFn.apply(logits, tar_real)
        loss.backward()
        self._fe_pairs = [(f, lf) for f, lf in zip(feats, leaves) if f.requires_grad]
        return loss

    def _bwd_fe(self):
        """G2: the feature extractor's backward from the level-output grads."""
        pairs = [(f, lf.grad) for f, lf in self._fe_pairs if lf.grad is not None and f.numel() > 0]
        if pairs:
            torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])

    def _exchange(self, part=None, wait=True):
        """SUM all-reduce of the gradient arena: part 0 = the transformer's
        range (+ the embedding's sparse-norm accumulator), part 1 = the
        feature extractor's range, None = all."""
        if self.world <= 1:
            return []
        g = self.arena.grad
        rng = {None: (0, self.arena.total), 0: (0, self.split_at), 1: (self.split_at, self.arena.total)}[part]
        extra = [self.arena.sumsq[self.emb_seg:self.emb_seg + 1]] if part in (None, 0) else None
        if rng[1] <= rng[0]:
            return []
        return fdist.allreduce_flat(g[rng[0]:rng[1]], self.bucket_bytes, self.group, extra=extra, wait=wait)

    def _update(self):
        self.arena.amsgrad_step(self.schedule, grad_scale=1.0 / self.world, **self.adam)
        flayers.prepare_all(self.model)

    def _eager(self, img, tok):
        if self.split:
            loss = self._fwd_bwd_split(img, tok)
            works = self._exchange(0, wait=False)
            self._bwd_fe()
            works += self._exchange(1, wait=False)
            for w in works:
                w.wait()
        else:
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
        if self.split:
            g1, g2, g3 = self.graphs
            g1.replay()
            works = self._exchange(0, wait=False)  # overlaps G2 on RCCL's stream
            g2.replay()
            works += self._exchange(1, wait=False)
            for w in works:
                w.wait()  # the compute stream waits; the host does not block
            g3.replay()
            return self.static[2]
        g_fb, g_up = self.graphs
        g_fb.replay()
        if g_up is not None:
            self._exchange()
            g_up.replay()
        return self.static[2]

    def _capture(self, img, tok):
        s_img = img.detach().clone()
        s_tok = tok.detach().clone()
        out = {}
        if self.split:
            def g1():
                out["loss"] = self._fwd_bwd_split(s_img, s_tok).detach()
            self.graphs = capture_sequence([g1, self._bwd_fe, self._update])
        elif self.world == 1:
            def g():
                out["loss"] = self._fwd_bwd(s_img, s_tok).detach()
                self._update()
            self.graphs = (capture_sequence([g])[0], None)
        else:
            def g1():
                out["loss"] = self._fwd_bwd(s_img, s_tok).detach()
            self.graphs = tuple(capture_sequence([g1, self._update]))
        self.static = (s_img, s_tok, out["loss"])


def capture_sequence(fns, pool=None):
    """Capture fns[i] into graph i, back to back on one side stream, sharing
    one private memory pool; replay them in the same order.

    torch.cuda.graph() runs gc.collect() + empty_cache() at every capture
    entry: between two captures of one step that can free (and hand out
    again) pool memory an earlier graph still writes, e.g. tensors kept
    alive only through reference cycles of the earlier capture's autograd
    graph — measured as a silently diverging split-backward step once other
    graphs replayed in between. Here the collection runs once, before the
    first capture."""
    import gc
    gc.collect()
    torch.cuda.synchronize()
    pool = pool if pool is not None else torch.cuda.graph_pool_handle()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    graphs = []
    with torch.cuda.stream(st):
        for fn in fns:
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=pool)
            try:
                fn()
            finally:
                g.capture_end()
            graphs.append(g)
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    return graphs
