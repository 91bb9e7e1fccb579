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

With world > 1 (or split_backward=True) the step is a sequence of graphs:
  G1      forward + loss + the decoder's backward (stops at the encoder
          output, which enters the decoder as a leaf)
  G2      the encoder's backward from that leaf's gradient (stops at the
          feature extractor's five level outputs, which enter the encoder as
          leaves)
  S1..S5  the feature extractor's backward one stage at a time, in backward
          order: the shared heads, the FPN, then the backbone segments
          C4->C5, C3->C4, input->C3 (FeatureExtractor.staged: every stage
          reads detached leaves of the previous one's outputs)
  G3      clip + AMSGrad + compute-copy refresh
and the gradient arena is ordered decoder, encoder layers, then the feature
extractor stage by stage, so each range's RCCL all-reduce is issued as soon
as its graph ends (the decoder's and vocabulary projection's ~45 M of 105 M
parameters after G1, the encoder layers' after G2, the res5 segment's 15 M
after S3, ...) and runs on RCCL's stream while the next graphs compute; only
the last segment's (input->C3, ~1.4 M at ResNet-50) is exposed. G3 waits for
all of them (stream waits; the host never blocks).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import fpnmt
from . import _lib as L
from . import dist as fdist
from . import layers as flayers
from . import ops
from .arena import ParamArena
from .layers import group_param_order


class TrainEngine:
    def __init__(self, transformer, schedule, beta1=0.9, beta2=0.98, eps=1e-9, clipnorm=1.0, use_graph=True,
                 group=None, bucket_bytes=fdist.DEFAULT_BUCKET_BYTES, split_backward=None, bucket_dtype=None,
                 sync_bn=True):
        from models.transformer import create_masks  # noqa: F401 (ensures import path)
        self.model = transformer
        self.schedule = schedule
        self.adam = dict(beta1=beta1, beta2=beta2, eps=eps, clipnorm=clipnorm)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_bytes = bucket_bytes
        self.bucket_dtype = bucket_dtype
        dev = next(transformer.parameters()).device
        emb = transformer.decoder.embedding.embeddings
        named = [(n, p) for n, p in transformer.named_parameters() if p.requires_grad]
        named = group_param_order(transformer, named)  # grouped projections: contiguous blocks
        self.split = (self.world > 1) if split_backward is None else bool(split_backward)
        fe_prefix = "encoder.feature_extractor."
        # transformer parameters first (stable: DenseGroups live in the
        # transformer and stay contiguous), then the feature extractor's
        # stage by stage in backward order (one contiguous range per stage)
        stage_pref = transformer.encoder.feature_extractor.stage_prefixes()
        fe = [x for x in named if x[0].startswith(fe_prefix)]
        stage_of = {}
        for n, _ in fe:
            rel = n[len(fe_prefix):]
            stage_of[n] = next((i for i, ps in enumerate(stage_pref) if any(rel.startswith(q) for q in ps)),
                               len(stage_pref))  # unmatched: a last range of its own
        unmatched = [n for n, _ in fe if stage_of[n] == len(stage_pref)]
        if unmatched:
            # every feature-extractor parameter must sit in an exchanged stage
            # range, or DP ranks would drift apart silently
            raise ValueError(f"TrainEngine: feature-extractor parameters outside every stage: {unmatched[:4]}")
        fe.sort(key=lambda x: stage_of[x[0]])  # stable within a stage
        # the decoder side (decoder + vocabulary projection) first: its
        # gradients are complete when G1 ends; then the encoder layers (G2)
        dec_side = [x for x in named if x[0].startswith(("decoder.", "final_layer."))]
        enc_side = [x for x in named if not x[0].startswith(("decoder.", "final_layer.", fe_prefix))]
        named = dec_side + enc_side + fe
        emb_name = [n for n, p in named if p is emb][0]
        self.arena = ParamArena(named, dev, sparse_names=[emb_name])
        fe_idx = [i for i, n in enumerate(self.arena.names) if n.startswith(fe_prefix)]
        self.split_at = self.arena.offsets[fe_idx[0]] if fe_idx else self.arena.total
        offs = self.arena.offsets + [self.arena.total]
        dec_end = offs[len(dec_side)]
        # exchange ranges: [0] the decoder side, [1] the encoder layers, then
        # one per feature-extractor stage
        bounds = [(0, dec_end), (dec_end, self.split_at)]
        for st in range(len(stage_pref) + 1):
            idx = [i for i in fe_idx if stage_of[self.arena.names[i]] == st]
            bounds.append((offs[idx[0]], offs[idx[-1] + 1]) if idx else (0, 0))
        self.ranges = bounds
        transformer.decoder.embedding.sumsq_slot = self.arena.sumsq_slot(emb)
        self.emb_seg = self.arena.seg_of(emb)
        ops.runtime.seed_tensor = self.arena.step
        # opt-in low-precision buckets: one preallocated staging copy of the
        # gradient arena; each range is cast into it at the end of the graph
        # that produced it and the reduced sum is cast back at the start of the
        # update graph (both casts captured; zeros in the alignment gaps)
        self.low = None
        if bucket_dtype is not None and bucket_dtype != self.arena.grad.dtype and self.world > 1:
            self.low = torch.zeros(self.arena.total, dtype=bucket_dtype, device=dev)
        if self.world > 1:
            # identical initial weights on every rank
            fdist.broadcast_(self.arena.flat, 0, group)
            self.bn_group = None
            if sync_bn and fdist.has_batchnorm(transformer):
                # training-mode BatchNorm (MobileNetV2) over the global batch,
                # as the reference's single-device step computes it. Its
                # collectives run on a communicator of their own: with the
                # split step they sit inside the stage graphs while the
                # gradient ranges' async all-reduces are still in flight on
                # the engine's group, and RCCL does not order two streams'
                # collectives on one communicator
                self.bn_group = fdist.new_group_like(group)
                fdist.set_sync_batchnorm(transformer, self.bn_group)
        flayers.invalidate_weights()
        self.dtype = None
        self.use_graph = use_graph
        # the optimizer blocks of the transformer's segments (the arena's head,
        # up to the feature extractor's first segment): _early_update's range
        self.early_blocks = self.arena.block_of(self.split_at)
        self._upd_stream = None
        self._early_pending = False
        self.calls = 0
        self.graphs = None
        self.static = None

    # ------------------------------------------------------------ pieces
    def _one(self, loss):
        """The loss's seed gradient, kept across steps (loss.backward() would
        fill a fresh one with a kernel launch every step)."""
        one = getattr(self, "_one_t", None)
        if one is None or one.device != loss.device or one.dtype != loss.dtype:
            one = self._one_t = torch.ones((), dtype=loss.dtype, device=loss.device)
        return one

    def _zero_grad_fork(self):
        """arena.zero_grad(), or — zero_grad_overlap_grid > 0 on a GPU — the
        same fill as a trickle of that many workgroups on a side stream forked
        here, so it runs beside the forward pass (which writes no gradient);
        _zero_grad_join() makes the compute stream wait for it before the
        backward. Graph-capturable (wait_stream fork / join)."""
        grid = fpnmt.config.zero_grad_overlap_grid
        if grid <= 0 or not self.arena.grad.is_cuda:
            self.arena.zero_grad()
            return None
        if getattr(self, "_zero_stream", None) is None:
            self._zero_stream = torch.cuda.Stream()
        zs = self._zero_stream
        zs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(zs):
            self.arena.zero_grad(max_blocks=grid)
        return zs

    @staticmethod
    def _zero_grad_join(zs):
        if zs is not None:
            torch.cuda.current_stream().wait_stream(zs)

    def _fwd_bwd(self, img, tok):
        ops.runtime.reset_sites()  # dropout sites numbered from the step's start
        ops.reset_grad_sums()
        zs = self._zero_grad_fork()
        early = (self.world == 1 and fpnmt.config.early_update and self.arena.flat.is_cuda
                 and 0 < self.early_blocks < self.arena.nblocks)
        ops.runtime.on_transformer_grads = self._early_update if early else None
        try:
            tar_inp, tar_real, mask = ops.decoder_targets(tok)  # tok[:, :-1], tok[:, 1:], create_masks(tar_inp)
            logits, _ = self.model(img, tar_inp, True, mask)
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            self._zero_grad_join(zs)
            with L.deferred_reductions(fpnmt.config.defer_reductions), ops.side_wgrad():
                torch.autograd.backward([loss], [self._one(loss)])  # ordered reductions batched at the exit
        finally:
            ops.runtime.on_transformer_grads = None
        self._stage_low(None)
        return loss

    def _early_update(self):
        """Called from the backward (ops.transformer_grads_barrier) once the
        transformer's backward is complete: its queued reductions run now,
        then the transformer's segments (the arena's leading blocks) get their
        clip + AMSGrad + compute-copy refresh on a second stream, overlapping
        the feature extractor's backward on the compute stream. _update joins
        the streams and runs the feature extractor's part (the same kernels
        over the remaining blocks: bitwise the one-launch update)."""
        ops.join_side()
        L.defer_checkpoint()
        if self._upd_stream is None:
            self._upd_stream = torch.cuda.Stream()
        st = self._upd_stream
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            # a few persistent workgroups without LDS (no fused compute-copy
            # refresh: those copies are written in the tail) so the waves sit
            # beside the backward's GEMM blocks; one workgroup per block held
            # every CU slot until it drained (profiles/r05/early_update_r5h.txt)
            self.arena.amsgrad_step(self.schedule, grad_scale=1.0 / self.world, preps=None,
                                    blocks=(0, self.early_blocks), inc_step=False,
                                    max_grid=fpnmt.config.early_update_grid, **self.adam)
        self._early_pending = True

    def _fwd_bwd_split(self, img, tok):
        """G1: forward + loss + the decoder's backward down to the encoder
        output (a leaf of the decoder)."""
        ops.runtime.reset_sites()
        ops.reset_grad_sums()
        zs = self._zero_grad_fork()
        m = self.model
        tar_inp, tar_real, mask = ops.decoder_targets(tok)
        feats, stages = m.encoder.feature_extractor.staged(img, training=True)
        leaves = [f.detach().requires_grad_(f.requires_grad) for f in feats]
        enc = m.encoder.from_features(leaves, True, None)
        enc_leaf = enc.detach().requires_grad_(True)
        dec, _ = m.decoder(tar_inp, enc_leaf, True, mask, None)
        logits = m.final_layer(dec)
        loss = ops.MaskedXentFn.apply(logits, tar_real)
        self._zero_grad_join(zs)
        with L.deferred_reductions(fpnmt.config.defer_reductions), ops.side_wgrad():
            torch.autograd.backward([loss], [self._one(loss)])
        self._enc = (enc, enc_leaf)
        self._stages = [(outs, lvs if lvs is not None else leaves) for outs, lvs, _ in stages]
        self._stage_low(0)
        return loss

    def _bwd_encoder(self):
        """G2: the encoder layers' backward from the encoder output's gradient
        down to the feature extractor's level outputs."""
        enc, enc_leaf = self._enc
        if enc_leaf.grad is not None and enc.requires_grad:
            with L.deferred_reductions(fpnmt.config.defer_reductions), ops.side_wgrad():
                torch.autograd.backward([enc], [enc_leaf.grad])
        self._stage_low(1)

    def _bwd_stage(self, i):
        """S_i: one feature-extractor stage's backward from its outputs'
        leaf gradients (left by the stages after it in forward order)."""
        outs, leaves = self._stages[i]
        pairs = [(o, lf.grad) for o, lf in zip(outs, leaves)
                 if o.requires_grad and lf.grad is not None and o.numel() > 0]
        if pairs:
            with L.deferred_reductions(fpnmt.config.defer_reductions), ops.side_wgrad():
                torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
        self._stage_low(2 + i)

    def _stage_low(self, part):
        """Cast the exchange range `part` (None: the whole arena) of the
        gradients into the low-precision staging copy (bucket mode only)."""
        if self.low is None:
            return
        a, b = (0, self.arena.total) if part is None else self.ranges[part]
        if b > a:
            fdist.cast_into(self.low[a:b], self.arena.grad[a:b])

    def _exchange(self, part=None, wait=True):
        """SUM all-reduce of the gradient arena: part 0 = the decoder side's
        range (+ the embedding's sparse-norm accumulator), 1 = the encoder
        layers', part k >= 2 = the feature extractor's stage k-2 range, None =
        all."""
        if self.world <= 1:
            return []
        g = self.arena.grad
        rng = (0, self.arena.total) if part is None else self.ranges[part]
        extra = [self.arena.sumsq[self.emb_seg:self.emb_seg + 1]] if part in (None, 0) else None
        if rng[1] <= rng[0]:
            return []
        staging = self.low[rng[0]:rng[1]] if self.low is not None else None
        return fdist.allreduce_flat(g[rng[0]:rng[1]], self.bucket_bytes, self.group, extra=extra, wait=wait,
                                    bucket_dtype=self.bucket_dtype, staging=staging)

    def _update(self):
        ops.check_grad_sums()  # no consumer-summed input gradient left parked by the backward(s)
        if self.low is not None:
            fdist.cast_into(self.arena.grad, self.low)  # the reduced sums back into the fp32 arena
        fp = flayers.fused_prep(self.model, self.arena)
        blocks = None
        skip = fp.layers if fp else ()
        if self._early_pending:  # the transformer's part ran beside the backward: join, then the rest
            torch.cuda.current_stream().wait_stream(self._upd_stream)
            self._early_pending = False
            blocks = (self.early_blocks, self.arena.nblocks)
            # the early part wrote no compute copies: only the late part's
            # layers are refreshed by the optimizer kernel
            if fp:
                skip = {id(m) for m in fp._mods
                        if self.arena.offsets[self.arena.index[id(m.kernel)]] >= self.split_at}
        self.arena.amsgrad_step(self.schedule, grad_scale=1.0 / self.world, preps=fp.table if fp else None,
                                blocks=blocks, **self.adam)
        flayers.prepare_all(self.model, skip=skip)
        if fp:
            fp.mark_fresh()

    def _eager(self, img, tok):
        if self.split:
            loss = self._fwd_bwd_split(img, tok)
            works = self._exchange(0, wait=False)
            self._bwd_encoder()
            works += self._exchange(1, wait=False)
            for i in range(len(self._stages)):
                self._bwd_stage(i)
                works += self._exchange(2 + i, wait=False)
            for w in works:
                w.wait()
        else:
            loss = self._fwd_bwd(img, tok)
            self._exchange()
        self._update()
        return loss.detach()

    # ---------------------------------------------------------- timeline
    def enable_timeline(self, on=True):
        """Record HIP events around every graph replay and every range's
        exchange of the following replayed split steps (timeline() reads
        them): where each exchange completes against the stage graphs that
        run under it, and what is left exposed before the update graph."""
        self._tl = [] if on else None

    def timeline(self):
        """Per recorded step: the graphs' end times and the exchanges' issue /
        completion times, in ms from the step's start (synchronizes)."""
        torch.cuda.synchronize()
        return [t.read() for t in (self._tl or [])]

    _tl = None

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
        if img.shape != self.static[0].shape or tok.shape != self.static[1].shape:
            # a batch of another shape (the short last batch of an epoch: the
            # loaders keep tf.data's drop_remainder=False) cannot go through
            # the static buffers; tf.function retraces for it, this runs it
            # eagerly on the same arena / optimizer state
            import fpnmt
            flayers.prepare_all(self.model, fpnmt.compute_dtype())
            return self._eager(img, tok)
        self.static[0].copy_(img)
        self.static[1].copy_(tok)
        if self.split:
            g1, g2, *gs, g3 = self.graphs
            tl = _Timeline() if self._tl is not None else None
            g1.replay()
            works = self._exchange(0, wait=False)  # overlaps the next graphs on RCCL's stream
            if tl:
                tl.graph("G1")
                tl.exchange(0, works)
            g2.replay()
            w = self._exchange(1, wait=False)
            works += w
            if tl:
                tl.graph("G2")
                tl.exchange(1, w)
            for i, g in enumerate(gs):
                g.replay()
                w = self._exchange(2 + i, wait=False)
                works += w
                if tl:
                    tl.graph(f"S{i + 1}")
                    tl.exchange(2 + i, w)
            for w in works:
                w.wait()  # the compute stream waits; the host does not block
            if tl:
                tl.graph("waits")
            g3.replay()
            if tl:
                tl.graph("G3")
                self._tl.append(tl)
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
            n = len(self.model.encoder.feature_extractor.stage_prefixes())
            stage_fns = [(lambda i=i: self._bwd_stage(i)) for i in range(n)]
            self.graphs = capture_sequence([g1, self._bwd_encoder] + stage_fns + [self._update])
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


class _Timeline:
    """Events of one split step (TrainEngine.enable_timeline). A graph's
    event is recorded on the compute stream after its replay; an exchange's
    completion on a probe stream made to wait for the collective right after
    it is issued (the probe is otherwise idle, so its event fires when the
    collective ends) — or the gloo worker's own `done` event."""

    def __init__(self):
        self.t0 = self._rec()
        self.graphs, self.exch = [], []

    @staticmethod
    def _rec(stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream or torch.cuda.current_stream())
        return e

    def graph(self, name):
        self.graphs.append((name, self._rec()))

    def exchange(self, part, works):
        issued = self._rec()
        dones = []
        for w in works:
            ev = getattr(w, "done_event", None)
            if ev is None:
                probe = torch.cuda.Stream()
                with torch.cuda.stream(probe):
                    getattr(w, "work", w).wait()  # the collective itself (not a cast-back)
                    ev = self._rec(probe)
            dones.append(ev)  # a gloo job's `done` is recorded by its worker before Work.wait() returns
        self.exch.append((part, issued, dones))

    def read(self):
        f = lambda e: round(self.t0.elapsed_time(e), 4)
        out = {"graphs": [{"name": n, "end_ms": f(e)} for n, e in self.graphs], "exchanges": []}
        for part, issued, dones in self.exch:
            done = [f(e) for e in dones if e is not None]
            out["exchanges"].append({"range": part, "issued_ms": f(issued), "done_ms": max(done) if done else None})
        return out


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
