"""Keras-equivalent layers over the fpnmt kernels (NHWC, Keras weight layouts).

These are the building blocks the reference gets from tf.keras.layers
(Conv2D, Dense, LayerNormalization, Embedding, keras-resnet's frozen
BatchNormalization). Weight masters are fp32 in Keras layouts (conv HWIO,
dense (in, out)) so checkpoints and the CPU oracle share them verbatim;
kernel-layout compute copies (bf16 or fp32) are produced by
fpnmt_weight_prep and refreshed after every optimizer step.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib as L
from . import ops
from ._lib import call, ptr, stream_ptr, dtype_code

_GEN = [0]


def invalidate_weights():
    """Mark every compute copy stale (call after editing parameters by hand)."""
    _GEN[0] += 1


# ------------------------------------------------------------ initializers
class Init:
    """Keras initializer semantics, drawn from a torch.Generator."""

    def __init__(self, gen=None):
        self.gen = gen

    def _g(self):
        return self.gen

    def glorot_uniform(self, shape, fan_in, fan_out):
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        return (torch.rand(shape, generator=self._g()) * 2 - 1) * lim

    def he_normal(self, shape, fan_in):
        # TF2 VarianceScaling(2, fan_in, truncated_normal)
        std = math.sqrt(2.0 / fan_in) / 0.87962566103423978
        t = torch.randn(shape, generator=self._g())
        bad = t.abs() > 2
        while bad.any():
            t[bad] = torch.randn(int(bad.sum()), generator=self._g())
            bad = t.abs() > 2
        return t * std

    def normal(self, shape, std):
        return torch.randn(shape, generator=self._g()) * std

    def uniform(self, shape, lim):
        return (torch.rand(shape, generator=self._g()) * 2 - 1) * lim


DEFAULT_INIT = Init(None)


def _make_kernel(init, kind, shape, fan_in, fan_out, std=0.01):
    if kind == "he_normal":
        return init.he_normal(shape, fan_in)
    if kind == "normal":
        return init.normal(shape, std)
    return init.glorot_uniform(shape, fan_in, fan_out)


class _WeightLayer(nn.Module):
    """Shared compute-copy management for Conv2D / Dense."""

    def _init_copies(self):
        self._copies = {}
        self._gen = -1

    def _rsck(self):
        raise NotImplementedError

    def ensure_copies(self, dt):
        grp = self.__dict__.get("_group")
        if grp is not None and dt not in self._copies:
            grp[0].ensure(dt)  # forward copies are slices of the group's stacked operand
        if dt not in self._copies:
            r, s, c, k = self._rsck()
            dev = self.kernel.device
            self._copies[dt] = (torch.empty(r * s * c * k, dtype=dt, device=dev),
                                torch.empty(r * s * c * k, dtype=dt, device=dev))
        return self._copies[dt]

    def prepare(self, dtype=None):
        """(Re)build the kernel-layout compute copies for every dtype in use."""
        dts = [dtype] if dtype is not None else (list(self._copies) or [])
        r, s, c, k = self._rsck()
        for dt in dts:
            wf, wb = self.ensure_copies(dt)
            call("fpnmt_weight_prep", ptr(self.kernel), r, s, c, k, ptr(self.bn_scale), dtype_code(dt),
                 ptr(wf), ptr(wb), self.flip_ld(), stream_ptr())
        self._gen = _GEN[0]

    def flip_ld(self):
        """Row stride (elements) of the flipped copy: r*s*k, or the group's
        n*out when the flip is a column block of a DenseGroup's stack."""
        grp = self.__dict__.get("_group")
        if grp is not None:
            return grp[0].n * grp[0].fout
        r, s, c, k = self._rsck()
        return r * s * k

    def compute_weights(self, dtype):
        if dtype not in self._copies or self._gen != _GEN[0]:
            self.prepare(dtype)
            if len(self._copies) > 1:
                self.prepare()
        return self._copies[dtype]


class Conv2D(_WeightLayer):
    """tf.keras.layers.Conv2D (NHWC, HWIO kernel). padding: 'same' | 'valid' |
    (pt, pb, pl, pr). Optional frozen BatchNormalization folded in (keras-resnet
    freeze_bn=True: inference-mode BN, non-trainable): y = act(bn(conv(x)) [+ res])."""

    def __init__(self, in_channels, filters, kernel_size, strides=1, padding="same", activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", std=0.01, frozen_bn=False,
                 bn_epsilon=1e-5, act_alpha=0.2, init=None, name=None):
        super().__init__()
        ks = kernel_size if isinstance(kernel_size, (tuple, list)) else (kernel_size, kernel_size)
        st = strides if isinstance(strides, (tuple, list)) else (strides, strides)
        self.kh, self.kw = ks
        self.sh, self.sw = st
        self.in_channels, self.filters = in_channels, filters
        self.padding = padding
        self.activation = activation
        self.act_alpha = act_alpha
        self.lname = name
        init = init or DEFAULT_INIT
        fan_in = self.kh * self.kw * in_channels
        fan_out = self.kh * self.kw * filters
        self.kernel = nn.Parameter(_make_kernel(init, kernel_initializer, (self.kh, self.kw, in_channels, filters),
                                                fan_in, fan_out, std))
        self.bias = nn.Parameter(torch.zeros(filters)) if use_bias else None
        if frozen_bn:
            # gamma=1, beta=0, moving mean 0, moving var 1 (fresh keras-resnet BN)
            self.register_buffer("bn_gamma", torch.ones(filters))
            self.register_buffer("bn_beta", torch.zeros(filters))
            self.register_buffer("bn_mean", torch.zeros(filters))
            self.register_buffer("bn_var", torch.ones(filters))
            self.bn_epsilon = bn_epsilon
            self.register_buffer("bn_scale", torch.empty(filters))
            self.register_buffer("bn_shift", torch.empty(filters))
            self.refresh_bn()
        else:
            self.bn_scale = None
            self.bn_shift = None
        self._init_copies()

    def refresh_bn(self):
        with torch.no_grad():
            sc = self.bn_gamma / torch.sqrt(self.bn_var + self.bn_epsilon)
            self.bn_scale.copy_(sc)
            self.bn_shift.copy_(self.bn_beta - self.bn_mean * sc)

    def _rsck(self):
        return self.kh, self.kw, self.in_channels, self.filters

    def pads_for(self, h, w):
        if isinstance(self.padding, (tuple, list)):
            return tuple(self.padding)
        if self.padding == "valid":
            return 0, 0, 0, 0
        # TF 'same': total = max((ceil(h/s)-1)*s + k - h, 0), before = total//2
        ho, wo = -(-h // self.sh), -(-w // self.sw)
        th = max((ho - 1) * self.sh + self.kh - h, 0)
        tw = max((wo - 1) * self.sw + self.kw - w, 0)
        return th // 2, th - th // 2, tw // 2, tw - tw // 2

    def desc(self, n, h, w, c, dtype):
        key = (n, h, w, c, dtype)
        cache = self.__dict__.setdefault("_desc_cache", {})
        d = cache.get(key)
        if d is None:
            d = L.ConvDesc()
            d.n, d.h, d.w, d.c = n, h, w, c
            d.k, d.r, d.s = self.filters, self.kh, self.kw
            d.stride_h, d.stride_w = self.sh, self.sw
            d.pad_t, d.pad_b, d.pad_l, d.pad_r = self.pads_for(h, w)
            d.dtype = dtype_code(dtype)
            d.act = L.ACT_CODES[self.activation]
            d.act_alpha = self.act_alpha
            cache[key] = d
        return d

    def epilogue_bias(self):
        if self.bn_shift is not None:
            if self.bias is not None:
                raise NotImplementedError("conv bias + frozen BN")
            return self.bn_shift
        return self.bias

    def groupable(self, xs):
        """A list of inputs (pyramid levels) can go through this layer as one
        grouped launch per pass: stride 1, level-independent pads, one dtype."""
        return self.sh == 1 and self.sw == 1 and len({self.pads_for(*t.shape[1:3]) for t in xs}) == 1 and \
            len({t.dtype for t in xs}) == 1

    def check_input(self, x):
        if x is not None and x.shape[-1] != self.in_channels:
            raise ValueError(f"Conv2D {self.lname}: expected {self.in_channels} channels, got {x.shape[-1]}")

    def forward(self, x, residual=None):
        """x: one NHWC tensor, or a list of them (the pyramid levels through
        this one shared layer: a grouped launch per pass when stride is 1 and
        the 'same'/'valid' pads do not depend on the level size)."""
        if isinstance(x, (list, tuple)):
            for t in x:
                self.check_input(t)
            if residual is None and len(x) > 1 and self.groupable(x):
                return list(ops.ConvGroupedFn.apply(self, *x))
            res = residual if residual is not None else [None] * len(x)
            return [self.forward(t, r) for t, r in zip(x, res)]
        self.check_input(x)
        return ops.Conv2dFn.apply(x, self.kernel, self.bias, residual, self)


class Dense(_WeightLayer):
    """tf.keras.layers.Dense: kernel (in, out), y = act(x W + b)."""

    def __init__(self, in_features, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 act_alpha=0.2, out_f32=False, init=None, name=None):
        super().__init__()
        init = init or DEFAULT_INIT
        self.kernel = nn.Parameter(_make_kernel(init, kernel_initializer, (in_features, units), in_features, units))
        self.bias = nn.Parameter(torch.zeros(units)) if use_bias else None
        self.activation = activation
        self.act_alpha = act_alpha
        self.out_f32 = out_f32
        self.bn_scale = None
        self.lname = name
        self._init_copies()

    def _rsck(self):
        fin, fout = self.kernel.shape
        return 1, 1, fin, fout

    def forward(self, x, dropout=0.0, residual=None):
        """dropout / residual: residual + Dropout(dropout)(self(x)) fused into
        the GEMM epilogue (linear Dense only)."""
        return ops.LinearFn.apply(x, self.kernel, self.bias, self, float(dropout), residual)


class BatchNormalization(nn.Module):
    """tf.keras.layers.BatchNormalization(epsilon, momentum) over the channel
    (last) axis: gamma / beta trainable, moving_mean / moving_variance
    buffers (0 / 1). forward(x, training, activation, residual): training
    normalises with the batch statistics and moves the averages; inference
    uses the moving statistics. The activation ('relu6' | 'relu' | None) and
    a residual add follow the normalisation in the same kernel."""

    def __init__(self, channels, epsilon=1e-3, momentum=0.999):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))
        self.epsilon, self.momentum = epsilon, momentum
        # process group of a cross-replica (sync) BN under data parallelism
        # (fpnmt.dist.set_sync_batchnorm; None: this rank's batch only)
        self.sync_group = None

    def forward(self, x, training=True, activation=None, residual=None):
        act = L.ACT_CODES[activation]
        if training:
            return ops.BatchNormFn.apply(x, self.gamma, self.beta, self, act, residual)
        return ops.batch_norm_inference(x, self, act, residual)


class DepthwiseConv2D(nn.Module):
    """tf.keras.layers.DepthwiseConv2D(kernel_size, strides, use_bias=False):
    kernel (kh, kw, C, 1), glorot_uniform (fan_in = kh*kw*C, fan_out = kh*kw).
    pads = (top, bottom, left, right): 'same' at stride 1, or the explicit
    ZeroPadding2D(correct_pad) + 'valid' of MobileNetV2's stride-2 blocks."""

    def __init__(self, channels, kernel_size=3, strides=1, pads=(1, 1, 1, 1), init=None, name=None):
        super().__init__()
        init = init or DEFAULT_INIT
        self.kh = self.kw = kernel_size
        self.stride = strides
        self.pads = tuple(pads)
        self.lname = name
        k = kernel_size * kernel_size
        self.kernel = nn.Parameter(init.glorot_uniform((kernel_size, kernel_size, channels, 1), k * channels, k))

    def forward(self, x):
        return ops.DepthwiseConvFn.apply(x, self.kernel, self)


class LayerNormalization(nn.Module):
    def __init__(self, d, epsilon=1e-6):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(d))
        self.beta = nn.Parameter(torch.zeros(d))
        self.epsilon = epsilon

    def forward(self, x, residual=None, pe=None):
        return ops.LayerNormFn.apply(x, self.gamma, self.beta, residual, pe, self.epsilon, self)


class Embedding(nn.Module):
    """tf.keras.layers.Embedding (uniform(-0.05, 0.05) init); gathered straight
    from the fp32 master, fused with the positional-encoding add."""

    def __init__(self, vocab, d, init=None):
        super().__init__()
        init = init or DEFAULT_INIT
        self.embeddings = nn.Parameter(init.uniform((vocab, d), 0.05))
        self.sumsq_slot = None  # arena slot for the IndexedSlices clip norm

    def forward(self, tok, pe, dtype, dropout=0.0):
        """dropout: the caller's Dropout on the output, in the same launch."""
        slot = self.sumsq_slot
        if slot is None:
            slot = torch.zeros(1, dtype=torch.float32, device=self.embeddings.device)
        return ops.EmbedPosencFn.apply(tok, self.embeddings, pe, dtype, self, slot, dropout)


class DenseGroup:
    """Dense layers that read the SAME input — the K/V projections of one
    encoder view in every layer, the Q projections of all views in a layer, a
    decoder layer's self-attention Q/K/V, the cross-attention K/V of every
    decoder layer (reference: MultiHeadAttention.call, transformer.py:139-141,
    run per layer / per view). They run as ONE GEMM whose output columns are
    the members' outputs side by side (x @ [W_1 .. W_n] + [b_1 .. b_n]); the
    backward is one bias column-sum, one bwd-data GEMM over the concatenated
    gradient and one batched bwd-filter GEMM (see ops.ProjectionGroupFn).

    The members keep their own parameters (state dicts unchanged); their
    forward compute copies become slices of one stacked (n*out, in) operand.
    ``arena_order`` lists the members' kernels then biases so a ParamArena
    built in that order holds each as one contiguous block."""

    def __init__(self, layers):
        self.layers = list(layers)
        fin, fout = self.layers[0].kernel.shape
        for m in self.layers:
            if tuple(m.kernel.shape) != (fin, fout) or m.activation not in (None, "linear") or m.out_f32 \
                    or m.bias is None:
                raise ValueError("DenseGroup: members need equal shapes, linear activation, a bias")
        self.fin, self.fout, self.n = fin, fout, len(self.layers)
        for i, m in enumerate(self.layers):
            if m.__dict__.get("_group") is not None or m._copies:
                raise ValueError("DenseGroup: layer already grouped or already holds compute copies")
            m.__dict__["_group"] = (self, i)
        self._stack = {}

    def ensure(self, dt):
        if dt in self._stack:
            return
        n, fin, fout = self.n, self.fin, self.fout
        dev = self.layers[0].kernel.device
        stack = torch.empty(n * fout * fin, dtype=dt, device=dev)
        # flipped copies interleaved: (in, n*out), member i in columns [i*out, (i+1)*out)
        flip = torch.empty(fin, n * fout, dtype=dt, device=dev)
        self._stack[dt] = (stack, flip)
        for i, m in enumerate(self.layers):
            m._copies[dt] = (stack[i * fout * fin:(i + 1) * fout * fin], flip[:, i * fout:(i + 1) * fout])
            # the new slices hold no weights yet: every member must prepare
            # them (a member whose _gen is current would otherwise skip it)
            m._gen = -1

    def to_device_moved(self):
        """Drop stacked copies (after .to(device)); rebuilt on next use."""
        self._stack = {}
        for m in self.layers:
            m._copies = {}

    def stacked(self, dt):
        """((n*out, in) forward operand, (in, n*out) flipped operand), refreshed
        if stale."""
        for m in self.layers:
            m.compute_weights(dt)
        return self._stack[dt]

    def params(self):
        return [m.kernel for m in self.layers] + [m.bias for m in self.layers]

    @staticmethod
    def _contig(ts, per):
        base = ts[0]
        es = base.element_size()
        sp = base.untyped_storage().data_ptr()
        for i, t in enumerate(ts):
            # same storage (adjacent separate allocations do not count)
            if t is None or t.untyped_storage().data_ptr() != sp or t.data_ptr() != base.data_ptr() + i * per * es:
                return False
        return True

    def bias_cat(self):
        """[n*out] fp32 bias: a view when the biases are adjacent (arena order),
        else a fresh concatenation."""
        bs = [m.bias for m in self.layers]
        if self._contig(bs, self.fout):
            return bs[0].detach().view(-1).as_strided((self.n * self.fout,), (1,))
        return torch.cat([b.detach() for b in bs])

    def grad_views(self):
        """(kernel grads as (n, in, out), bias grads as (n*out,)) when each set
        is one contiguous block of gradient storage, else (None, None)."""
        from .ops import _grad_of
        kg = [_grad_of(m.kernel) for m in self.layers]
        bg = [_grad_of(m.bias) for m in self.layers]
        k = kg[0].as_strided((self.n, self.fin, self.fout), (self.fin * self.fout, self.fout, 1)) \
            if self._contig(kg, self.fin * self.fout) else None
        b = bg[0].as_strided((self.n * self.fout,), (1,)) if self._contig(bg, self.fout) else None
        return k, b

    def __call__(self, x):
        """x (..., in) -> tuple of n outputs (..., out): strided views of one
        (rows, n*out) buffer."""
        return ops.ProjectionGroupFn.apply(x, self, self.layers[0].kernel)


def group_param_order(model, named):
    """Reorder (name, param) pairs so that every DenseGroup of `model` has its
    kernels, then its biases, adjacent (one contiguous arena block each)."""
    groups = []
    seen = set()
    for m in model.modules():
        g = m.__dict__.get("_group")
        if g is not None and id(g[0]) not in seen:
            seen.add(id(g[0]))
            groups.append(g[0])
    name_of = {id(p): n for n, p in named}
    first = {}
    for g in groups:
        ps = [p for p in g.params() if id(p) in name_of]
        if len(ps) != len(g.params()):
            continue  # some member frozen: keep the default order
        for p in ps:
            first[id(p)] = g
    out, done = [], set()
    for n, p in named:
        if id(p) in done:
            continue
        g = first.get(id(p))
        if g is None:
            out.append((n, p))
            done.add(id(p))
            continue
        for q in g.params():
            if id(q) not in done:
                out.append((name_of[id(q)], q))
                done.add(id(q))
    return out


def weight_layers(model):
    return [m for m in model.modules() if isinstance(m, _WeightLayer)]


class WeightPrepPlan:
    """All compute-copy refreshes of a model as ONE fpnmt_weight_prep_batched
    launch per dtype (the item table is static: masters live in the arena,
    copies are allocated once), so the per-step refresh is a single graph node."""

    def __init__(self, model, dtypes, skip=()):
        self.layers = [m for m in weight_layers(model) if id(m) not in skip]
        self.tables = []
        for dt in dtypes:
            items = (L.WPrepItem * max(1, len(self.layers)))()
            tiles = 0
            for i, m in enumerate(self.layers):
                r, s, c, k = m._rsck()
                wf, wb = m.ensure_copies(dt)
                it = items[i]
                it.w_hwio = m.kernel.data_ptr()
                it.scale = m.bn_scale.data_ptr() if m.bn_scale is not None else None
                it.w_ohwi, it.w_flip = wf.data_ptr(), wb.data_ptr()
                it.r, it.s, it.c, it.k = r, s, c, k
                it.tile_start = tiles
                it.ld_flip = m.flip_ld()
                tiles += r * s * ((c + 31) // 32) * ((k + 31) // 32)
            raw = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8)
            dev = self.layers[0].kernel.device if self.layers else torch.device("cpu")
            self.tables.append((dt, raw.to(dev), len(self.layers), tiles))

    def run(self):
        for dt, table, n, tiles in self.tables:
            call("fpnmt_weight_prep_batched", table.data_ptr(), n, tiles, dtype_code(dt), stream_ptr())
        for m in self.layers:
            m._gen = _GEN[0]


def _fastdiv(d):
    """(magic, shift) with q // d == ((q * magic >> 32) + q) >> shift (csrc make_fastdiv)."""
    d = max(int(d), 1)
    sh = 0
    while (1 << sh) < d:
        sh += 1
    return (((1 << 32) * ((1 << sh) - d)) // d + 1) & 0xFFFFFFFF, sh


class FusedPrep:
    """Per-segment fpnmt_seg_prep table for fpnmt_amsgrad_step_prep: the
    trainable conv / dense kernels whose compute copies are bf16 only and
    whose k is a power of two in [16, 4096] get their copies written by the
    optimizer kernel; `layers` is the set the separate refresh then skips."""

    def __init__(self, model, arena):
        self.layers = set()
        self._mods = []
        n = len(arena.params)
        tab = (L.SegPrep * max(1, n))()
        for m in weight_layers(model):
            seg = arena.index.get(id(m.kernel))
            if seg is None or set(m._copies) != {torch.bfloat16}:
                continue
            r, s, c, k = m._rsck()
            wf, wb = m._copies[torch.bfloat16]
            scale_ok = m.bn_scale is None or m.bn_scale.data_ptr() % 16 == 0
            if (k & (k - 1)) or not 16 <= k <= 4096 or not scale_ok or m.flip_ld() % 4 \
                    or wf.data_ptr() % 8 or wb.data_ptr() % 8:
                continue
            e = tab[seg]
            e.ohwi, e.flip = wf.data_ptr(), wb.data_ptr()
            e.scale = m.bn_scale.data_ptr() if m.bn_scale is not None else None
            e.r, e.s, e.c, e.k = r, s, c, k
            e.ld_flip = m.flip_ld()
            e.c_magic, e.c_shift = _fastdiv(c)
            self.layers.add(id(m))
            self._mods.append(m)
        raw = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8)
        self.table = raw.to(arena.flat.device) if self.layers else None

    def mark_fresh(self):
        for m in self._mods:
            m._gen = _GEN[0]


def fused_prep(model, arena):
    """The model's FusedPrep for this arena (rebuilt when the compute copies
    or the arena change; None when config.fuse_optimizer_prep is off)."""
    import fpnmt
    if not fpnmt.config.fuse_optimizer_prep or not arena.flat.is_cuda:
        return None
    wl = weight_layers(model)
    key = (arena.flat.data_ptr(), tuple((tuple(sorted(str(d) for d in m._copies)),
                                         tuple(t.data_ptr() for c in m._copies.values() for t in c)) for m in wl))
    # every table ever built stays alive: a captured optimizer graph holds its
    # device pointer (a replaced, freed table would be reused memory there)
    tabs = model.__dict__.setdefault("_fpnmt_fused_preps", {})
    if key not in tabs:
        tabs[key] = FusedPrep(model, arena)
    return tabs[key]


def prepare_all(model, dtype=None, skip=()):
    """Refresh every compute copy (one batched launch per dtype in use);
    layers whose id is in `skip` were refreshed by the optimizer kernel."""
    dts = set()
    wl = [m for m in weight_layers(model) if id(m) not in skip]
    for m in wl:
        dts.update(m._copies.keys())
    if dtype is not None:
        dts.add(dtype)
    # the item table holds raw master / BN-scale pointers: a model re-adopted
    # by a new ParamArena (a second TrainEngine) must get a new table, or the
    # launch would read the old arena's (possibly unmapped) storage
    ptrs = tuple((m.kernel.data_ptr(), m.bn_scale.data_ptr() if m.bn_scale is not None else 0) for m in wl)
    key = (tuple(sorted(str(d) for d in dts)), ptrs)
    # plans are kept per key, never replaced: a captured graph holds the item
    # table's device pointer, and the refresh with and without the fused
    # optimizer layers (skip) alternate between capture and eager / restore
    plans = model.__dict__.setdefault("_fpnmt_wprep_plans", {})
    if key not in plans:
        plans[key] = WeightPrepPlan(model, sorted(dts, key=str), skip)
    plans[key].run()
