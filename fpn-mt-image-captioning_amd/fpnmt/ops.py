"""autograd Functions over the libfpnmt C-ABI.

Each Function launches hand-written gfx950 kernels on torch's current stream
(so whole training steps are hipGraph-capturable) and writes parameter
gradients straight into the arena's fp32 gradient views (``param.grad``),
accumulating — shared weights (the per-level FPN heads, retinanet.py:297-301)
therefore sum their five contributions with no extra kernels. Such Functions
return ``None`` for the parameter inputs so autograd never allocates or adds
parameter gradients itself.

Numerics follow the reference's TF ops (see oracle/ref_cpu.py for the CPU
restatement they are checked against).
"""
from __future__ import annotations

import math

import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr, dtype_code

class Runtime:
    """Dropout keys: hash(base_seed, site, seed_tensor) where `site` numbers
    the dropout sites of one forward in call order (the TrainEngine restarts
    it at every step, so the n-th site of a step is the same layer in eager
    steps, captured graphs and a resumed process alike) and seed_tensor is the
    device-side optimizer step (a replayed graph draws new masks every step).
    A resumed run therefore reproduces the uninterrupted run's masks."""
    seed_tensor = None  # device int64 (optimizer step) mixed into dropout keys
    base_seed = 0x5EED
    site = 0
    on_transformer_grads = None  # callback: the transformer's backward is complete (transformer_grads_barrier)

    def reset_sites(self):
        self.site = 0

    def next_seed(self):
        self.site += 1
        return (self.base_seed * 1000003 + self.site) & 0xFFFFFFFFFFFF


runtime = Runtime()


class _SideStream:
    """Weight-gradient launches on a second HIP stream (ops.side_wgrad()).

    In the backward, a layer's dgrad feeds the next layer's backward (the
    critical path) while its weight gradient only feeds the optimizer; most
    of the transformer's and the small pyramid levels' launches are
    latency-bound and leave CUs idle, so the weight gradients run beside the
    dgrad chain. Each launch forks from the compute stream (an event wait:
    captured as a graph edge), uses its own split-K workspace (the process
    workspace is swapped for the call; the pointers are baked into the
    launch), and keeps its operands alive until side_wgrad() joins the
    streams. Weight-gradient launches of one step all go to the one side
    stream, so two accumulations into a shared weight's gradient never race."""

    def __init__(self):
        self.active = False
        self.mode = None
        self.stream = None
        self.keep = []
        self.queue = []
        self.pending = False


_side = _SideStream()


def _wgrad(fn, *keep, conv=False):
    """Run fn() (a weight-gradient launch on the current stream) inline, or on
    the side stream inside side_wgrad(). conv: a convolution's (kept on the
    compute stream unless config.side_wgrad == "all": the pyramid's weight
    gradients are large MFMA GEMMs that contend with the dgrads instead of
    filling idle CUs)."""
    sd = _side
    if not sd.active or (conv and sd.mode != "all"):
        if not conv:
            # inside deferred_reductions a Dense weight gradient is queued and
            # run at the flush (grouped launches): its operands must live until then
            for t in keep:
                L.defer_keep(t)
        fn()
        return
    # deferred and launched in batches: every fork / join is a cross-stream
    # dependency in the captured graph, which costs more than a small launch
    sd.queue.append(fn)
    sd.keep.extend(keep)
    if len(sd.queue) >= SIDE_BATCH:
        _flush_side()


SIDE_BATCH = 16


def _flush_side():
    sd = _side
    if not sd.queue:
        return
    sd.stream.wait_stream(torch.cuda.current_stream())
    with L.side_workspace(), torch.cuda.stream(sd.stream):
        for fn in sd.queue:
            fn()
    sd.queue.clear()
    sd.pending = True


class side_wgrad:
    """Context: weight-gradient launches of the backward(s) inside run on the
    side stream; on exit the compute stream waits for them (graph-capturable
    fork / join). Off unless fpnmt.config.side_wgrad."""

    def __init__(self, enabled=True):
        self.enabled = enabled

    def __enter__(self):
        from . import config
        self.prev = _side.active
        if self.enabled and config.side_wgrad and not L.defer_active():  # the deferral is single-stream
            if _side.stream is None:
                _side.stream = torch.cuda.Stream()
            _side.active = True
            _side.mode = config.side_wgrad
        return self

    def __exit__(self, *exc):
        _side.active = self.prev
        if not self.prev:
            join_side()
        return False


def join_side():
    """The compute stream waits for every weight-gradient launch so far."""
    _flush_side()
    if _side.pending:
        torch.cuda.current_stream().wait_stream(_side.stream)
        _side.pending = False
    _side.keep.clear()


class _TransformerGradsBarrier(torch.autograd.Function):
    """Identity on the feature extractor's level outputs, placed where the
    encoder takes them. Its backward runs once the gradients of all five
    levels are in, which is after EVERY transformer node's backward: autograd
    runs the ready node created last first, the transformer's nodes were all
    created after this one, and none of them waits for a node created before
    it. There the transformer's parameter gradients are complete (once the
    deferred queue is flushed), and runtime.on_transformer_grads (the
    TrainEngine's early optimizer part) is called."""

    @staticmethod
    def forward(ctx, *xs):
        return tuple(x.view_as(x) for x in xs)

    @staticmethod
    def backward(ctx, *gs):
        cb = runtime.on_transformer_grads
        if cb is not None:
            cb()
        return gs


def transformer_grads_barrier(xs):
    """xs (the level outputs) through _TransformerGradsBarrier when a callback
    is armed and a backward will run; xs unchanged otherwise."""
    if runtime.on_transformer_grads is None or not torch.is_grad_enabled() or not any(x.requires_grad for x in xs):
        return xs
    return list(_TransformerGradsBarrier.apply(*xs))


def _grad_of(p):
    """fp32 gradient view of a parameter (arena view when adopted)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p, dtype=torch.float32)
    return p.grad


def _empty(shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


# --------------------------------------------------------------------- conv
def conv_out_size(h, pa, pb, k, s):
    return (h + pa + pb - k) // s + 1


def _conv_fwd(layer, x, residual):
    n, h, w, c = x.shape
    pt, pb, pl, pr = layer.pads_for(h, w)
    ho = max(conv_out_size(h, pt, pb, layer.kh, layer.sh), 0)
    wo = max(conv_out_size(w, pl, pr, layer.kw, layer.sw), 0)
    y = _empty((n, ho, wo, layer.filters), x.dtype, x.device)
    d = layer.desc(n, h, w, c, x.dtype)
    wf, _ = layer.compute_weights(x.dtype)
    call("fpnmt_conv2d_fwd", d, ptr(x), ptr(wf), None, ptr(layer.epilogue_bias()), ptr(residual), ptr(y),
         stream_ptr())
    return y


def _bias_grad_ptr(layer):
    return _grad_of(layer.bias).data_ptr() if (layer.bias is not None and layer.bias.requires_grad) else None


def _act_grad(layer, dy, y, s, fold=True):
    """(dz, folded): dz = dy * act'(y) (+ the bias gradient's column sums);
    folded: with no activation (dz == dy) the column sums are left to the
    layer's weight-gradient launch (_fold_bias; fold=False: never)."""
    act = L.ACT_CODES[layer.activation]
    if act == L.ACT_NONE:
        if fold and _fold_bias(layer):
            return dy, True
        bias_grad(dtype_code(y.dtype), y.numel() // layer.filters if layer.filters else 0, layer.filters, dy,
                  _bias_grad_ptr(layer), s)
        return dy, False
    dz = torch.empty_like(dy)
    act_bwd(dtype_code(y.dtype), y.numel() // layer.filters if layer.filters else 0, layer.filters, act,
            layer.act_alpha, dy, y, dz, _bias_grad_ptr(layer), s)
    return dz, False


def _fold_bias(layer):
    """The layer's bias gradient rides in its weight-gradient launch
    (fpnmt_conv2d_bwd_filter_bias: the column sums of the dz tiles the LDS-DMA
    wgrad kernel streams anyway; fpnmt.config.fuse_bias_wgrad) instead of a
    separate column pass over dz. Only where that pass would read dz itself
    (not where act_bwd produces dz and sums it in the same pass)."""
    import fpnmt
    return (fpnmt.config.fuse_bias_wgrad and layer.kernel.requires_grad and layer.bias is not None
            and layer.bias.requires_grad)


def _bwd_filter(d, layer, x, dz, gk, fold):
    """dw (+ db when fold) of one conv: fpnmt_conv2d_bwd_filter[_bias]. A
    column pass the library queues in a deferred region reads dz at the flush:
    dz is held until then (L.defer_keep)."""
    if fold:
        L.defer_keep(dz)
        call("fpnmt_conv2d_bwd_filter_bias", d, ptr(x), ptr(dz), ptr(layer.bn_scale), ptr(gk), _bias_grad_ptr(layer),
             stream_ptr())
    else:
        call("fpnmt_conv2d_bwd_filter", d, ptr(x), ptr(dz), ptr(layer.bn_scale), ptr(gk), stream_ptr())


def _fusable_act(layer):
    """Activations whose backward a bwd-data epilogue can apply: 0/1 derivatives."""
    a = L.ACT_CODES[layer.activation]
    return a if a in (L.ACT_RELU, L.ACT_RELU6) else None


def _input_act(x):
    """(act, producer node) when x is the ReLU / ReLU6 output of a Conv2dFn or
    of a ConvChainFn's last layer (a ResNet stage output, the stem, a ReLU FPN
    conv): a consumer's backward can fold that act' into the gradient it
    writes (fuse_input_act); (None, None) otherwise."""
    import fpnmt
    prev = getattr(x, "grad_fn", None) if fpnmt.config.fuse_input_act else None
    if prev is None:
        return None, None
    kind = type(prev).__name__
    if kind == "ConvChainFnBackward":
        act = _fusable_act(prev.layers[-1])
    elif kind == "Conv2dFnBackward":
        act = _fusable_act(prev.layer)
    else:
        return None, None
    return (act, prev) if act is not None else (None, None)


def _pool_input_act(x, nonoverlap):
    """(act, alpha, producer node) for a max pool's input x: a ReLU / ReLU6
    output of a conv / conv chain / grouped conv (chain), or a LeakyReLU one
    when the windows do not overlap (the derivative then multiplies one
    routed dy: the same single rounding as the separate pass)."""
    import fpnmt
    prev = getattr(x, "grad_fn", None) if fpnmt.config.fuse_input_act else None
    if prev is None:
        return None, 0.0, None
    kind = type(prev).__name__
    if kind in ("ConvChainFnBackward", "ConvGroupedChainFnBackward"):
        layer = prev.layers[-1]
    elif kind in ("Conv2dFnBackward", "ConvGroupedFnBackward"):
        layer = prev.layer
    else:
        return None, 0.0, None
    act = L.ACT_CODES[layer.activation]
    if act in (L.ACT_RELU, L.ACT_RELU6) or (act == L.ACT_LEAKY and nonoverlap):
        return act, float(layer.act_alpha), prev
    return None, 0.0, None


def _act_applied(dy, node):
    """dy is exactly the gradient some consumer(s) already multiplied by the
    act' of `node`'s output (tagged, and not modified since)."""
    tag = getattr(dy, "_fpnmt_act_applied", None)
    if tag is not None and tag[0] is node and tag[1] == dy._version:
        return True
    if getattr(node, "_fpnmt_leaky_folded", False):
        # a max pool multiplied ITS routed dy by LeakyReLU'(y) (not
        # idempotent, unlike ReLU's 0/1 mask) and autograd then summed it
        # with another consumer's gradient, dropping the tag: the producer's
        # act_bwd would scale the pool's negative entries by alpha twice
        raise RuntimeError("fpnmt: a LeakyReLU output folded into its max pool's backward has another "
                           "consumer; set fpnmt.config.fuse_input_act = False for this model")
    return False


def _bwd_data_into(ctx, d, dz, wflip, dx, accumulate, x, s):
    """dx (+)= conv_transpose(dz, w), times act'(x) of x's producer when
    ctx.in_act is set (every contribution masked: fpnmt_conv2d_bwd_data_mask)."""
    if ctx.in_act is not None:
        call("fpnmt_conv2d_bwd_data_mask", d, ptr(dz), ptr(wflip), ptr(dx), 1 if accumulate else 0, ptr(x),
             ctx.in_act, s)
    else:
        call("fpnmt_conv2d_bwd_data", d, ptr(dz), ptr(wflip), ptr(dx), 1 if accumulate else 0, s)


class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, bias, residual, layer):
        ctx.gsum = _gsum_register(x)
        ctx.in_act, ctx.in_prev = _input_act(x)
        x = x.contiguous()
        if residual is not None:
            residual = residual.contiguous()
        y = _conv_fwd(layer, x, residual)
        ctx.layer = layer
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        layer = ctx.layer
        n, h, w, c = x.shape
        d = layer.desc(n, h, w, c, x.dtype)
        s = stream_ptr()
        if _act_applied(dy, ctx):  # the consumers' epilogues multiplied dy by act'(y)
            dz, fold = dy, _fold_bias(layer)
            if not fold:
                bias_grad(dtype_code(dy.dtype), dy.numel() // layer.filters, layer.filters, dy, _bias_grad_ptr(layer),
                          s)
        else:
            dz, fold = _act_grad(layer, dy.contiguous(), y, s)
        dx = None
        if ctx.needs_input_grad[0]:
            _, wflip = layer.compute_weights(x.dtype)
            acc = _gsum_acc(ctx.gsum)
            dx = acc if acc is not None else torch.empty_like(x)
            _bwd_data_into(ctx, d, dz, wflip, dx, acc is not None, x, s)
            dx = _gsum_done(ctx.gsum, dx, True, mask_node=ctx.in_prev)
        if layer.kernel.requires_grad:
            gk = _grad_of(layer.kernel)
            _wgrad(lambda: _bwd_filter(d, layer, x, dz, gk, fold), x, dz, conv=True)
        return dx, None, None, (dz if ctx.has_res else None), None


class ConvChainFn(torch.autograd.Function):
    """Conv2D layers applied in sequence whose intermediate outputs have no
    other consumer — keras-resnet's bottleneck 2a -> 2b -> 2c(+shortcut), a
    retinanet submodel's ReLU convs and the head after them. Same forward
    launches as layer-by-layer Conv2dFn; the backward fuses each intermediate's
    ReLU / ReLU6 derivative into the bwd-data GEMM that produces its gradient
    (fpnmt_conv2d_bwd_data_act), so the intermediates get no act_bwd pass
    (bit-identical: the derivative is a 0/1 mask)."""

    @staticmethod
    def forward(ctx, x, residual, *layers):
        ctx.gsum = _gsum_register(x) if residual is not x else None
        ctx.in_act, ctx.in_prev = _input_act(x)
        x = x.contiguous()
        if residual is not None:
            residual = residual.contiguous()
        ys = []
        cur = x
        for i, layer in enumerate(layers):
            cur = _conv_fwd(layer, cur, residual if i == len(layers) - 1 else None)
            ys.append(cur)
        ctx.layers = layers
        ctx.has_res = residual is not None
        ctx.res_is_x = residual is not None and residual is x  # identity bottleneck
        # x produced by another chain whose last layer ends in a 0/1-derivative
        # activation (the previous bottleneck's output ReLU): its act' can go
        # into this chain's fused bwd-data epilogue (backward, i == 0)
        ctx.x_act, ctx.x_prev = None, None
        prev = x.grad_fn
        if ctx.res_is_x and prev is not None and type(prev).__name__ == "ConvChainFnBackward":
            ctx.x_act = _fusable_act(prev.layers[-1])
            ctx.x_prev = prev if ctx.x_act is not None else None
        ctx.save_for_backward(x, *ys)
        return cur

    @staticmethod
    def backward(ctx, dy):
        x, *ys = ctx.saved_tensors
        layers = ctx.layers
        s = stream_ptr()
        last = len(layers) - 1
        if _act_applied(dy, ctx):
            # the consumer chain's bwd-data epilogue already multiplied this
            # exact gradient by act'(y) and nothing was added to it since (an
            # autograd accumulation in place would have bumped its version;
            # an out-of-place one yields an untagged tensor): only the bias
            # column sums remain (bias_grad == act_bwd's, bit for bit)
            dz, fold = dy, _fold_bias(layers[last])
            if not fold:
                bias_grad(dtype_code(dy.dtype), dy.numel() // layers[last].filters, layers[last].filters, dy,
                          _bias_grad_ptr(layers[last]), s)
        else:
            dz, fold = _act_grad(layers[last], dy.contiguous(), ys[last], s)
        dres = dz if ctx.has_res else None
        dx = None
        for i in range(last, -1, -1):
            layer = layers[i]
            xin = x if i == 0 else ys[i - 1]
            n, h, w, c = xin.shape
            d = layer.desc(n, h, w, c, xin.dtype)
            if layer.kernel.requires_grad:
                gk = _grad_of(layer.kernel)
                _wgrad(lambda d=d, xin=xin, dz=dz, layer=layer, gk=gk, fold=fold: _bwd_filter(
                    d, layer, xin, dz, gk, fold), xin, dz, conv=True)
            if i == 0 and not ctx.needs_input_grad[0]:
                break
            _, wflip = layer.compute_weights(xin.dtype)
            dprev = torch.empty_like(xin)
            if i == 0:
                import fpnmt
                if (dres is not None and ctx.res_is_x and fpnmt.config.fuse_identity_residual
                        and layer.sh == 1 and layer.sw == 1):
                    # x is also the residual: its two gradients summed in the epilogue
                    if ctx.x_act is not None and fpnmt.config.fuse_block_act:
                        # ... times act'(x) of the producing chain's output activation
                        call("fpnmt_conv2d_bwd_data_res_act", d, ptr(dz), ptr(wflip), ptr(dprev), ptr(dres),
                             ptr(x), ctx.x_act, s)
                        dprev._fpnmt_act_applied = (ctx.x_prev, dprev._version)
                    else:
                        call("fpnmt_conv2d_bwd_data_res", d, ptr(dz), ptr(wflip), ptr(dprev), ptr(dres), s)
                    dres = None
                else:
                    acc = _gsum_acc(ctx.gsum)
                    if acc is not None:
                        dprev = acc
                    _bwd_data_into(ctx, d, dz, wflip, dprev, acc is not None, x, s)
                    dprev = _gsum_done(ctx.gsum, dprev, True, mask_node=ctx.in_prev)
                dx = dprev
                break
            prev = layers[i - 1]
            act = _fusable_act(prev)
            if act is not None and layer.sh == 1 and layer.sw == 1:
                call("fpnmt_conv2d_bwd_data_act", d, ptr(dz), ptr(wflip), ptr(dprev), ptr(xin), act, s)
                db = _bias_grad_ptr(prev)
                fold = db is not None and _fold_bias(prev)
                if db is not None and not fold:  # column sums only (dz == dy: nothing rewritten)
                    bias_grad(dtype_code(xin.dtype), xin.numel() // prev.filters, prev.filters, dprev, db, s)
                dz = dprev
            else:
                call("fpnmt_conv2d_bwd_data", d, ptr(dz), ptr(wflip), ptr(dprev), 0, s)
                dz, fold = _act_grad(prev, dprev, xin, s)
        return (dx, dres) + (None,) * len(layers)


_BOTTLENECK_SHAPES = {(56, 56, 256, 64), (28, 28, 512, 128)}  # fpnmt_bottleneck_fwd's kernels


def bottleneck_fused(block, x):
    """A keras-resnet identity bottleneck (2a 1x1 -> 2b 3x3 -> 2c 1x1 + x, all
    ReLU, frozen BN folded; reference models/resnet.py:99-112) as ONE
    fpnmt_bottleneck_fwd launch, the intermediates kept on chip. Inference
    only (no autograd graph is recorded): returns None when the block, the
    dtype or the shape has no fused kernel, or a gradient is needed, and the
    caller runs the three convs."""
    a, b, c = block.conv2a, block.conv2b, block.conv2c
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in block.parameters())):
        return None
    if x.dtype != torch.bfloat16 or x.dim() != 4 or not x.is_cuda:
        return None
    n, h, w, cin = x.shape
    cm = a.filters
    if (h, w, cin, cm) not in _BOTTLENECK_SHAPES or c.filters != cin or b.filters != cm:
        return None
    if (a.kh, a.kw, a.sh, a.sw) != (1, 1, 1, 1) or (b.kh, b.kw, b.sh, b.sw) != (3, 3, 1, 1) or \
            (c.kh, c.kw, c.sh, c.sw) != (1, 1, 1, 1) or b.pads_for(h, w) != (1, 1, 1, 1):
        return None  # the kernel assumes unit strides everywhere and a 'same' 3x3
    if any(L.ACT_CODES[m.activation] != L.ACT_RELU for m in (a, b, c)):
        return None
    x = x.contiguous()
    y = torch.empty_like(x)
    wa, _ = a.compute_weights(x.dtype)
    w3, _ = b.compute_weights(x.dtype)
    wc, _ = c.compute_weights(x.dtype)
    ba, b3, bc = (_f32_bias(m) for m in (a, b, c))
    st = L.lib.fpnmt_bottleneck_fwd(n, h, w, cin, cm, ptr(x), ptr(wa), ptr(ba), ptr(w3), ptr(b3), ptr(wc), ptr(bc),
                                    ptr(y), stream_ptr())
    if st == L.E_UNSUPPORTED:
        return None
    L.check(st, "fpnmt_bottleneck_fwd")
    return y


def _f32_bias(layer):
    """The layer's fp32 epilogue bias (the folded BN shift), zeros if none."""
    bi = layer.epilogue_bias()
    if bi is None:
        z = layer.__dict__.get("_zero_bias")
        if z is None or z.device != layer.kernel.device:
            z = layer.__dict__["_zero_bias"] = torch.zeros(layer.filters, dtype=torch.float32,
                                                           device=layer.kernel.device)
        return z
    return bi if bi.dtype == torch.float32 else bi.float()


def conv_chain(layers, x, residual=None):
    """y = layers[-1](... layers[0](x) ..., residual=residual) with the fused
    chain backward (ConvChainFn); a list x (pyramid levels through shared
    layers) runs every layer as one grouped launch per pass
    (ConvGroupedChainFn) when each layer qualifies for grouping."""
    if isinstance(x, (list, tuple)):
        for t in x:
            layers[0].check_input(t)
        if residual is None and len(x) > 1 and all(layer.groupable(x) for layer in layers):
            return list(ConvGroupedChainFn.apply(tuple(layers), *x))
        res = residual if residual is not None else [None] * len(x)
        return [conv_chain(layers, t, r) for t, r in zip(x, res)]
    layers[0].check_input(x)
    return ConvChainFn.apply(x, residual, *layers)


def _grouped_desc(layer, xs):
    d = L.ConvDesc()
    d.c, d.k, d.r, d.s = layer.in_channels, layer.filters, layer.kh, layer.kw
    d.stride_h, d.stride_w = 1, 1
    d.pad_t, d.pad_b, d.pad_l, d.pad_r = layer.pads_for(*xs[0].shape[1:3])
    d.dtype = dtype_code(xs[0].dtype)
    d.act = L.ACT_CODES[layer.activation]
    d.act_alpha = layer.act_alpha
    return d


def _grouped_fwd(layer, xs):
    d = _grouped_desc(layer, xs)
    lv = (L.ConvLevel * len(xs))()
    ys = []
    for i, x in enumerate(xs):
        n, h, w, _ = x.shape
        ho = conv_out_size(h, d.pad_t, d.pad_b, d.r, 1)
        wo = conv_out_size(w, d.pad_l, d.pad_r, d.s, 1)
        y = _empty((n, max(ho, 0), max(wo, 0), layer.filters), x.dtype, x.device)
        lv[i].n, lv[i].h, lv[i].w = n, h, w
        lv[i].x, lv[i].y = ptr(x) or None, ptr(y) or None
        ys.append(y)
    wf, _ = layer.compute_weights(xs[0].dtype)
    call("fpnmt_conv2d_fwd_grouped", d, len(xs), lv, ptr(wf), None, ptr(layer.epilogue_bias()), stream_ptr())
    return ys


def _grouped_act_grad(layer, dys, ys, s, node=None):
    """(dzs, folded): per level dz = dy * act'(y) (+ bias column sums); None
    for levels with no gradient or no pixels. A level's dy that its consumer
    already multiplied by act'(y) (tagged for `node`, this Function's
    backward) gets the bias column sums only. folded: every level's dz is its
    dy (no act_bwd pass), and the column sums are left to the grouped
    weight-gradient launch (_fold_bias)."""
    live = [(y, dy) for y, dy in zip(ys, dys) if dy is not None and y.numel() > 0]
    applied = [node is not None and _act_applied(dy, node) for _, dy in live]
    if live and _fold_bias(layer) and (all(applied) or L.ACT_CODES[layer.activation] == L.ACT_NONE):
        return [dy.contiguous() if (dy is not None and y.numel() > 0) else None for y, dy in zip(ys, dys)], True
    dzs = []
    for y, dy in zip(ys, dys):
        if dy is None or y.numel() == 0:
            dzs.append(None)
            continue
        if node is not None and _act_applied(dy, node):
            bias_grad(dtype_code(dy.dtype), dy.numel() // layer.filters, layer.filters, dy, _bias_grad_ptr(layer), s)
            dzs.append(dy)
            continue
        dz, _ = _act_grad(layer, dy.contiguous(), y, s, fold=False)
        dzs.append(dz)
    return dzs, False


def _grouped_bwd_filter(layer, xs, dzs, s=None, fold=False):
    """dw (+ db, the column sums of every level's dz, when fold) of a shared
    conv over the levels: one fpnmt_conv2d_bwd_filter_grouped[_bias] launch."""
    d = _grouped_desc(layer, xs)
    lv = (L.ConvLevel * len(xs))()
    for i, (x, dz) in enumerate(zip(xs, dzs)):
        if dz is None:
            continue
        lv[i].n, lv[i].h, lv[i].w = x.shape[:3]
        lv[i].x, lv[i].dz = ptr(x) or None, ptr(dz) or None
    gk = _grad_of(layer.kernel)
    if fold:
        for z in dzs:
            if z is not None:
                L.defer_keep(z)  # a queued column pass reads it at the flush
        fn = lambda: call("fpnmt_conv2d_bwd_filter_grouped_bias", d, len(xs), lv, ptr(layer.bn_scale), ptr(gk),
                          _bias_grad_ptr(layer), stream_ptr())
    else:
        fn = lambda: call("fpnmt_conv2d_bwd_filter_grouped", d, len(xs), lv, ptr(layer.bn_scale), ptr(gk),
                          stream_ptr())
    _wgrad(fn, *xs, *[z for z in dzs if z is not None], conv=True)


def _grouped_bwd_data(layer, xs, dzs, s, act_in=None, acc=None, mask=None):
    """dx per level; act_in: the producing layer's fusable activation, whose
    derivative at y_in = xs is applied in the epilogue; acc: per-level running
    gradient sums to accumulate into (returned as the dxs); mask = (act, ys):
    each level's contribution times act'(ys[i]) (None: that level unmasked;
    fpnmt_conv2d_bwd_data_grouped_mask, accumulating too)."""
    d = _grouped_desc(layer, xs)
    _, wflip = layer.compute_weights(xs[0].dtype)
    lv = (L.ConvLevel * len(xs))()
    dxs = []
    for i, (x, dz) in enumerate(zip(xs, dzs)):
        if acc is not None:
            dx = acc[i]
        else:
            dx = torch.empty_like(x) if dz is not None else torch.zeros_like(x)
        dxs.append(dx)
        if dz is None:
            continue  # n = 0: level skipped
        lv[i].n, lv[i].h, lv[i].w = x.shape[:3]
        lv[i].x, lv[i].y = ptr(dz) or None, ptr(dx) or None
        lv[i].residual = ptr(x) or None
        if mask is not None:
            lv[i].residual = ptr(mask[1][i]) if mask[1][i] is not None else None
    if mask is not None:
        call("fpnmt_conv2d_bwd_data_grouped_mask", d, len(xs), lv, ptr(wflip), 1 if acc is not None else 0,
             mask[0], s)
    elif act_in is None:
        call("fpnmt_conv2d_bwd_data_grouped", d, len(xs), lv, ptr(wflip), 1 if acc is not None else 0, s)
    else:
        call("fpnmt_conv2d_bwd_data_grouped_act", d, len(xs), lv, ptr(wflip), act_in, s)
    return dxs


class ConvGroupedFn(torch.autograd.Function):
    """One shared-weight Conv2D over a list of inputs (the FPN levels) as ONE
    grouped implicit GEMM per pass (fpnmt_conv2d_*_grouped): forward, bwd-data
    and bwd-filter each launch once for all levels (retinanet.py:297-301 runs
    the same layers per level). Stride-1 convs with level-independent pads."""

    @staticmethod
    def forward(ctx, layer, *xs):
        xs = [x.contiguous() for x in xs]
        ys = _grouped_fwd(layer, xs)
        ctx.layer = layer
        ctx.save_for_backward(*xs, *ys)
        ctx.n = len(xs)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        saved = ctx.saved_tensors
        n = ctx.n
        xs, ys = saved[:n], saved[n:]
        layer = ctx.layer
        s = stream_ptr()
        dzs, fold = _grouped_act_grad(layer, dys, ys, s, node=ctx)
        dxs = [None] * n
        if any(ctx.needs_input_grad[1:]):
            dxs = _grouped_bwd_data(layer, xs, dzs, s)
        if layer.kernel.requires_grad:
            _grouped_bwd_filter(layer, xs, dzs, s, fold)
        return (None, *dxs)


class ConvGroupedChainFn(torch.autograd.Function):
    """ConvChainFn over the pyramid levels: each layer of the chain one grouped
    launch per pass for all levels; the intermediates' ReLU derivatives fused
    into the grouped bwd-data epilogues."""

    @staticmethod
    def forward(ctx, layers, *xs):
        ctx.gsums = [_gsum_register(x) for x in xs]
        ctx.in_acts = [_input_act(x) for x in xs]  # per level (act, producer node)
        xs = [x.contiguous() for x in xs]
        outs = [xs]
        for layer in layers:
            outs.append(_grouped_fwd(layer, outs[-1]))
        ctx.layers = layers
        ctx.n = len(xs)
        ctx.save_for_backward(*[t for lvl in outs for t in lvl])
        return tuple(outs[-1])

    @staticmethod
    def backward(ctx, *dys):
        n, layers = ctx.n, ctx.layers
        saved = ctx.saved_tensors
        acts = [list(saved[i * n:(i + 1) * n]) for i in range(len(layers) + 1)]  # acts[0] = xs
        s = stream_ptr()
        last = len(layers) - 1
        dzs, fold = _grouped_act_grad(layers[last], dys, acts[last + 1], s, node=ctx)
        dxs = [None] * n
        for i in range(last, -1, -1):
            layer, xin = layers[i], acts[i]
            if layer.kernel.requires_grad:
                _grouped_bwd_filter(layer, xin, dzs, s, fold)
            if i == 0:
                if any(ctx.needs_input_grad[1:]):
                    acc = [_gsum_acc(g) for g in ctx.gsums]
                    acc = acc if all(a is not None for a in acc) else None
                    acts = {a for a, _ in ctx.in_acts if a is not None}
                    if len(acts) == 1:  # the levels' producers' ReLU' on each contribution
                        ys = [x if a is not None else None for x, (a, _) in zip(xin, ctx.in_acts)]
                        dxs = _grouped_bwd_data(layer, xin, dzs, s, acc=acc, mask=(acts.pop(), ys))
                        nodes = [node for _, node in ctx.in_acts]
                    else:
                        dxs = _grouped_bwd_data(layer, xin, dzs, s, acc=acc)
                        nodes = [None] * n
                    dxs = [_gsum_done(g, dx, acc is not None, mask_node=nd)
                           for g, dx, nd in zip(ctx.gsums, dxs, nodes)]
                break
            prev = layers[i - 1]
            act = _fusable_act(prev)
            dprev = _grouped_bwd_data(layer, xin, dzs, s, act_in=act)
            if act is not None:
                db = _bias_grad_ptr(prev)
                fold = db is not None and _fold_bias(prev)
                for dp, dz in zip(dprev, dzs):
                    if db is not None and not fold and dz is not None and dp.numel() > 0:
                        bias_grad(dtype_code(dp.dtype), dp.numel() // prev.filters, prev.filters, dp, db, s)
                dzs = [dp if dz is not None else None for dp, dz in zip(dprev, dzs)]
            else:
                dzs, fold = _grouped_act_grad(prev, [dp if dz is not None else None for dp, dz in zip(dprev, dzs)],
                                              xin, s)
        return (None, *dxs)


def bias_grad(dt, rows, c, dy, db, s):
    """db += column sums of dy (act_bwd with act NONE and dz == dy, bit for
    bit); queued inside L.deferred_reductions, so dy is held until its flush."""
    if db is None or rows <= 0:
        return
    L.defer_keep(dy)
    call("fpnmt_bias_grad", dt, rows, c, ptr(dy), db, s)


def act_bwd(dt, rows, c, act, alpha, dy, y, dz, db, s, drop=None):
    """dz = dy * act'(y) [* fused-dropout mask]; db += column sums of dz through
    a per-chunk workspace. drop = (p, seed, seed_tensor) of a fused epilogue."""
    dp, dseed, dst = drop if drop is not None else (0.0, 0, None)
    # ws NULL: the chunk partials go to the fpnmt workspace (or the deferred
    # arena inside L.deferred_reductions)
    call("fpnmt_act_bwd", dt, rows, c, act, alpha, ptr(dy), ptr(y), ptr(dz), db, None, float(dp), dseed,
         ptr(dst), s)


# ------------------------------------------------------ MobileNetV2 pieces
class BatchNormFn(torch.autograd.Function):
    """Keras BatchNormalization in training mode (batch statistics; the moving
    averages move in the same launch sequence) + optional ReLU6 / ReLU and a
    residual add after the normalisation (MobileNetV2's project BN + Add).
    NHWC, channels last; gamma / beta gradients accumulate into the arena."""

    @staticmethod
    def forward(ctx, x, gamma, beta, layer, act, residual):
        x = x.contiguous()
        c = x.shape[-1]
        rows = x.numel() // c if c else 0
        dt = dtype_code(x.dtype)
        s = stream_ptr()
        mean = _empty((c,), torch.float32, x.device)
        var = _empty((c,), torch.float32, x.device)
        group = getattr(layer, "sync_group", None)
        ctx.sync = group is not None
        if ctx.sync:
            # SyncBN: this rank's fp64 sums -> SUM over the ranks -> global stats
            from . import dist as fdist
            sums = _empty((2 * c + 1,), torch.float64, x.device)
            call("fpnmt_bn_stats_sums", dt, rows, c, ptr(x), ptr(sums), s)
            fdist.allreduce_sum_(sums, group)
            call("fpnmt_bn_stats_finalize", c, ptr(sums), ptr(mean), ptr(var), ptr(layer.moving_mean),
                 ptr(layer.moving_variance), float(layer.momentum), stream_ptr())
            ctx.group = group
        else:
            call("fpnmt_bn_stats", dt, rows, c, ptr(x), ptr(mean), ptr(var), ptr(layer.moving_mean),
                 ptr(layer.moving_variance), float(layer.momentum), s)
        if residual is not None:
            residual = residual.contiguous()
        y = torch.empty_like(x)
        call("fpnmt_bn_apply", dt, rows, c, ptr(x), ptr(mean), ptr(var), ptr(gamma), ptr(beta), float(layer.epsilon),
             act, ptr(residual), ptr(y), s)
        ctx.layer, ctx.act, ctx.has_res = layer, act, residual is not None
        ctx.save_for_backward(x, y, mean, var)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, var = ctx.saved_tensors
        layer = ctx.layer
        c = x.shape[-1]
        rows = x.numel() // c if c else 0
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dg = _grad_of(layer.gamma).data_ptr() if layer.gamma.requires_grad else None
        db = _grad_of(layer.beta).data_ptr() if layer.beta.requires_grad else None
        dt = dtype_code(x.dtype)
        if ctx.sync:
            from . import dist as fdist
            sums = _empty((2 * c + 1,), torch.float64, x.device)
            call("fpnmt_bn_bwd_sums", dt, rows, c, ptr(x), ptr(mean), ptr(var), float(layer.epsilon), ctx.act,
                 ptr(y), ptr(dy), ptr(sums), dg, db, stream_ptr())
            fdist.allreduce_sum_(sums, ctx.group)
            # the global row count is read on the device from the all-reduced
            # sums[2c] (the forward's statistics used the same count), so
            # shards of different sizes (a short last batch) normalise alike
            call("fpnmt_bn_bwd_dx", dt, rows, c, ptr(x), ptr(mean), ptr(var), ptr(layer.gamma), float(layer.epsilon),
                 ctx.act, ptr(y), ptr(dy), ptr(sums), ptr(dx), stream_ptr())
        else:
            call("fpnmt_bn_bwd", dt, rows, c, ptr(x), ptr(mean), ptr(var), ptr(layer.gamma),
                 float(layer.epsilon), ctx.act, ptr(y), ptr(dy), ptr(dx), dg, db, stream_ptr())
        return dx, None, None, None, None, (dy if ctx.has_res else None)


def batch_norm_inference(x, layer, act, residual=None):
    """BatchNormalization with the moving statistics (training=False)."""
    x = x.contiguous()
    c = x.shape[-1]
    y = torch.empty_like(x)
    if residual is not None:
        residual = residual.contiguous()
    call("fpnmt_bn_apply", dtype_code(x.dtype), x.numel() // c if c else 0, c, ptr(x), ptr(layer.moving_mean),
         ptr(layer.moving_variance), ptr(layer.gamma), ptr(layer.beta), float(layer.epsilon), act, ptr(residual),
         ptr(y), stream_ptr())
    return y


class DepthwiseConvFn(torch.autograd.Function):
    """DepthwiseConv2D (kh x kw <= 3x3, no bias), NHWC, fp32 (kh, kw, C, 1) master."""

    @staticmethod
    def forward(ctx, x, kernel, layer):
        x = x.contiguous()
        n, h, w, c = x.shape
        pt, pb, pl, pr = layer.pads
        st = layer.stride
        ho = max((h + pt + pb - layer.kh) // st + 1, 0)
        wo = max((w + pl + pr - layer.kw) // st + 1, 0)
        y = _empty((n, ho, wo, c), x.dtype, x.device)
        call("fpnmt_depthwise_fwd", dtype_code(x.dtype), n, h, w, c, layer.kh, layer.kw, st, pt, pb, pl, pr, ptr(x),
             ptr(kernel), ptr(y), stream_ptr())
        ctx.layer = layer
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        layer = ctx.layer
        n, h, w, c = x.shape
        pt, pb, pl, pr = layer.pads
        dy = dy.contiguous()
        s = stream_ptr()
        dt = dtype_code(x.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            call("fpnmt_depthwise_bwd_data", dt, n, h, w, c, layer.kh, layer.kw, layer.stride, pt, pb, pl, pr,
                 ptr(dy), ptr(layer.kernel), ptr(dx), s)
        if layer.kernel.requires_grad:
            gk = _grad_of(layer.kernel)
            _wgrad(lambda: call("fpnmt_depthwise_bwd_filter", dt, n, h, w, c, layer.kh, layer.kw, layer.stride,
                                pt, pb, pl, pr, ptr(x), ptr(dy), ptr(gk), stream_ptr()), x, dy, conv=True)
        return dx, None, None


# ------------------------------------------------ residual-gradient sinks
class _ResSink:
    """Pairs the two consumers of a sublayer input x: a GEMM consumer (Dense /
    grouped projection: dx = dz W^T) and a residual consumer (LayerNorm(a + x)
    or a Dense epilogue's `+ x`). Whichever backward runs first decides: the
    residual consumer's gradient is parked here and added by the GEMM's
    bwd-data epilogue (R operand) if the GEMM has not run yet; otherwise it is
    returned to autograd as usual. Either order gives dx = dz W^T + g_res."""
    __slots__ = ("grad", "gemm_done", "res_claimed")

    def __init__(self):
        self.grad, self.gemm_done, self.res_claimed = None, False, False


def _sink_for_gemm(x):
    import fpnmt
    if not fpnmt.config.fuse_residual_grads or not x.requires_grad:
        return None
    s = _ResSink()
    x.__dict__["_fpnmt_rsink"] = s
    return s


def _sink_for_res(res):
    if res is None:
        return None
    s = res.__dict__.get("_fpnmt_rsink")
    if s is None or s.res_claimed or s.gemm_done:
        return None
    s.res_claimed = True
    return s


def _sink_put(sink, g):
    """Residual consumer's backward: park g for the GEMM (returns None), or
    hand it back to autograd when the GEMM already ran."""
    if sink is None or sink.gemm_done or g is None:
        return g
    sink.grad = g.contiguous()
    return None


def _sink_take(sink):
    """GEMM consumer's backward: the parked residual gradient (or None)."""
    if sink is None:
        return None
    sink.gemm_done = True
    g, sink.grad = sink.grad, None
    return g


class _GradSum:
    """The gradient of a tensor read by n declared GEMM consumers
    (expect_consumers): each consumer's bwd-data launch accumulates into the
    running sum (a read-modify-write epilogue) instead of writing its own dx
    for autograd to add; the last one to run hands the total to autograd and
    the others return None for that input. A consumer registers in its
    forward; while fewer than n registered, nobody parks (plain autograd)."""
    __slots__ = ("n", "reg", "arrived", "grad", "mask_node", "unmasked")

    def __init__(self):
        self.n = self.reg = self.arrived = 0
        self.grad = None
        # every arrival multiplied its contribution by act' of this producer
        # node's output (fuse_input_act): the total is then tagged for it
        self.mask_node, self.unmasked = None, False


def expect_consumers(x, k):
    """Declare k more GEMM consumers of x whose gradients are to be summed in
    their bwd-data epilogues. Model code declares only consumers that are
    always back-propagated together (a parked partial sum is handed on by the
    last one)."""
    import fpnmt
    if not fpnmt.config.fuse_grad_sums or not isinstance(x, torch.Tensor) or not x.requires_grad:
        return
    gs = x.__dict__.get("_fpnmt_gsum")
    if gs is None:
        gs = x.__dict__["_fpnmt_gsum"] = _GradSum()
    gs.n += k


def _gsum_register(x):
    gs = x.__dict__.get("_fpnmt_gsum") if isinstance(x, torch.Tensor) else None
    if gs is None or gs.reg >= gs.n:
        return None
    gs.reg += 1
    return gs


def _gsum_acc(gs):
    """The running sum this consumer's bwd-data accumulates into (None: it
    writes a fresh dx)."""
    if gs is None or gs.reg < gs.n:
        return None
    return gs.grad


def _tag_act_applied(g, node):
    if g is not None and node is not None:
        g._fpnmt_act_applied = (node, g._version)
    return g


def _gsum_done(gs, dx, accumulated, mask_node=None):
    """After a consumer's bwd-data: dx is the new running sum (accumulated
    True) or this consumer's own gradient. Returns what autograd gets.
    mask_node: this consumer multiplied its contribution by act' of that
    node's output; the gradient handed on is tagged for the node when every
    contribution was (the node then skips its act_bwd pass)."""
    if gs is None or gs.reg < gs.n:
        return _tag_act_applied(dx, mask_node)
    gs.arrived += 1
    if mask_node is None or (gs.mask_node is not None and gs.mask_node is not mask_node):
        gs.unmasked = True
    gs.mask_node = mask_node
    if dx is not None:
        if gs.grad is not None and not accumulated:
            dx = dx + gs.grad  # a consumer path without an accumulating epilogue
        gs.grad = dx
    if gs.arrived < gs.n:
        _gsum_open.add(gs)
        return None
    _gsum_open.discard(gs)
    g, gs.grad = gs.grad, None
    node = gs.mask_node if not gs.unmasked else None
    gs.mask_node, gs.unmasked = None, False
    return _tag_act_applied(g, node)


_gsum_open = set()  # running sums some but not all of whose consumers have run


def reset_grad_sums():
    """Forget running sums left open by an earlier backward that stopped
    midway (an exception, or autograd.grad over a subset in a probe / eval):
    TrainEngine calls it at each step's start so check_grad_sums covers only
    the current step's backward, and the parked tensors are released."""
    for gs in _gsum_open:
        gs.grad, gs.arrived, gs.mask_node, gs.unmasked = None, 0, None, False
    _gsum_open.clear()


def check_grad_sums():
    """Raise if a consumer-summed gradient was left parked: some of its
    declared consumers' backwards ran and the rest never did (a pruned
    branch, autograd.grad over a subset of inputs, a frozen head), so the
    input's whole gradient would be dropped silently. TrainEngine runs it
    after the step's last backward (a staged step's stages included)."""
    if _gsum_open:
        bad = [(gs.arrived, gs.n) for gs in _gsum_open]
        _gsum_open.clear()
        raise RuntimeError(f"expect_consumers: {len(bad)} gradient sum(s) incomplete at the end of the backward "
                           f"(arrived / declared: {bad[:4]}); every declared consumer must be back-propagated")



class _DropTok:
    """A Dense's fused dropout (p, seed, seed tensor) handed to the single
    LayerNorm that normalises its output (`LN(res + dropout(dense))`,
    transformer.py:232-242): that LayerNorm's backward writes the Dense's
    masked gradient dz beside dx (fpnmt_layernorm_bwd_drop) and tags dx; the
    Dense's backward uses dz when it receives exactly that dx (same tensor,
    same version) and otherwise runs its own act_bwd on what it got."""
    __slots__ = ("drop", "claimed", "dz")

    def __init__(self, drop):
        self.drop, self.claimed, self.dz = drop, False, None


class _ActTok:
    """The activation of a Dense (ffn1) whose output only feeds the next Dense
    (ffn2; declared by the model: layers.Dense.act_into_next): ffn2's
    bwd-data GEMM applies act'(y1) in its epilogue (fpnmt_gemm_act_in) and
    tags its dx; ffn1's backward then skips its act_bwd pass when it receives
    exactly that tensor (same object, same version)."""
    __slots__ = ("act", "alpha", "claimed")

    def __init__(self, act, alpha):
        self.act, self.alpha, self.claimed = act, alpha, False


def _drop_tok_claim(x):
    t = x.__dict__.get("_fpnmt_drop")
    if t is None or t.claimed:
        return None
    t.claimed = True
    return t


# ------------------------------------------------------------------- dense
def _gemm_desc(m, n, k, dt, lda, ldb, ldc, a_trans=0, b_trans=0, act=0, act_alpha=0.0,
               accumulate=0, c_f32=0, alpha=1.0):
    g = L.GemmDesc()
    g.m, g.n, g.k = m, n, k
    g.batch, g.batch_inner = 1, 1
    g.dtype = dt
    g.a_trans, g.b_trans = a_trans, b_trans
    g.lda, g.ldb, g.ldc, g.ldr = lda, ldb, ldc, ldc
    g.alpha = alpha
    g.act, g.act_alpha = act, act_alpha
    g.accumulate, g.c_f32, g.split_k = accumulate, c_f32, (0 if accumulate == 2 else 1)
    return g


class LinearFn(torch.autograd.Function):
    """y = act(x @ W + b), x (..., in) with unit stride in the last dim."""

    @staticmethod
    def forward(ctx, x, kernel, bias, layer, drop_p=0.0, residual=None):
        """drop_p > 0 / residual: y = residual + dropout(x W + b) in the GEMM
        epilogue (the reference's `out + dropout(mha)` / `dropout(ffn)` pairs)."""
        x0 = x
        if x.stride(-1) != 1 or (x.dim() > 2 and not x.is_contiguous()):
            x = x.contiguous()
        fin, fout = layer.kernel.shape
        lead = x.shape[:-1]
        rows = x.numel() // fin if fin else 0
        lda = x.stride(-2) if x.dim() >= 2 and rows > 1 else fin
        out_dtype = torch.float32 if layer.out_f32 else x.dtype
        y = _empty((*lead, fout), out_dtype, x.device)
        dt = dtype_code(x.dtype)
        wf, _ = layer.compute_weights(x.dtype)
        act = L.ACT_CODES[layer.activation]
        g = _gemm_desc(rows, fout, fin, dt, lda, fin, fout, act=act, act_alpha=layer.act_alpha,
                       c_f32=1 if (layer.out_f32 and x.dtype != torch.float32) else 0)
        ctx.drop = None
        if drop_p > 0.0:
            if act != L.ACT_NONE:
                raise ValueError("fused dropout needs a linear Dense (act' would need the pre-dropout output)")
            seed = runtime.next_seed()
            st = runtime.seed_tensor
            g.drop_p, g.drop_seed, g.drop_seed_dev = float(drop_p), seed, ptr(st)
            ctx.drop = (float(drop_p), seed, st)
        ctx.drop_tok = None
        import fpnmt
        ctx.act_tok = None  # this layer's activation, applied by the next Dense's bwd-data
        if (act in (L.ACT_RELU, L.ACT_RELU6, L.ACT_LEAKY) and getattr(layer, "act_into_next", False)
                and fpnmt.config.fuse_ffn_act and not layer.out_f32):
            ctx.act_tok = _ActTok(act, float(layer.act_alpha))
            y.__dict__["_fpnmt_actsrc"] = ctx.act_tok
        ctx.act_in = None  # the producer's activation, applied in this layer's bwd-data
        t = x0.__dict__.get("_fpnmt_actsrc")
        if t is not None and not t.claimed and x is x0 and residual is None:
            t.claimed = True
            ctx.act_in = t
        if ctx.drop is not None and residual is None and not layer.out_f32 and fpnmt.config.fuse_drop_ln:
            ctx.drop_tok = _DropTok(ctx.drop)
            y.__dict__["_fpnmt_drop"] = ctx.drop_tok
        ctx.rsink_res = None
        if residual is not None:
            if residual.shape != y.shape or residual.dtype != y.dtype:
                raise ValueError("Dense residual must match the output shape / dtype")
            if residual is not x0:
                ctx.rsink_res = _sink_for_res(residual)
            residual = residual.contiguous()
        ctx.rsink_gemm = _sink_for_gemm(x0)
        call("fpnmt_gemm", g, ptr(x), ptr(wf), ptr(y), None, ptr(layer.bias), ptr(residual), stream_ptr())
        ctx.layer = layer
        ctx.lda = lda
        ctx.rows = rows
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        layer = ctx.layer
        fin, fout = layer.kernel.shape
        rows = ctx.rows
        s = stream_ptr()
        cdt = x.dtype
        dt = dtype_code(cdt)
        tok, dz_ln = ctx.drop_tok, None
        if tok is not None:
            tag = dy.__dict__.get("_fpnmt_dropdz")
            if tag is not None and tag[0] is tok and tag[1] == dy._version and tok.dz is not None:
                dz_ln = tok.dz  # the LayerNorm backward already applied the dropout mask
            tok.dz = None
        if ctx.act_tok is not None and dz_ln is None:
            tag = dy.__dict__.get("_fpnmt_actdone")
            if tag is not None and tag[0] is ctx.act_tok and tag[1] == dy._version:
                dz_ln = dy  # the next Dense's bwd-data epilogue already applied act'(y)
        dy = dy.contiguous()
        act = L.ACT_CODES[layer.activation]
        if dy.dtype != cdt:
            dyc = torch.empty(dy.shape, dtype=cdt, device=dy.device)
            call("fpnmt_cast", dtype_code(dy.dtype), dt, dy.numel(), ptr(dy), ptr(dyc), s)
            dy = dyc
            y_for_act = None
        else:
            y_for_act = y
        db = _grad_of(layer.bias).data_ptr() if (layer.bias is not None and layer.bias.requires_grad) else None
        dres = _sink_put(ctx.rsink_res, dy) if ctx.has_res else None
        if dz_ln is not None:
            dz = dz_ln
            bias_grad(dt, rows, fout, dz, db, s)
        elif act != L.ACT_NONE or ctx.drop is not None:
            dz = torch.empty_like(dy)
            act_bwd(dt, rows, fout, act, layer.act_alpha, dy, y_for_act, dz, db, s, drop=ctx.drop)
        else:
            dz = dy
            bias_grad(dt, rows, fout, dy, db, s)
        dx = None
        if ctx.needs_input_grad[0]:
            _, wflip = layer.compute_weights(cdt)
            dx = torch.empty(x.shape, dtype=cdt, device=x.device)
            g = _gemm_desc(rows, fin, fout, dt, fout, layer.flip_ld(), fin)
            r = _sink_take(ctx.rsink_gemm)  # + the residual branch's gradient of x
            if r is not None and (r.dtype != cdt or r.numel() != dx.numel()):
                r = r.to(cdt).reshape(dx.shape).contiguous()
            if ctx.act_in is not None and r is None and ctx.lda == fin:
                # dx * act'(x): the producing Dense's activation backward, x its output
                g.ldr = fin
                call("fpnmt_gemm_act_in", g, ptr(dz), ptr(wflip), ptr(dx), ptr(x), ctx.act_in.act, ctx.act_in.alpha, s)
                dx.__dict__["_fpnmt_actdone"] = (ctx.act_in, dx._version)
            else:
                call("fpnmt_gemm", g, ptr(dz), ptr(wflip), ptr(dx), None, None, ptr(r), s)
        if layer.kernel.requires_grad and rows > 0:
            g = _gemm_desc(fin, fout, rows, dt, ctx.lda, fout, fout, a_trans=1, b_trans=1, accumulate=2, c_f32=1)
            gk = _grad_of(layer.kernel)
            _wgrad(lambda: call("fpnmt_gemm_wgrad", g, ptr(x), ptr(dz), ptr(gk), stream_ptr()), x, dz)
        return dx, None, None, None, None, dres


# ------------------------------------------------------------- pooling
class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, sh, sw, pt, pl, ho, wo):
        x = x.contiguous()
        n, h, w, c = x.shape
        y = _empty((n, ho, wo, c), x.dtype, x.device)
        am = _empty((n, ho, wo, c), torch.uint8, x.device)
        call("fpnmt_maxpool2d_fwd", dtype_code(x.dtype), n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo,
             ptr(x), ptr(y), ptr(am), stream_ptr())
        # x = a conv's ReLU output (the ResNet stem; LeakyReLU under
        # non-overlapping windows): the backward applies that derivative too
        # (fuse_input_act; x is held by the producer's backward anyway)
        ctx.in_act, ctx.in_alpha, ctx.in_prev = _pool_input_act(x, kh <= sh and kw <= sw)
        ctx.save_for_backward(am, x if ctx.in_act is not None else None)
        ctx.shape = (n, h, w, c)
        ctx.xdtype = x.dtype
        ctx.cfg = (kh, kw, sh, sw, pt, pl, ho, wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        am, xa = ctx.saved_tensors
        kh, kw, sh, sw, pt, pl, ho, wo = ctx.cfg
        n, h, w, c = ctx.shape
        dx = _empty((n, h, w, c), ctx.xdtype, dy.device)
        if ctx.in_act is not None:
            call("fpnmt_maxpool2d_bwd_act", dtype_code(ctx.xdtype), n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo,
                 ptr(am), ptr(dy.contiguous()), ptr(xa), ctx.in_act, ctx.in_alpha, ptr(dx), stream_ptr())
            _tag_act_applied(dx, ctx.in_prev)
            if ctx.in_act == L.ACT_LEAKY:
                ctx.in_prev._fpnmt_leaky_folded = True  # _act_applied refuses a summed gradient
        else:
            call("fpnmt_maxpool2d_bwd", dtype_code(ctx.xdtype), n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo,
                 None, ptr(am), ptr(dy.contiguous()), ptr(dx), stream_ptr())
        return dx, None, None, None, None, None, None, None, None


def max_pool2d_valid(x, k=2, s=2):
    """Keras MaxPooling2D() (2x2, stride 2, VALID; 1x1 -> 0x0 is legal)."""
    n, h, w, c = x.shape
    ho = max((h - k) // s + 1, 0)
    wo = max((w - k) // s + 1, 0)
    return MaxPoolFn.apply(x, k, k, s, s, 0, 0, ho, wo)


def max_pool2d_same(x, k=3, s=2):
    """Keras MaxPooling2D(k, s, padding='same'): pad total = max((ceil(h/s)-1)*s+k-h, 0),
    split floor/ceil (before/after), padded taps never win."""
    n, h, w, c = x.shape
    ho, wo = -(-h // s), -(-w // s)
    pth = max((ho - 1) * s + k - h, 0)
    ptw = max((wo - 1) * s + k - w, 0)
    return MaxPoolFn.apply(x, k, k, s, s, pth // 2, ptw // 2, ho, wo)


# ----------------------------------------------------------- FPN top-down
class FpnTopDownFn(torch.autograd.Function):
    """(lat5, lat4, lat3) -> (P4_merged, P3_merged) in one sweep
    (retinanet.py:119,123-125,129-130)."""

    @staticmethod
    def forward(ctx, lat5, lat4, lat3):
        ctx.gsum = _gsum_register(lat5)
        lat5, lat4, lat3 = lat5.contiguous(), lat4.contiguous(), lat3.contiguous()
        n, h5, w5, c = lat5.shape
        _, h4, w4, _ = lat4.shape
        _, h3, w3, _ = lat3.shape
        p4m = torch.empty_like(lat4)
        p3m = torch.empty_like(lat3)
        call("fpnmt_fpn_topdown_fwd", dtype_code(lat4.dtype), n, c, h5, w5, h4, w4, h3, w3,
             ptr(lat5), ptr(lat4), ptr(lat3), ptr(p4m), ptr(p3m), stream_ptr())
        ctx.shapes = (n, c, h5, w5, h4, w4, h3, w3)
        ctx.dt = lat4.dtype
        return p4m, p3m

    @staticmethod
    def backward(ctx, dp4m, dp3m):
        n, c, h5, w5, h4, w4, h3, w3 = ctx.shapes
        dev = dp4m.device if dp4m is not None else dp3m.device
        if dp4m is None:
            dp4m = torch.zeros((n, h4, w4, c), dtype=ctx.dt, device=dev)
        if dp3m is None:
            dp3m = torch.zeros((n, h3, w3, c), dtype=ctx.dt, device=dev)
        dp4m, dp3m = dp4m.contiguous(), dp3m.contiguous()
        dl4 = torch.empty_like(dp4m)
        acc = _gsum_acc(ctx.gsum)
        dl5 = acc if acc is not None else torch.empty((n, h5, w5, c), dtype=ctx.dt, device=dev)
        call("fpnmt_fpn_topdown_bwd", dtype_code(ctx.dt), n, c, h5, w5, h4, w4, h3, w3,
             ptr(dp4m), ptr(dp3m), ptr(dl4), ptr(dl5), 1 if acc is not None else 0, stream_ptr())
        return _gsum_done(ctx.gsum, dl5, True), dl4, dp3m


class UpsampleFn(torch.autograd.Function):
    """Nearest resize of source (n,h,w,c) to (ht, wt) — the FPN kernel with a
    zero lateral (layers/_misc.py:39-42)."""

    @staticmethod
    def forward(ctx, src, ht, wt):
        src = src.contiguous()
        n, h, w, c = src.shape
        zero = torch.zeros((n, ht, wt, c), dtype=src.dtype, device=src.device)
        out = torch.empty_like(zero)
        call("fpnmt_fpn_topdown_fwd", dtype_code(src.dtype), n, c, h, w, ht, wt, 0, 0,
             ptr(src), ptr(zero), None, ptr(out), None, stream_ptr())
        ctx.shapes = (n, c, h, w, ht, wt)
        ctx.dt = src.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        n, c, h, w, ht, wt = ctx.shapes
        dout = dout.contiguous()
        dl4 = torch.empty_like(dout)
        dsrc = torch.empty((n, h, w, c), dtype=ctx.dt, device=dout.device)
        call("fpnmt_fpn_topdown_bwd", dtype_code(ctx.dt), n, c, h, w, ht, wt, 0, 0,
             ptr(dout), None, ptr(dl4), ptr(dsrc), 0, stream_ptr())
        return dsrc, None, None


# ------------------------------------------------------ spatial softmax
class SpatialSoftmaxFn(torch.autograd.Function):
    """CoAttention_CNN.call (coattention.py:13-32): softmax of score over h*w,
    times hs broadcast over channels."""

    @staticmethod
    def forward(ctx, score, hs):
        score, hs = score.contiguous(), hs.contiguous()
        n, h, w, c = hs.shape
        ctx_out = torch.empty_like(hs)
        a = torch.empty((n, h * w), dtype=torch.float32, device=hs.device)
        call("fpnmt_spatial_softmax_fwd", dtype_code(hs.dtype), n, h * w, c, ptr(score), ptr(hs),
             ptr(ctx_out), ptr(a), stream_ptr())
        ctx.save_for_backward(a, hs)
        ctx.score_shape = score.shape
        return ctx_out

    @staticmethod
    def backward(ctx, dctx):
        a, hs = ctx.saved_tensors
        n, h, w, c = hs.shape
        dscore = torch.empty(ctx.score_shape, dtype=hs.dtype, device=hs.device)
        dhs = torch.empty_like(hs)
        ws = torch.empty((n * h * w,), dtype=torch.float64, device=hs.device)
        call("fpnmt_spatial_softmax_bwd", dtype_code(hs.dtype), n, h * w, c, ptr(a), ptr(hs),
             ptr(dctx.contiguous()), ptr(dscore), ptr(dhs), ptr(ws), stream_ptr())
        return dscore, dhs


# --------------------------------------------------------------- attention
def _ldw(lk):
    return max(8, (lk + 7) // 8 * 8)


def _row_ld(t):
    """Row stride of a (B, L, HD) tensor whose rows (b, i) sit at b*L + i rows
    of a 2-D (rows, ld) layout."""
    B, Lt, HD = t.shape
    if Lt > 1:
        return t.stride(1)
    if B > 1:
        return t.stride(0)
    return HD


def _rows_view(t):
    """t itself if its rows are uniformly strided with unit inner stride, else a
    dense copy."""
    B, Lt, HD = t.shape
    if t.stride(-1) == 1 and (B <= 1 or Lt <= 1 or t.stride(0) == Lt * t.stride(1)):
        return t
    return t.contiguous()


def _attn_prep(q, k, v, mask, num_heads, scale, out=None):
    """Descriptor and buffers of one fpnmt_attention_fwd on (B, L, H*D)
    projections (heads by column offset). out: a (B, Lq, H*D) destination
    whose rows may sit in a wider buffer (uniform row stride), else a fresh
    tensor. Returns (desc, q, k, v, mask_ptr, out, wbuf, ws, mask_keep, slots)."""
    slots = [_slot_of(t) for t in (q, k, v)]
    slots = [sl if sl is not None and sl[0].claim(sl[1]) else None for sl in slots]
    q, k, v = [_rows_view(t) for t in (q, k, v)]
    B, Lq, HD = q.shape
    Lk = k.shape[1]
    D = HD // num_heads
    d = L.AttnDesc()
    d.b, d.h, d.lq, d.lk, d.d = B, num_heads, Lq, Lk, D
    d.dtype = dtype_code(q.dtype)
    d.ldq, d.ldk, d.ldv = _row_ld(q), _row_ld(k), _row_ld(v)
    d.ldw = _ldw(Lk)
    d.scale = scale
    mptr, mask_keep = None, None
    if mask is not None:
        m4 = mask.to(dtype=torch.float32)
        while m4.dim() < 4:
            m4 = m4.unsqueeze(0)
        m4 = torch.broadcast_to(m4, (B, num_heads, Lq, Lk))
        d.m_sb, d.m_sh, d.m_si, d.m_sj = m4.stride()
        mptr = m4.data_ptr()
        mask_keep = m4
    if out is None:
        out = _empty((B, Lq, HD), q.dtype, q.device)
    d.ldo = _row_ld(out)
    wbuf = _empty((B, num_heads, Lq, d.ldw), q.dtype, q.device)
    ws = _empty((L.lib.fpnmt_attention_ws_bytes(d),), torch.uint8, q.device)
    return d, q, k, v, mptr, out, wbuf, ws, mask_keep, slots


def _attn_fwd(q, k, v, mask, num_heads, scale, out=None):
    """fpnmt_attention_fwd (see _attn_prep). Returns (out, state) with state =
    (desc, q, k, v, wbuf, mask_keep, slots) for _attn_bwd."""
    d, q, k, v, mptr, out, wbuf, ws, mask_keep, slots = _attn_prep(q, k, v, mask, num_heads, scale, out)
    call("fpnmt_attention_fwd", d, ptr(q), ptr(k), ptr(v), mptr, ptr(out), ptr(wbuf), ptr(ws), stream_ptr())
    return out, (d, q, k, v, wbuf, mask_keep, slots)


def _ptr_table(xs):
    import ctypes
    return (ctypes.c_void_p * len(xs))(*[x if isinstance(x, int) or x is None else ptr(x) for x in xs])


def _attn_fwd_views(qkvs, mask, num_heads, scale, outs):
    """The views' attentions [(q, k, v)] into outs[i] as ONE
    fpnmt_attention_fwd_views call (one launch when the views qualify).
    Returns the per-view states of _attn_fwd."""
    pr = [_attn_prep(q, k, v, mask, num_heads, scale, o) for (q, k, v), o in zip(qkvs, outs)]
    n = len(pr)
    descs = (L.AttnDesc * n)(*[p[0] for p in pr])
    call("fpnmt_attention_fwd_views", n, descs, *[_ptr_table([p[j] for p in pr]) for j in (1, 2, 3, 4, 5, 6, 7)],
         stream_ptr())
    return [(p[0], p[1], p[2], p[3], p[6], p[8], p[9]) for p in pr]


def _attn_bwd_prep(d, q, k, v, wbuf, slots, dout):
    """Descriptor and buffers of one fpnmt_attention_bwd: each of q / k / v
    that came from a ProjectionGroupFn is read in place and its gradient
    written into the group's gradient buffer (same row stride); otherwise a
    dense gradient. dout: (B, Lq, H*D), rows uniformly strided (may sit in a
    wider buffer). Returns (desc, ins, grads, dout, ws)."""
    dout = _rows_view(dout)
    bd = L.AttnDesc.from_buffer_copy(d)
    bd.ldo = _row_ld(dout)
    ins, grads, lds = [], [], []
    for t, slot in zip((q, k, v), slots):
        if slot is not None and _row_ld(slot[0].view(slot[1], t.shape)) == _row_ld(t):
            ins.append(t)
            grads.append(slot[0].view(slot[1], t.shape))
            lds.append(_row_ld(t))
        else:
            tc = t if t.is_contiguous() else t.contiguous()
            ins.append(tc)
            grads.append(torch.empty(t.shape, dtype=t.dtype, device=t.device))
            lds.append(t.shape[-1])
    bd.ldq, bd.ldk, bd.ldv = lds
    ws = _empty((L.lib.fpnmt_attention_ws_bytes(bd),), torch.uint8, q.device)
    return bd, ins, grads, dout, ws


def _attn_bwd(d, q, k, v, wbuf, slots, dout):
    """fpnmt_attention_bwd: (dq, dk, dv) (see _attn_bwd_prep)."""
    bd, ins, grads, dout, ws = _attn_bwd_prep(d, q, k, v, wbuf, slots, dout)
    call("fpnmt_attention_bwd", bd, ptr(ins[0]), ptr(ins[1]), ptr(ins[2]), ptr(wbuf), ptr(dout),
         ptr(grads[0]), ptr(grads[1]), ptr(grads[2]), ptr(ws), stream_ptr())
    return grads


def _attn_bwd_views(states, douts):
    """The views' attention backwards as ONE fpnmt_attention_bwd_views call;
    states: [(desc, q, k, v, wbuf, slots)]. Returns [dq, dk, dv] per view,
    flattened."""
    pr = [_attn_bwd_prep(d, q, k, v, wbuf, slots, do) for (d, q, k, v, wbuf, slots), do in zip(states, douts)]
    n = len(pr)
    descs = (L.AttnDesc * n)(*[p[0] for p in pr])
    tabs = [_ptr_table([p[1][j] for p in pr]) for j in range(3)]
    tabs.append(_ptr_table([st[4] for st in states]))
    tabs.append(_ptr_table([p[3] for p in pr]))
    tabs += [_ptr_table([p[2][j] for p in pr]) for j in range(3)]
    tabs.append(_ptr_table([p[4] for p in pr]))
    call("fpnmt_attention_bwd_views", n, descs, *tabs, stream_ptr())
    return [g for p in pr for g in p[2]]


class AttentionFn(torch.autograd.Function):
    """scaled_dot_product_attention (transformer.py:70-104) on (B, L, H*D)
    projections, heads addressed by column offset (no split/merge copies)."""

    @staticmethod
    def forward(ctx, q, k, v, mask, num_heads, scale):
        out, (d, qc, kc, vc, wbuf, mask_keep, slots) = _attn_fwd(q, k, v, mask, num_heads, scale)
        ctx.desc, ctx.slots, ctx.mask_keep = d, slots, mask_keep
        ctx.set_materialize_grads(False)  # the weights output never gets a gradient: no zero fill
        ctx.save_for_backward(qc, kc, vc, wbuf)
        weights = wbuf[..., :k.shape[1]]
        ctx.mark_non_differentiable(weights)
        return out, weights

    @staticmethod
    def backward(ctx, dout, _dw):
        q, k, v, wbuf = ctx.saved_tensors
        if dout is None:
            return None, None, None, None, None, None
        dq, dk, dv = _attn_bwd(ctx.desc, q, k, v, wbuf, ctx.slots, dout)
        return dq, dk, dv, None, None, None


class MultiViewAttnProjFn(torch.autograd.Function):
    """EncoderLayer's view loop (transformer.py:184-190):
        out = baseline + sum_i Dropout(MHA_i(v = k = view_i, q = baseline))
    as ONE autograd node over the NUM_OF_PYRAMIDS - 1 views: every view's
    attention writes its output side by side into one (rows, nseg*d) buffer,
    then ONE launch applies the views' output Dense layers, biases, dropout
    masks and the residual sum (fpnmt_view_proj_fwd). Backward: one launch for
    the masked per-view gradients and bias sums (fpnmt_view_proj_bwd_dz), one
    batched bwd-data GEMM, one batched bwd-filter GEMM into the group's
    contiguous gradients, then the views' attention backwards (their q / k / v
    gradients straight into the grouped projections' buffers). The baseline's
    residual gradient is handed to the baseline's query-projection GEMM when
    that runs later (the _ResSink pairing), else returned."""

    @staticmethod
    def forward(ctx, baseline, group, drop_p, num_heads, scale, mask, *qkv):
        nseg, fin, fout = group.n, group.fin, group.fout
        if len(qkv) != 3 * nseg:
            raise ValueError("MultiViewAttnProjFn: one (q, k, v) per view")
        B, Lq, HD = qkv[0].shape
        if HD != fin or baseline.shape[-1] != fout:
            raise ValueError("MultiViewAttnProjFn: view width / output width mismatch")
        rows = B * Lq
        cdt = baseline.dtype
        dt = dtype_code(cdt)
        dev = baseline.device
        O = _empty((rows, nseg * fin), cdt, dev)
        outs = [O[:, i * fin:(i + 1) * fin].view(B, Lq, fin) for i in range(nseg)]
        states = _attn_fwd_views([qkv[3 * i:3 * i + 3] for i in range(nseg)], mask, num_heads, scale, outs)
        stack, _ = group.stacked(cdt)
        bias = group.bias_cat()
        seed, st_dev = 0, None
        if drop_p > 0.0:
            seed = runtime.next_seed()
            st_dev = runtime.seed_tensor
        res = baseline.contiguous()
        ctx.rsink_res = _sink_for_res(baseline)
        y = _empty(tuple(baseline.shape), cdt, dev)
        call("fpnmt_view_proj_fwd", dt, rows, fout, fin, nseg, ptr(O), nseg * fin, ptr(stack), ptr(bias), ptr(res),
             fout, ptr(y), fout, float(drop_p), seed, ptr(st_dev), stream_ptr())
        ctx.group, ctx.drop = group, (float(drop_p), seed, st_dev)
        ctx.descs = [st[0] for st in states]
        ctx.slots = [st[6] for st in states]
        ctx.mask_keep = [st[5] for st in states]
        ctx.view_shape = (B, Lq, fin)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(O, *[t for st in states for t in (st[1], st[2], st[3], st[4])])
        return y

    @staticmethod
    def backward(ctx, dy):
        O, *saved = ctx.saved_tensors
        group = ctx.group
        nseg, fin, fout = group.n, group.fin, group.fout
        if dy is None:
            return (None,) * (6 + 3 * nseg)
        cdt = O.dtype
        dt = dtype_code(cdt)
        s = stream_ptr()
        rows = O.shape[0]
        dy = dy.contiguous()
        if dy.dtype != cdt:
            dyc = torch.empty(dy.shape, dtype=cdt, device=dy.device)
            call("fpnmt_cast", dtype_code(dy.dtype), dt, dy.numel(), ptr(dy), ptr(dyc), s)
            dy = dyc
        p, seed, st_dev = ctx.drop
        kg, bg = group.grad_views()
        dz = _empty((rows, nseg * fout), cdt, O.device)
        tmp = None
        if bg is None:
            tmp = torch.zeros(nseg * fout, dtype=torch.float32, device=O.device)
        call("fpnmt_view_proj_bwd_dz", dt, rows, fout, nseg, ptr(dy), fout, ptr(dz),
             (bg if bg is not None else tmp).data_ptr(), p, seed, ptr(st_dev), s)
        if tmp is not None:
            for i, m in enumerate(group.layers):
                _grad_of(m.bias).add_(tmp[i * fout:(i + 1) * fout])
        # the views' attention-output gradients: dO_i = dz_i W_i^T, one batched launch
        _, flip = group.stacked(cdt)
        dO = _empty((rows, nseg * fin), cdt, O.device)
        g = _gemm_desc(rows, fin, fout, dt, nseg * fout, nseg * fout, nseg * fin)
        g.batch = nseg
        g.a_so, g.b_so, g.c_so = fout, fout, fin
        call("fpnmt_gemm", g, ptr(dz), ptr(flip), ptr(dO), None, None, None, s)
        # the views' output-kernel gradients: dW_i += O_i^T dz_i
        if kg is not None:
            g = _gemm_desc(fin, fout, rows, dt, nseg * fin, nseg * fout, fout, a_trans=1, b_trans=1,
                           accumulate=2, c_f32=1)
            g.batch = nseg
            g.a_so, g.b_so, g.c_so = fin, fout, fin * fout
            _wgrad(lambda: call("fpnmt_gemm_wgrad", g, ptr(O), ptr(dz), ptr(kg), stream_ptr()), O, dz)
        else:
            for i, m in enumerate(group.layers):
                g = _gemm_desc(fin, fout, rows, dt, nseg * fin, nseg * fout, fout, a_trans=1, b_trans=1,
                               accumulate=2, c_f32=1)
                gk = _grad_of(m.kernel)
                _wgrad(lambda g=g, i=i, gk=gk: call("fpnmt_gemm_wgrad", g, O[:, i * fin:].data_ptr(),
                                                    dz[:, i * fout:].data_ptr(), ptr(gk),
                                                    stream_ptr()), O, dz)
        B, Lq, _ = ctx.view_shape
        grads = _attn_bwd_views([(ctx.descs[i], *saved[4 * i:4 * i + 4], ctx.slots[i]) for i in range(nseg)],
                                [dO[:, i * fin:(i + 1) * fin].view(B, Lq, fin) for i in range(nseg)])
        dres = _sink_put(ctx.rsink_res, dy)
        return (dres, None, None, None, None, None, *grads)


# ----------------------------------------------------- grouped projections
class _GradSlot:
    """Gradient buffer shared by the outputs of one ProjectionGroupFn: the
    consumers (AttentionFn) write their input gradients straight into their
    column range, so the group's backward finds the concatenated gradient
    already assembled (no per-slice zero-fill / copy / add)."""

    def __init__(self, rows, cols, dtype, device):
        self.rows, self.cols, self.dtype, self.device = rows, cols, dtype, device
        self.buf = None
        self.claimed = set()

    def claim(self, off):
        """One writer per column range (a second consumer of the same output
        falls back to a dense gradient that autograd then sums)."""
        if off in self.claimed:
            return False
        self.claimed.add(off)
        return True

    def get(self):
        if self.buf is None:
            self.buf = torch.empty((self.rows, self.cols), dtype=self.dtype, device=self.device)
        return self.buf

    def view(self, off, shape):
        w = shape[-1]
        return self.get()[:, off:off + w].view(shape)


def _slot_of(t):
    s = t.__dict__.get("_fpnmt_gslot") if hasattr(t, "__dict__") else None
    return s


class ProjectionGroupFn(torch.autograd.Function):
    """layers.DenseGroup: y_i = x W_i + b_i for every member as ONE GEMM into
    a (rows, n*out) buffer; returns the n column slices."""

    @staticmethod
    def forward(ctx, x, group, _anchor):
        fin, fout, n = group.fin, group.fout, group.n
        ctx.rsink_gemm = _sink_for_gemm(x)
        if x.stride(-1) != 1 or not x.is_contiguous():
            x = x.contiguous()
        lead = x.shape[:-1]
        rows = x.numel() // fin if fin else 0
        x2 = x.view(rows, fin)
        cdt = x.dtype
        dt = dtype_code(cdt)
        y = _empty((rows, n * fout), cdt, x.device)
        stack, _ = group.stacked(cdt)
        bias = group.bias_cat()
        g = _gemm_desc(rows, n * fout, fin, dt, fin, fin, n * fout)
        call("fpnmt_gemm", g, ptr(x2), ptr(stack), ptr(y), None, ptr(bias), None, stream_ptr())
        slot = _GradSlot(rows, n * fout, cdt, x.device)
        outs = []
        for i in range(n):
            o = y[:, i * fout:(i + 1) * fout].view(*lead, fout)
            o.__dict__["_fpnmt_gslot"] = (slot, i * fout)
            outs.append(o)
        ctx.group, ctx.slot, ctx.rows = group, slot, rows
        ctx.in_shape = x.shape
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x2)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        (x2,) = ctx.saved_tensors
        group, slot, rows = ctx.group, ctx.slot, ctx.rows
        fin, fout, n = group.fin, group.fout, group.n
        cdt = x2.dtype
        dt = dtype_code(cdt)
        s = stream_ptr()
        buf = slot.get()
        for i, gi in enumerate(gs):
            dst = buf[:, i * fout:(i + 1) * fout]
            if gi is None:
                dst.zero_()
            elif not (gi.data_ptr() == dst.data_ptr() and gi.dim() >= 2 and gi.stride(-1) == 1 and
                      (rows <= 1 or gi.reshape(-1, fout).stride(0) == n * fout)):
                dst.copy_(gi.reshape(rows, fout))
        kg, bg = group.grad_views()
        # bias gradients: column sums of the concatenated gradient
        if bg is not None:
            bias_grad(dt, rows, n * fout, buf, bg.data_ptr(), s)
        else:
            tmp = torch.zeros(n * fout, dtype=torch.float32, device=buf.device)
            act_bwd(dt, rows, n * fout, L.ACT_NONE, 0.0, buf, None, buf, tmp.data_ptr(), s)
            for i, m in enumerate(group.layers):
                _grad_of(m.bias).add_(tmp[i * fout:(i + 1) * fout])
        dx = None
        if ctx.needs_input_grad[0]:
            _, flip = group.stacked(cdt)
            dx = _empty((rows, fin), cdt, buf.device)
            # dx = dY @ [W_1 .. W_n]^T: the interleaved flipped copy (in, n*out) is B (n, k)
            g = _gemm_desc(rows, fin, n * fout, dt, n * fout, n * fout, fin)
            r = _sink_take(ctx.rsink_gemm)  # + the residual branch's gradient of x
            if r is not None and (r.dtype != cdt or r.numel() != dx.numel()):
                r = r.to(cdt).reshape(dx.shape).contiguous()
            call("fpnmt_gemm", g, ptr(buf), ptr(flip), ptr(dx), None, None, ptr(r), s)
            dx = dx.view(ctx.in_shape)
        if rows > 0:
            if kg is not None:  # one batched launch: dW_i = x^T dY_i
                g = _gemm_desc(fin, fout, rows, dt, fin, n * fout, fout, a_trans=1, b_trans=1,
                               accumulate=2, c_f32=1)
                g.batch = n
                g.a_so, g.b_so, g.c_so = 0, fout, fin * fout
                _wgrad(lambda: call("fpnmt_gemm_wgrad", g, ptr(x2), ptr(buf), ptr(kg), stream_ptr()),
                       x2, buf)
            else:
                for i, m in enumerate(group.layers):
                    g = _gemm_desc(fin, fout, rows, dt, fin, n * fout, fout, a_trans=1, b_trans=1,
                                   accumulate=2, c_f32=1)
                    gk = _grad_of(m.kernel)
                    _wgrad(lambda g=g, i=i, gk=gk: call("fpnmt_gemm_wgrad", g, ptr(x2), buf[:, i * fout:].data_ptr(),
                                                        ptr(gk), stream_ptr()), x2, buf)
        return dx, None, None


# --------------------------------------------------------------- layernorm
class LayerNormFn(torch.autograd.Function):
    """LayerNormalization(epsilon) over the last axis of (x [+ res]); optional
    positional-encoding add after the norm (Encoder, transformer.py:290-292)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, pe, eps, layer):
        ctx.rsink_res = _sink_for_res(res) if res is not x else None
        ctx.drop_tok = _drop_tok_claim(x)
        x = x.contiguous()
        d = x.shape[-1]
        rows = x.numel() // d if d else 0
        if res is not None:
            res = res.contiguous()
        y = torch.empty_like(x)
        mean = _empty((max(rows, 1),), torch.float32, x.device)
        rstd = _empty((max(rows, 1),), torch.float32, x.device)
        pe_rows = 0
        if pe is not None:
            pe_rows = x.shape[-2]
        call("fpnmt_layernorm_fwd", dtype_code(x.dtype), rows, d, eps, ptr(x), ptr(res), ptr(gamma),
             ptr(beta), ptr(pe), pe_rows, ptr(y), ptr(mean), ptr(rstd), stream_ptr())
        ctx.layer = layer
        ctx.has_res = res is not None
        ctx.save_for_backward(x, res if res is not None else x, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, mean, rstd = ctx.saved_tensors
        layer = ctx.layer
        d = x.shape[-1]
        rows = x.numel() // d if d else 0
        dx = torch.empty_like(x)
        tok = ctx.drop_tok
        if tok is None:
            call("fpnmt_layernorm_bwd", dtype_code(x.dtype), rows, d, ptr(x), ptr(res) if ctx.has_res else None,
                 ptr(layer.gamma), ptr(mean), ptr(rstd), ptr(dy.contiguous()), ptr(dx),
                 ptr(_grad_of(layer.gamma)), ptr(_grad_of(layer.beta)), stream_ptr())
        else:
            p, seed, st = tok.drop
            dz = torch.empty_like(x)
            call("fpnmt_layernorm_bwd_drop", dtype_code(x.dtype), rows, d, ptr(x),
                 ptr(res) if ctx.has_res else None, ptr(layer.gamma), ptr(mean), ptr(rstd), ptr(dy.contiguous()),
                 ptr(dx), ptr(_grad_of(layer.gamma)), ptr(_grad_of(layer.beta)), p, seed, ptr(st), ptr(dz),
                 stream_ptr())
            tok.dz = dz
            dx.__dict__["_fpnmt_dropdz"] = (tok, dx._version)
        return dx, None, None, (_sink_put(ctx.rsink_res, dx) if ctx.has_res else None), None, None, None


class LayerNormViewsFn(torch.autograd.Function):
    """The Encoder's per-view input normalisation (transformer.py:279-292:
    the shared LayerNormalization, + pe[:L_i], Dropout) for all views as ONE
    launch per pass (fpnmt_layernorm_views_fwd / _bwd); the same rows, masks
    (seeds drawn in view order) and per-view gamma / beta sums as one
    LayerNormFn + DropoutFn per view."""

    @staticmethod
    def forward(ctx, layer, pe, drop_p, *xs):
        xs = [x.contiguous() for x in xs]
        n, d = len(xs), xs[0].shape[-1]
        tab = (L.LnView * n)()
        ys, stats, seeds = [], [], []
        for i, x in enumerate(xs):
            rows = x.numel() // d if d else 0
            y = torch.empty_like(x)
            mean = _empty((max(rows, 1),), torch.float32, x.device)
            rstd = _empty((max(rows, 1),), torch.float32, x.device)
            seed = runtime.next_seed() if drop_p > 0.0 and rows > 0 else 0
            tab[i].x, tab[i].y, tab[i].mean, tab[i].rstd = ptr(x), ptr(y), ptr(mean), ptr(rstd)
            tab[i].rows, tab[i].pe_rows, tab[i].seed = rows, (x.shape[-2] if pe is not None else 0), seed
            ys.append(y)
            stats += [mean, rstd]
            seeds.append(seed)
        st = runtime.seed_tensor if drop_p > 0.0 else None
        call("fpnmt_layernorm_views_fwd", dtype_code(xs[0].dtype), n, d, float(layer.epsilon), tab, ptr(layer.gamma),
             ptr(layer.beta), ptr(pe), float(drop_p), ptr(st), stream_ptr())
        ctx.layer, ctx.p, ctx.st, ctx.seeds, ctx.n = layer, float(drop_p), st, seeds, n
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(*xs, *stats)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        n = ctx.n
        saved = ctx.saved_tensors
        xs, stats = saved[:n], saved[n:]
        layer = ctx.layer
        d = xs[0].shape[-1]
        tab = (L.LnView * n)()
        dxs, keep = [], []
        for i, (x, dy) in enumerate(zip(xs, dys)):
            if dy is None or x.numel() == 0:
                dxs.append(None)
                continue
            dy = dy.contiguous()
            dx = torch.empty_like(x)
            tab[i].x, tab[i].y, tab[i].dy = ptr(x), ptr(dx), ptr(dy)
            tab[i].mean, tab[i].rstd = ptr(stats[2 * i]), ptr(stats[2 * i + 1])
            tab[i].rows, tab[i].seed = x.numel() // d, ctx.seeds[i]
            dxs.append(dx)
            keep.append(dy)
        call("fpnmt_layernorm_views_bwd", dtype_code(xs[0].dtype), n, d, tab, ptr(layer.gamma), ctx.p, ptr(ctx.st),
             ptr(_grad_of(layer.gamma)), ptr(_grad_of(layer.beta)), stream_ptr())
        return (None, None, None, *dxs)


# --------------------------------------------------------------- embedding
class EmbedPosencFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tok, emb, pe, dtype, layer, sumsq_slot, drop_p=0.0):
        """drop_p > 0: the decoder's Dropout after the embedding (transformer.py:
        331) in the same launch (fpnmt_embed_posenc_fwd_drop)."""
        tok = tok.to(torch.int32).contiguous()
        b, t = tok.shape
        d = emb.shape[1]
        y = _empty((b, t, d), dtype, emb.device)
        ctx.drop = None
        if drop_p > 0.0 and y.numel() > 0:
            ctx.drop = (float(drop_p), runtime.next_seed(), runtime.seed_tensor)
            p, seed, st = ctx.drop
            call("fpnmt_embed_posenc_fwd_drop", dtype_code(dtype), b, t, d, ptr(tok), ptr(emb), ptr(pe), ptr(y), p,
                 seed, ptr(st), stream_ptr())
        else:
            call("fpnmt_embed_posenc_fwd", dtype_code(dtype), b, t, d, ptr(tok), ptr(emb), ptr(pe), ptr(y),
                 stream_ptr())
        ctx.save_for_backward(tok)
        ctx.layer = layer
        ctx.sumsq = sumsq_slot
        ctx.dt = dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (tok,) = ctx.saved_tensors
        b, t = tok.shape
        emb = ctx.layer.embeddings
        if ctx.drop is not None:
            p, seed, st = ctx.drop
            call("fpnmt_embed_posenc_bwd_drop", dtype_code(ctx.dt), b, t, emb.shape[1], ptr(tok),
                 ptr(dy.contiguous()), ptr(_grad_of(emb)), ptr(ctx.sumsq), p, seed, ptr(st), stream_ptr())
        else:
            call("fpnmt_embed_posenc_bwd", dtype_code(ctx.dt), b, t, emb.shape[1], ptr(tok), ptr(dy.contiguous()),
                 ptr(_grad_of(emb)), ptr(ctx.sumsq), stream_ptr())
        return None, None, None, None, None, None, None


# ----------------------------------------------------------- step targets
def decoder_targets(tok):
    """(tar_inp, tar_real, mask) of a training step (utils/pipeline.py:66-69:
    tok[:, :-1], tok[:, 1:], create_masks(tar_inp)) from the padded (b, T)
    captions in one launch (fpnmt_decoder_targets); the ids as int32
    (what the embedding and loss kernels read), the mask (b, 1, T-1, T-1)
    fp32 = max(padding, look-ahead). int64 or int32 captions."""
    if tok.dtype not in (torch.int64, torch.int32) or tok.dim() != 2 or tok.stride(1) != 1 or not tok.is_cuda:
        tin, tout = tok[:, :-1], tok[:, 1:]
        t = tin.shape[1]
        la = 1.0 - torch.tril(torch.ones((t, t), device=tok.device))
        return tin, tout, torch.maximum((tin == 0).to(torch.float32)[:, None, None, :], la)
    b, T = tok.shape
    t = T - 1
    tin = _empty((b, t), torch.int32, tok.device)
    tout = _empty((b, t), torch.int32, tok.device)
    mask = _empty((b, 1, t, t), torch.float32, tok.device)
    call("fpnmt_decoder_targets", b, T, ptr(tok), tok.element_size(), tok.stride(0), ptr(tin), ptr(tout), ptr(mask),
         stream_ptr())
    return tin, tout, mask


# ------------------------------------------------------------------- loss
class MaskedXentFn(torch.autograd.Function):
    """Pipeline.loss (utils/pipeline.py:50-57): sparse CE from logits times
    (label != 0), mean over ALL B*T positions. Gradient computed in the same
    kernel (saved) — the loss must be the root of backward."""

    @staticmethod
    def forward(ctx, logits, labels):
        v = logits.shape[-1]
        lg = logits.reshape(-1, v)
        if lg.dtype != torch.float32:
            raise TypeError("MaskedXentFn expects fp32 logits")
        lg = lg.contiguous()
        lab = labels.reshape(-1).to(torch.int32).contiguous()
        rows = lg.shape[0]
        loss = torch.empty((1,), dtype=torch.float32, device=lg.device)
        dlog = torch.empty_like(lg)
        call("fpnmt_xent_fwd_bwd", L.F32, rows, v, ptr(lg), v, ptr(lab), ptr(loss), ptr(dlog), v, 1.0,
             stream_ptr())
        ctx.save_for_backward(dlog)
        ctx.shape = logits.shape
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        (dlog,) = ctx.saved_tensors
        return dlog.reshape(ctx.shape), None


# ------------------------------------------------------------ elementwise
class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        x = x.contiguous()
        seed = runtime.next_seed()
        y = torch.empty_like(x)
        st = runtime.seed_tensor
        call("fpnmt_dropout", dtype_code(x.dtype), x.numel(), float(p), seed, ptr(st), ptr(x), ptr(y), stream_ptr())
        ctx.seed = seed
        ctx.p = p
        ctx.st = st
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        call("fpnmt_dropout", dtype_code(dy.dtype), dy.numel(), float(ctx.p), ctx.seed, ptr(ctx.st), ptr(dy),
             ptr(dx), stream_ptr())
        return dx, None


def dropout(x, p, training):
    if not training or p <= 0.0 or x.numel() == 0:
        return x
    return DropoutFn.apply(x, p)


class AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        out = torch.empty_like(a)
        call("fpnmt_add", dtype_code(a.dtype), a.numel(), ptr(a), ptr(b), ptr(out), stream_ptr())
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g


def add(a, b):
    return AddFn.apply(a, b)


def cast(x, dtype):
    if x.dtype == dtype:
        return x
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=dtype, device=x.device)
    call("fpnmt_cast", dtype_code(x.dtype), dtype_code(dtype), x.numel(), ptr(x), ptr(y), stream_ptr())
    return y
