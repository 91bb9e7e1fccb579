"""Flat parameter arena: every trainable tensor of a model lives in ONE fp32
buffer (params), with matching flat gradient / AMSGrad-state buffers.

Why: the optimizer step becomes one fused multi-tensor kernel over the arena
(fpnmt_grad_sumsq + fpnmt_amsgrad_step), the data-parallel gradient exchange is
a handful of large RCCL all-reduces over contiguous buckets, the gradient
zeroing is one memset, and nothing allocates inside a captured hipGraph.
Parameters stay ordinary ``nn.Parameter`` objects (views into the arena), so
``module.parameters()`` / state dicts behave as usual.

The compute copies of conv / dense weights (bf16 or fp32, kernel layouts)
are refreshed by ``prepare()`` after every optimizer step.
"""
from __future__ import annotations

import math

import torch

from . import _lib as L

ALIGN = 64  # elements (256 B) per segment start: keeps 16-B vector loads aligned
BLOCK_ELEMS = 16384


class ParamArena:
    def __init__(self, params, device, sparse_names=()):
        """params: ordered list of (name, nn.Parameter) — shared parameters
        appear once. sparse_names: parameters updated with the Keras sparse
        (IndexedSlices) path — the decoder embedding."""
        self.device = torch.device(device)
        self.names, self.params, self.offsets = [], [], []
        seen = set()
        off = 0
        for name, p in params:
            if id(p) in seen:
                continue
            seen.add(id(p))
            self.names.append(name)
            self.params.append(p)
            self.offsets.append(off)
            off += int(math.ceil(p.numel() / ALIGN) * ALIGN)
        self.total = off
        dev = self.device
        self.flat = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.m = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.vhat = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)  # Keras `iterations`
        nseg = len(self.params)
        self.sumsq = torch.zeros(max(nseg, 1), dtype=torch.float32, device=dev)
        self.index = {}
        seg_off = []
        flags = []
        sparse = set(sparse_names)
        for i, (name, p, o) in enumerate(zip(self.names, self.params, self.offsets)):
            n = p.numel()
            with torch.no_grad():
                self.flat[o:o + n].copy_(p.detach().reshape(-1).to(dev, torch.float32))
            p.data = self.flat[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)
            self.index[id(p)] = i
            seg_off.append(o)
            flags.append(3 if name in sparse else 0)
        seg_off.append(self.total)
        # segment end = start + numel (padding is never touched)
        ends = [o + p.numel() for o, p in zip(self.offsets, self.params)]
        # blocks that never cross a segment
        blk_seg, blk_start = [], []
        for i, (o, e) in enumerate(zip(self.offsets, ends)):
            s = o
            while s < e:
                blk_seg.append(i)
                blk_start.append(s)
                s += BLOCK_ELEMS
        self.nblocks = len(blk_seg)
        # first block of every segment (blocks are in segment order): the
        # optimizer sums a segment's per-block norm partials in block order
        seg_blk0, b = [], 0
        for i in range(nseg):
            seg_blk0.append(b)
            while b < len(blk_seg) and blk_seg[b] == i:
                b += 1
        seg_blk0.append(len(blk_seg))
        self._seg_blk0_host = seg_blk0
        self.seg_blk0 = torch.tensor(seg_blk0, dtype=torch.int32, device=dev)
        self.blk_part = torch.zeros(max(len(blk_seg), 1), dtype=torch.float32, device=dev)
        self.blk_seg = torch.tensor(blk_seg or [0], dtype=torch.int32, device=dev)
        self.blk_start = torch.tensor(blk_start or [0], dtype=torch.int64, device=dev)
        # the kernels clamp block ends at off[seg+1] = END of segment seg
        seg_end = torch.tensor([*ends], dtype=torch.int64)
        self.seg_bounds = torch.zeros(nseg + 1, dtype=torch.int64)
        self.seg_bounds[1:] = seg_end
        self.seg_bounds[0] = 0
        self.seg_bounds = self.seg_bounds.to(dev)
        self.seg_flags = torch.tensor(flags or [0], dtype=torch.int32, device=dev)
        self.preparers = []

    # -------------------------------------------------------------- grads
    def zero_grad(self, max_blocks=0):
        """Gradient arena + the per-tensor sum-of-squares slots to zero (HIP
        zero-fill kernels: no eager-PyTorch kernel inside the replayed step).
        max_blocks > 0: the arena's fill on at most that many workgroups (a
        background trickle beside other work on another stream)."""
        if self.grad.is_cuda:
            from ._lib import call, stream_ptr
            nbytes = self.grad.numel() * self.grad.element_size()
            if max_blocks > 0:
                call("fpnmt_fill_zero_grid", self.grad.data_ptr(), nbytes, int(max_blocks), stream_ptr())
            else:
                call("fpnmt_fill_zero", self.grad.data_ptr(), nbytes, stream_ptr())
            call("fpnmt_fill_zero", self.sumsq.data_ptr(), self.sumsq.numel() * self.sumsq.element_size(),
                 stream_ptr())
        else:  # CPU arenas of the host-only tests
            self.grad.zero_()
            self.sumsq.zero_()

    def seg_of(self, p) -> int:
        return self.index[id(p)]

    def sumsq_slot(self, p):
        i = self.index[id(p)]
        return self.sumsq[i:i + 1]

    # ---------------------------------------------------------- optimizer
    def block_of(self, offset):
        """First optimizer block of the segment starting at `offset` (the
        arena's total: nblocks), for amsgrad_step(blocks=...)."""
        if offset >= self.total:
            return self.nblocks
        i = self.offsets.index(offset)
        return self._seg_blk0_host[i]

    def amsgrad_step(self, lr_schedule, beta1=0.9, beta2=0.98, eps=1e-9, clipnorm=1.0, grad_scale=1.0,
                     preps=None, blocks=None, inc_step=True, max_grid=0):
        """Keras AMSGrad + per-tensor clip_by_norm over the arena. preps: a
        device table of fpnmt_seg_prep (one per segment, layers.FusedPrep)
        whose non-null entries get their bf16 compute copies written by the
        same kernel. blocks: (first, end) block range of whole segments (one
        part of a step updated in parts); inc_step: advance `iterations`
        (only the step's last part); max_grid: at most that many workgroups
        striding over the range (0: one per block)."""
        d = L.AdamDesc()
        d.beta1, d.beta2, d.eps, d.clipnorm = beta1, beta2, eps, clipnorm
        d.grad_scale = grad_scale
        if isinstance(lr_schedule, (int, float)):
            d.sched_d_model = 0.0
            d.const_lr = float(lr_schedule)
        else:
            d.sched_d_model = float(lr_schedule.d_model)
            d.sched_warmup = float(lr_schedule.warmup_steps)
            d.sched_mult = float(lr_schedule.multiplier)
            d.sched_warm_pow = float(lr_schedule.warmup_steps ** -1.5)
        b0, b1 = (0, self.nblocks) if blocks is None else blocks
        s = L.stream_ptr()
        if clipnorm > 0 and b1 > b0:  # clipnorm 0: no clip_by_norm, no norms needed
            L.call("fpnmt_grad_sumsq_part", b0, b1 - b0, max_grid, L.ptr(self.blk_seg), L.ptr(self.blk_start), BLOCK_ELEMS,
                   L.ptr(self.seg_bounds), L.ptr(self.seg_flags), L.ptr(self.grad), grad_scale,
                   L.ptr(self.blk_part), s)
        L.call("fpnmt_amsgrad_step_part", d, b0, b1 - b0, 1 if inc_step else 0, max_grid, L.ptr(self.blk_seg),
               L.ptr(self.blk_start), BLOCK_ELEMS, L.ptr(self.seg_bounds), L.ptr(self.seg_flags), L.ptr(self.flat),
               L.ptr(self.grad), L.ptr(self.m), L.ptr(self.v), L.ptr(self.vhat), L.ptr(self.sumsq),
               L.ptr(self.blk_part), L.ptr(self.seg_blk0), L.ptr(self.step),
               L.ptr(preps) if preps is not None else None, s)

    # ------------------------------------------------------ compute copies
    def register_preparer(self, fn):
        self.preparers.append(fn)

    def prepare(self):
        for fn in self.preparers:
            fn()
