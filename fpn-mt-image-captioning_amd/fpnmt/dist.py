"""Data-parallel gradient exchange over the flat gradient arena.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
MI355X; "gloo" on CPU for tests). The per-rank masked-CE mean over an equal
shard equals the reference's global reduce_mean (utils/pipeline.py:57) after
averaging, so the exchange is a SUM all-reduce of the arena's fp32 gradients in
large contiguous buckets; the 1/world factor is folded into the optimizer
kernels (grad_scale) instead of a separate scaling pass. The embedding's
IndexedSlices clip-norm accumulator is summed alongside (and scaled by
grad_scale^2 in the optimizer).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 64 << 20  # few, large collectives: ring all-reduce is per-link bound on xGMI


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (RANK,
    WORLD_SIZE, MASTER_ADDR/PORT). Returns (rank, world, local_rank).

    FPNMT_DIST_BACKEND=gloo (read here, before any GPU call) overrides the
    default "nccl" (RCCL): a rehearsal of the multi-rank path with several
    ranks on one GPU, which RCCL refuses (see device_for_local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = os.environ.get("FPNMT_DIST_BACKEND") or None
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def device_for_local_rank(local):
    """The GPU a local rank drives: its own under RCCL (one process per GPU);
    under a gloo rehearsal on a box with fewer GPUs than ranks, ranks share
    them round-robin (torch.cuda.device_count() does not initialise HIP)."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        n = torch.cuda.device_count()
        return local % n if n > 0 else local
    return local


def barrier(group=None):
    """dist.barrier after any async gloo job of this process has finished."""
    if not dist.is_initialized():
        return
    if dist.get_backend(group) == "gloo":
        drain_gloo()
    dist.barrier(group=group)


def allreduce_max_scalar(x: float, group=None) -> float:
    """MAX over ranks of a host scalar (bench timing), on the group's backend:
    a device tensor for RCCL, a host tensor for gloo."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    dev = "cpu" if dist.get_backend(group) == "gloo" else "cuda"
    if dev == "cpu":
        drain_gloo()
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def bucket_ranges(total, bucket_elems):
    out, s = [], 0
    while s < total:
        e = min(total, s + bucket_elems)
        out.append((s, e))
        s = e
    return out


class _CastBackWork:
    """An all-reduce of a reduced-precision copy of a bucket: wait() orders
    the current stream after the collective, then writes the summed copy back
    into the fp32 bucket's place (overwrite)."""

    def __init__(self, work, low, dst):
        self.work, self.low, self.dst = work, low, dst

    def wait(self):
        self.work.wait()
        cast_into(self.dst, self.low)


def cast_into(dst: torch.Tensor, src: torch.Tensor):
    """dst[:] = src converted to dst's dtype (equal sizes, contiguous): the
    HIP cast kernel on the GPU (captured with the graph that calls it), a
    torch copy on the CPU (gloo tests)."""
    if dst.numel() != src.numel():
        raise ValueError(f"cast_into: {dst.numel()} vs {src.numel()} elements")
    if src.is_cuda:
        from . import _lib as L
        L.call("fpnmt_cast", L.dtype_code(src.dtype), L.dtype_code(dst.dtype), src.numel(), L.ptr(src), L.ptr(dst),
               L.stream_ptr())
    else:
        dst.copy_(src.reshape(dst.shape))


_staging = {}  # (device, dtype) -> reusable low-precision bucket buffer of allreduce_flat


def _stage_buffer(flat, dtype):
    key = (flat.device, dtype)
    buf = _staging.get(key)
    if buf is None or buf.numel() < flat.numel():
        buf = torch.empty(flat.numel(), dtype=dtype, device=flat.device)
        _staging[key] = buf
    return buf[:flat.numel()]


def allreduce_flat(flat: torch.Tensor, bucket_bytes=DEFAULT_BUCKET_BYTES, group=None, extra=None, wait=True,
                   bucket_dtype=None, staging=None):
    """SUM all-reduce of a flat fp32 tensor in contiguous buckets (all issued
    asynchronously). ``extra``: small tensors reduced as well (always fp32).
    wait=False returns the work handles (RCCL runs on its own stream, ordered
    after the work already queued on the current stream; Work.wait() makes
    the current stream wait for it without blocking the host).

    bucket_dtype=torch.bfloat16 (opt-in): buckets travel as bf16, half the
    xGMI bytes. Error: each rank's gradient is rounded to bf16 once, and a
    ring all-reduce rounds the running partial sum to bf16 at every hop of
    its reduce-scatter phase (world - 1 roundings), so
    |err| <~ 2^-8 * (sum_i |g_i| + sum over hops of |partial sum|), growing
    ~linearly with world (about 2^-8 * world * max|partial| at 8 GPUs).
    ``staging``: a preallocated bucket_dtype tensor of flat's size that
    already holds flat's cast (the TrainEngine casts inside its captured
    graphs and casts the sum back inside its update graph); the reduction
    then runs on it in place and nothing is written back here. Without it,
    the buckets are cast into a buffer here (a reused per-device one when
    wait=True, a fresh one otherwise) and written back into ``flat`` when
    waited for."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return []
    if dist.get_backend(group) == "gloo" and (flat.is_cuda or GLOO_ASYNC_DELAY_S > 0):
        if wait or not GLOO_ASYNC:
            return _allreduce_flat_gloo(flat, bucket_bytes, group, extra, bucket_dtype, staging)
        return [_gloo_async(flat, bucket_bytes, group, extra, bucket_dtype, staging)]
    if dist.get_backend(group) == "gloo":
        drain_gloo()
    low_dt = bucket_dtype is not None and bucket_dtype != flat.dtype
    esz = torch.empty((), dtype=bucket_dtype).element_size() if low_dt else flat.element_size()
    be = max(1, bucket_bytes // esz)
    if low_dt and staging is not None:
        if staging.dtype != bucket_dtype or staging.numel() != flat.numel():
            raise ValueError("allreduce_flat: staging must be a bucket_dtype tensor of flat's size")
    buf = None
    if low_dt and staging is None:
        # the reused per-device cast buffer only when this call completes
        # here; a call left in flight (wait=False) casts into a buffer of its
        # own (held by its works), so two such calls cannot overwrite each
        # other's buckets
        buf = _stage_buffer(flat, bucket_dtype) if wait else torch.empty(flat.numel(), dtype=bucket_dtype,
                                                                          device=flat.device)
    works = []
    for s, e in bucket_ranges(flat.numel(), be):
        if not low_dt:
            works.append(dist.all_reduce(flat[s:e], op=dist.ReduceOp.SUM, group=group, async_op=True))
        elif staging is not None:
            works.append(dist.all_reduce(staging[s:e], op=dist.ReduceOp.SUM, group=group, async_op=True))
        else:
            low = buf[s:e]
            cast_into(low, flat[s:e])
            works.append(_CastBackWork(dist.all_reduce(low, op=dist.ReduceOp.SUM, group=group, async_op=True),
                                       low, flat[s:e]))
    for t in extra or []:
        works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True))
    if wait:
        for w in works:
            w.wait()
        return []
    return works


def _allreduce_flat_gloo(flat, bucket_bytes, group, extra, bucket_dtype, staging):
    """allreduce_flat over gloo for device tensors (the multi-process tests that
    share one GPU; RCCL cannot put two ranks on one device): each bucket is
    reduced as a host copy, synchronously, with the same bucket cut and
    low-precision semantics as the RCCL path (a caller's staging is reduced
    in place; otherwise the low-precision sum is written back into flat).
    Returns [] (nothing left in flight)."""
    drain_gloo()
    low_dt = bucket_dtype is not None and bucket_dtype != flat.dtype
    src, own = flat, False
    if low_dt:
        if staging is None:
            staging, own = torch.empty(flat.numel(), dtype=bucket_dtype, device=flat.device), True
            cast_into(staging, flat)
        src = staging
    be = max(1, bucket_bytes // src.element_size())
    for s, e in bucket_ranges(src.numel(), be):
        h = src[s:e].cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        src[s:e].copy_(h)
    if own:
        cast_into(flat, staging)
    for t in extra or []:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    return []


# ---- asynchronous gloo exchange of device tensors -------------------------
# The multi-process GPU tests put two gloo ranks on one device (RCCL cannot),
# and gloo reduces host memory. So that those tests exercise the same
# overlap as the RCCL path (a range's exchange left in flight while the next
# graphs replay, the compute stream made to wait only in Work.wait()), an
# exchange with wait=False is handed to ONE worker thread per process, which
# runs the jobs in issue order (the same order on every rank, as gloo needs):
#   side stream waits for the `ready` event recorded on the issuing stream ->
#   device -> host copy -> gloo SUM (after GLOO_ASYNC_DELAY_S, a test knob that
#   widens the window in which a later graph writing into a range still being
#   reduced would corrupt it) -> host -> device copy-back on the side stream ->
#   `done` event. Work.wait() joins the job and makes the CURRENT stream wait
#   for `done`: the same contract as an RCCL Work.
GLOO_ASYNC = True          # False: wait=False exchanges run synchronously (the reference arm of the tests)
GLOO_ASYNC_DELAY_S = 0.0   # > 0: every async job sleeps this long before its reduction (CPU tensors too)

_pool = [None]
_side = {}
_pending = []  # futures of async gloo jobs not yet known to be finished


def drain_gloo():
    """Finish every async gloo job of this process before the calling thread
    issues a gloo collective of its own: two threads enqueueing on one group
    could order the collectives differently on the ranks (a hang, or equal-size
    buckets reduced against each other). The synchronous gloo paths call it."""
    while _pending:
        _pending.pop(0).result()


def _executor():
    if _pool[0] is None:
        import concurrent.futures as cf
        _pool[0] = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="fpnmt-gloo")
    return _pool[0]


class _GlooAsyncWork:
    def __init__(self, fut, done_event):
        self.fut, self.done_event = fut, done_event

    def wait(self):
        self.fut.result()  # the job ran (and recorded `done` on the side stream)
        if self.done_event is not None:
            torch.cuda.current_stream().wait_event(self.done_event)


def _gloo_async(flat, bucket_bytes, group, extra, bucket_dtype, staging):
    """allreduce_flat(wait=False) over gloo: see the block comment above."""
    import time
    low_dt = bucket_dtype is not None and bucket_dtype != flat.dtype
    own = False
    src = flat
    if low_dt:
        if staging is None:
            # a buffer of this call's own (held by the job), cast on the issuing stream
            staging, own = torch.empty(flat.numel(), dtype=bucket_dtype, device=flat.device), True
            cast_into(staging, flat)
        src = staging
    extra = list(extra or [])
    dev = flat.is_cuda
    ready = done = side = None
    if dev:
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        side = _side.get(flat.device)
        if side is None:
            side = _side[flat.device] = torch.cuda.Stream(device=flat.device)
        done = torch.cuda.Event(enable_timing=True)
    be = max(1, bucket_bytes // src.element_size())
    delay = GLOO_ASYNC_DELAY_S

    def job():
        if dev:
            torch.cuda.set_device(flat.device)
            with torch.cuda.stream(side):
                side.wait_event(ready)
                hosts = [src[s:e].to("cpu", non_blocking=True) for s, e in bucket_ranges(src.numel(), be)]
                hx = [t.to("cpu", non_blocking=True) for t in extra]
                side.synchronize()
        else:
            hosts = [src[s:e].clone() for s, e in bucket_ranges(src.numel(), be)]
            hx = [t.clone() for t in extra]
        if delay > 0:
            time.sleep(delay)
        for h in hosts + hx:
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        if dev:
            with torch.cuda.stream(side):
                for (s, e), h in zip(bucket_ranges(src.numel(), be), hosts):
                    src[s:e].copy_(h, non_blocking=True)
                for t, h in zip(extra, hx):
                    t.copy_(h, non_blocking=True)
                if own:
                    cast_into(flat, staging)
                done.record(side)
                side.synchronize()  # the host buffers must outlive the copies
        else:
            for (s, e), h in zip(bucket_ranges(src.numel(), be), hosts):
                src[s:e].copy_(h)
            for t, h in zip(extra, hx):
                t.copy_(h)
            if own:
                cast_into(flat, staging)

    fut = _executor().submit(job)
    _pending[:] = [f for f in _pending if not f.done()] + [fut]
    return _GlooAsyncWork(fut, done)


def broadcast_(t: torch.Tensor, src=0, group=None):
    """In-place broadcast from rank ``src`` (the initial weights); gloo takes a
    host copy of a device tensor, as allreduce_sum_ does."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    if dist.get_backend(group) == "gloo":
        drain_gloo()
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.broadcast(h, src, group=group)
        t.copy_(h)
        return t
    dist.broadcast(t, src, group=group)
    return t


def world_size(group=None):
    return dist.get_world_size(group) if dist.is_initialized() else 1


def allreduce_sum_(t: torch.Tensor, group=None):
    """In-place SUM all-reduce of a small tensor on the compute stream's
    order (SyncBN's per-channel fp64 sums). RCCL ("nccl") takes the device
    tensor directly (and is hipGraph-capturable); gloo reduces a host copy."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    if dist.get_backend(group) == "gloo":
        drain_gloo()
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
        return t
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def has_batchnorm(model):
    from .layers import BatchNormalization
    return any(isinstance(m, BatchNormalization) for m in model.modules())


def new_group_like(group=None):
    """A new communicator over the ranks of ``group`` (None: the world); a
    collective call, every rank of the world must make it."""
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
    return dist.new_group(ranks)


def set_sync_batchnorm(model, group=None):
    """Make every training-mode BatchNormalization of ``model`` a cross-replica
    one over ``group`` (None: the default group): the statistics and the
    backward's channel sums are then the global batch's, the moving averages
    identical on every rank (MobileNetV2 under data parallelism; the frozen-BN
    ResNet has none)."""
    from .layers import BatchNormalization
    n = 0
    for m in model.modules():
        if isinstance(m, BatchNormalization):
            m.sync_group = group if group is not None else dist.group.WORLD
            n += 1
    return n
