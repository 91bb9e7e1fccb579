"""Data-parallel path on CPU (gloo, world_size 2, 127.0.0.1):

1. fpnmt.dist.allreduce_flat: bucketed SUM all-reduce of the flat gradient
   arena (uneven bucket split, extra scalars) equals the rank sum.
2. DP semantics: averaging per-rank masked-CE gradients over equal shards
   equals the full-batch gradient of the reference loss (utils/pipeline.py:57
   reduce_mean over B*T) — checked with the CPU oracle on a tiny decoder.
(The optimizer's grad_scale = 1/world folding, incl. the IndexedSlices norm
scaled by grad_scale^2, runs on the GPU kernels: tests/test_gpu_kernels.py::
test_amsgrad_grad_scale_equals_averaged_grads.)
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    try:
        torch.save(fn(rank, world), os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _spawn(fn, world=2):
    import tempfile
    ctx = mp.get_context("fork")
    port = _port()
    with tempfile.TemporaryDirectory() as outdir:
        ps = [ctx.Process(target=_run, args=(r, world, port, fn, outdir)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=120)
            assert p.exitcode == 0
        return {r: torch.load(os.path.join(outdir, f"r{r}.pt"), weights_only=False) for r in range(world)}


def _allreduce_case(rank, world):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fpn-mt-image-captioning_amd"))
    from fpnmt.dist import allreduce_flat
    g = torch.Generator().manual_seed(rank)
    flat = torch.randn(10007, generator=g)
    extra = torch.tensor([float(rank + 1)])
    mine = flat.clone()
    allreduce_flat(flat, bucket_bytes=4 * 1000, extra=[extra])  # 11 uneven buckets
    return mine, flat, extra


def test_bucketed_allreduce_sum():
    out = _spawn(_allreduce_case)
    total = out[0][0] + out[1][0]
    for r in (0, 1):
        assert torch.allclose(out[r][1], total, atol=1e-5)
        assert float(out[r][2]) == 3.0


def _tiny_decoder_sd(V=23, d=16):
    from oracle import ref_cpu as R
    g = torch.Generator().manual_seed(0)
    return {
        "decoder.embedding.embeddings": torch.randn(V, d, generator=g) * 0.1,
        "decoder.pos_encoding": R.raw_positional_encoding(12, d),
        "final_layer.kernel": torch.randn(d, V, generator=g) * 0.3,
        "final_layer.bias": torch.zeros(V),
    }


def _batch():
    g = torch.Generator().manual_seed(4)
    tok = torch.randint(4, 23, (4, 10), generator=g)
    tok[:, 0] = 2
    tok[1, 6:] = 0
    tok[3, 4:] = 0
    enc = torch.randn(4, 1, 16, generator=g)
    return tok, enc


def _grads(sd, tok, enc):
    from oracle import ref_cpu as R
    p = {k: v.clone().requires_grad_(k != "decoder.pos_encoding") for k, v in sd.items()}
    cfg = dict(num_layers=0, num_heads=2, backbone="resnet50")
    tar_inp, tar_real = tok[:, :-1], tok[:, 1:]
    logits, _ = R.transformer(p, enc, tar_inp, False, R.create_masks(tar_inp), cfg)
    R.masked_loss(tar_real, logits).backward()
    return {k: v.grad for k, v in p.items() if v.grad is not None}


def _dp_grad_case(rank, world):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sd = _tiny_decoder_sd()
    tok, enc = _batch()
    shard = slice(rank * 2, rank * 2 + 2)
    gr = _grads(sd, tok[shard], enc[shard])
    names = sorted(gr)
    flat = torch.cat([gr[n].reshape(-1) for n in names])
    dist.all_reduce(flat)
    flat /= world
    return names, flat


def test_dp_average_equals_full_batch_gradient():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    out = _spawn(_dp_grad_case)
    names, flat = out[0]
    full = _grads(_tiny_decoder_sd(), *_batch())
    ref = torch.cat([full[n].reshape(-1) for n in names])
    assert torch.allclose(flat, ref, atol=1e-6, rtol=1e-5)
    assert torch.allclose(out[1][1], flat)


def _split_exchange_case(rank, world):
    """TrainEngine's staged exchange (the decoder side's range after G1, the
    encoder layers' after G2, then one per feature-extractor stage, all async,
    then waited) on a real model's arena: every gradient element and the
    embedding's sparse-norm slot end up as the rank sum; the arena is ordered
    decoder side, encoder layers, feature extractor."""
    import math
    import sys
    torch.set_num_threads(1)  # forked child: keep off the parent's OpenMP pool
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "fpn-mt-image-captioning_amd"))
    sys.path.insert(0, root)
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from models.transformer import Transformer
    m = Transformer(1, 512, 8, 2048, math.ceil(64 / 16) ** 2, 50, 0.0, max_seq_len=8,
                    init=Init(torch.Generator().manual_seed(rank)))  # broadcast makes rank 0's weights win
    eng = TrainEngine(m, 1e-4, use_graph=False)
    assert eng.split and 0 < eng.split_at < eng.arena.total
    names = eng.arena.names
    first_fe = next(i for i, n in enumerate(names) if n.startswith("encoder.feature_extractor."))
    assert all(n.startswith("encoder.feature_extractor.") for n in names[first_fe:])
    g = torch.Generator().manual_seed(100 + rank)
    mine = torch.randn(eng.arena.total, generator=g)
    eng.arena.grad.copy_(mine)
    eng.arena.sumsq.fill_(float(rank + 1))
    # one range per exchange: the decoder side, the encoder layers, then the
    # feature extractor's stages (heads, FPN, backbone segments) — contiguous,
    # covering the arena
    dec_end = eng.ranges[0][1]
    assert all(n.startswith(("decoder.", "final_layer.")) for n, o in zip(names, eng.arena.offsets) if o < dec_end)
    assert all(not n.startswith(("decoder.", "final_layer.")) for n, o in zip(names, eng.arena.offsets) if o >= dec_end)
    rs = [r for r in eng.ranges if r[1] > r[0]]
    assert rs[0][0] == 0 and rs[1] == (dec_end, eng.split_at) and len(rs) >= 6
    covered = sorted(rs)
    assert all(a[1] <= b[0] for a, b in zip(covered, covered[1:]))
    assert sum(e - s for s, e in rs) >= eng.arena.total - 64 * len(eng.arena.names)
    works = []
    for part in range(len(eng.ranges)):
        works += eng._exchange(part, wait=False)
    for w in works:
        w.wait()
    return mine, eng.arena.grad.clone(), float(eng.arena.sumsq[eng.emb_seg]), eng.arena.flat.clone()


def test_split_exchange_sums_both_ranges():
    out = _spawn(_split_exchange_case)
    total = out[0][0] + out[1][0]
    for r in (0, 1):
        assert torch.allclose(out[r][1], total, atol=1e-5)
        assert out[r][2] == 3.0
    assert torch.equal(out[0][3], out[1][3])  # initial weights broadcast from rank 0


def _bf16_bucket_case(rank, world):
    """Opt-in bf16 gradient buckets: the summed gradient equals the fp32 sum
    within bf16 rounding (at world 2: each rank's contribution, then the one
    hop's partial sum)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fpn-mt-image-captioning_amd"))
    from fpnmt.dist import allreduce_flat
    g = torch.Generator().manual_seed(10 + rank)
    flat = torch.randn(5003, generator=g) * 10
    mine = flat.clone()
    # two calls in flight at once (two halves, as per-range exchanges are):
    # each casts into a buffer of its own
    works = allreduce_flat(flat[:3000], bucket_bytes=2 * 1000, wait=False, bucket_dtype=torch.bfloat16)
    works += allreduce_flat(flat[3000:], bucket_bytes=2 * 1000, wait=False, bucket_dtype=torch.bfloat16)
    assert len(works) == 6  # 1000 bf16 elements per bucket: 3 + 3
    for w in works:
        w.wait()
    return mine, flat


def test_bf16_buckets_sum_within_bf16_rounding():
    out = _spawn(_bf16_bucket_case)
    total = out[0][0] + out[1][0]
    for r in (0, 1):
        got = out[r][1]
        assert got.dtype == torch.float32
        # |err| <= (|a| + |b| + |a + b|) * 2^-8: one bf16 rounding of each input and of the sum
        bound = (out[0][0].abs() + out[1][0].abs() + total.abs()) * 2.0 ** -8
        assert bool(((got - total).abs() <= bound).all())
    assert torch.equal(out[0][1], out[1][1])


def _engine_bf16_staging_case(rank, world):
    """TrainEngine's bf16 bucket mode: each exchange range is cast into the
    preallocated staging copy (as at the end of its graph), reduced in place,
    and cast back into the fp32 arena (as at the start of the update graph)."""
    import math
    import sys
    torch.set_num_threads(1)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "fpn-mt-image-captioning_amd"))
    sys.path.insert(0, root)
    from fpnmt import dist as fdist
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from models.transformer import Transformer
    m = Transformer(1, 512, 8, 2048, math.ceil(64 / 16) ** 2, 50, 0.0, max_seq_len=8,
                    init=Init(torch.Generator().manual_seed(rank)))
    eng = TrainEngine(m, 1e-4, use_graph=False, bucket_dtype=torch.bfloat16, bucket_bytes=1 << 20)
    assert eng.low is not None and eng.low.dtype == torch.bfloat16 and eng.low.numel() == eng.arena.total
    buf = eng.low.data_ptr()
    mine = torch.randn(eng.arena.total, generator=torch.Generator().manual_seed(200 + rank))
    eng.arena.grad.copy_(mine)
    works = []
    for part in range(len(eng.ranges)):
        eng._stage_low(part)
        works += eng._exchange(part, wait=False)
    for w in works:
        w.wait()
    fdist.cast_into(eng.arena.grad, eng.low)
    assert eng.low.data_ptr() == buf  # no per-step staging allocation
    covered = torch.zeros(eng.arena.total, dtype=torch.bool)
    for a, b in eng.ranges:
        covered[a:b] = True
    return mine, eng.arena.grad.clone(), covered


def test_engine_bf16_staging_sum():
    out = _spawn(_engine_bf16_staging_case)
    total = out[0][0] + out[1][0]
    cov = out[0][2]
    bound = (out[0][0].abs() + out[1][0].abs() + total.abs()) * 2.0 ** -8
    for r in (0, 1):
        got = out[r][1]
        assert bool(((got - total).abs() <= bound)[cov].all())
        assert bool((got[~cov] == 0).all())  # alignment gaps stay zero
    assert torch.equal(out[0][1], out[1][1])


def _async_delayed_case(rank, world):
    """Three ranges exchanged with wait=False through the gloo worker (each
    job delayed 50 ms): right after issue the ranges still hold this rank's
    values (the exchange is in flight while the caller goes on); after the
    waits they hold the sums, bitwise equal to the synchronous arm."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fpn-mt-image-captioning_amd"))
    import time
    from fpnmt import dist as fd
    g = torch.Generator().manual_seed(10 + rank)
    base = torch.randn(30011, generator=g)
    ranges = [(0, 9000), (9000, 21000), (21000, 30011)]
    out = {}
    for arm in ("sync", "async"):
        fd.GLOO_ASYNC = arm == "async"
        fd.GLOO_ASYNC_DELAY_S = 0.05
        flat = base.clone()
        extra = torch.tensor([float(rank + 1)])
        t0 = time.perf_counter()
        works = []
        for i, (a, b) in enumerate(ranges):
            works += fd.allreduce_flat(flat[a:b], bucket_bytes=4 * 2500, group=None,
                                       extra=[extra] if i == 0 else None, wait=False)
        issue_s = time.perf_counter() - t0
        untouched = bool(torch.equal(flat, base))
        for w in works:
            w.wait()
        out[arm] = dict(flat=flat, extra=float(extra), issue_s=issue_s, untouched_after_issue=untouched,
                        n_works=len(works))
    fd.GLOO_ASYNC, fd.GLOO_ASYNC_DELAY_S = True, 0.0
    return base, out


def test_gloo_async_delayed_exchange_equals_sync():
    """fpnmt.dist's asynchronous gloo exchange (the path the world-2 GPU
    test's TrainEngine.step takes: exchanges in flight under later graphs,
    Work.wait() at the update): returns at once with the reduction pending,
    and the waited result equals the synchronous arm's bit for bit."""
    out = _spawn(_async_delayed_case)
    total = out[0][0] + out[1][0]
    for r in (0, 1):
        res = out[r][1]
        assert torch.equal(res["async"]["flat"], res["sync"]["flat"])
        assert torch.allclose(res["async"]["flat"], total, atol=1e-5)
        assert res["async"]["extra"] == 3.0 and res["sync"]["extra"] == 3.0
        assert res["async"]["n_works"] == 3 and res["sync"]["n_works"] == 0
        # the async arm returned before any 50 ms job finished, leaving the data untouched
        assert res["async"]["untouched_after_issue"] and res["async"]["issue_s"] < 0.05
        assert not res["sync"]["untouched_after_issue"]  # the synchronous arm reduced before returning


def _async_then_sync_case(rank, world):
    """An async exchange left pending (delayed 100 ms on the worker thread),
    then synchronous gloo collectives issued by the main thread before
    anything waits: allreduce_sum_ and broadcast_ drain the worker first, so
    both threads never enqueue on the group at once."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fpn-mt-image-captioning_amd"))
    from fpnmt import dist as fd
    fd.GLOO_ASYNC, fd.GLOO_ASYNC_DELAY_S = True, 0.1
    flat = torch.full((4096,), float(rank + 1))
    works = fd.allreduce_flat(flat, bucket_bytes=4 * 1024, wait=False)
    small = torch.full((7,), float(10 * (rank + 1)))  # same size as no bucket, different values
    fd.allreduce_sum_(small)
    b = torch.full((5,), float(rank))
    fd.broadcast_(b, src=1)
    for w in works:
        w.wait()
    fd.GLOO_ASYNC_DELAY_S = 0.0
    return flat, small, b


def test_gloo_sync_collectives_drain_async_jobs():
    out = _spawn(_async_then_sync_case)
    for r in (0, 1):
        flat, small, b = out[r]
        assert bool((flat == 3.0).all()) and bool((small == 30.0).all()) and bool((b == 1.0).all())
