"""Batched beam decode (BASELINE C5; reference utils/pipeline.py:82-154):
the decode-attention and beam-step kernels against torch restatements, and
the whole BeamDecoder against the CPU oracle's literal predict()."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("lk,row_div,use_src,D", [(1, 1, True, 64), (7, 1, True, 64), (70, 1, True, 64),
                                                  (4, 3, False, 64), (32, 1, True, 64), (129, 2, False, 64),
                                                  (7, 1, True, 32)])
def test_decode_attention(dt, lk, row_div, use_src, D):
    """bf16 at depth 64 runs the 16-B kernel (decode_attn_v_kernel), depth 32
    and fp32 the lane-per-position one."""
    from fpnmt import _lib as L
    g = torch.Generator().manual_seed(lk * 10 + row_div)
    R, H, T = 12, 8, 140
    q = torch.randn(R, H * D, generator=g)
    nrows = R if use_src else R // row_div
    kv = torch.randn(nrows, T, 2 * H * D, generator=g)
    src = torch.randint(0, nrows, (R, T), generator=g, dtype=torch.int32)
    out = torch.empty(R, H * D, dtype=dt, device=DEV)
    qd, kvd = q.to(dt).to(DEV), kv.to(dt).to(DEV)
    srcd = src.to(DEV)
    scale = 1 / 8.0
    L.call("fpnmt_decode_attention", L.dtype_code(dt), R, H, D, lk, scale, qd.data_ptr(), H * D, kvd.data_ptr(),
           T * 2 * H * D, 2 * H * D, 0, H * D, srcd.data_ptr() if use_src else None, T, row_div, out.data_ptr(),
           H * D, L.stream_ptr())
    torch.cuda.synchronize()
    qf, kvf = q.to(dt).float(), kv.to(dt).float()
    ref = torch.empty(R, H * D)
    for r in range(R):
        rows = src[r, :lk].long() if use_src else torch.full((lk,), r // row_div, dtype=torch.long)
        K = kvf[rows, torch.arange(lk), :H * D].reshape(lk, H, D)
        V = kvf[rows, torch.arange(lk), H * D:].reshape(lk, H, D)
        qq = qf[r].reshape(H, D)
        s = torch.einsum("hd,jhd->hj", qq, K) * scale
        p = torch.softmax(s, -1)
        ref[r] = torch.einsum("hj,jhd->hd", p, V).reshape(-1)
    tol = 2e-5 if dt == torch.float32 else 2e-2
    assert float((out.float().cpu() - ref).abs().max()) <= tol


def _beam_ref(logits, beam_prob, beam_n, V):
    """utils/pipeline.py:115-141 per image (torch restatement)."""
    p = torch.softmax(logits, -1)
    cand = (p * beam_prob[:, None]).reshape(-1)
    vals, idx = torch.sort(cand, descending=True, stable=True)
    vals, idx = vals[:beam_n], idx[:beam_n]
    return vals, idx // V, idx % V


@pytest.mark.parametrize("beam_n,V", [(4, 200), (8, 10000), (1, 37), (16, 1000)])
def test_beam_step(beam_n, V):
    from fpnmt import _lib as L
    g = torch.Generator().manual_seed(beam_n * V)
    n_img, T, t = 3, 12, 5
    R = n_img * beam_n
    logits = torch.randn(R, V, generator=g)
    # exact ties across beams and within a row (tf.math.top_k: lower index first)
    logits[1] = logits[0]
    logits[0, 7] = logits[0, 3] = logits[0].max() + 1
    prob = torch.rand(R, generator=g) + 0.5
    prob[1] = prob[0]
    hist = torch.randint(4, V, (R, T + 1), generator=g, dtype=torch.int32)
    src = torch.randint(0, R, (R, T), generator=g, dtype=torch.int32)
    d = {k: v.to(DEV) for k, v in dict(logits=logits, prob=prob.clone(), hist=hist, src=src).items()}
    hout = torch.zeros_like(d["hist"])
    sout = torch.zeros_like(d["src"])
    tok = torch.zeros(R, dtype=torch.int32, device=DEV)
    result = torch.zeros(n_img, T, dtype=torch.int32, device=DEV)
    rlen = torch.zeros(n_img, dtype=torch.int32, device=DEV)
    status = torch.zeros(n_img, dtype=torch.int32, device=DEV)
    end = int(logits[2 * beam_n: 3 * beam_n].argmax()) % V if n_img > 2 else 3  # image 2 ends
    L.call("fpnmt_beam_step", n_img, beam_n, V, d["logits"].data_ptr(), V, d["prob"].data_ptr(),
           d["hist"].data_ptr(), hout.data_ptr(), T + 1, t, d["src"].data_ptr(), sout.data_ptr(), T, end,
           tok.data_ptr(), result.data_ptr(), T, rlen.data_ptr(), status.data_ptr(), L.stream_ptr())
    torch.cuda.synchronize()
    for i in range(n_img):
        rows = slice(i * beam_n, (i + 1) * beam_n)
        vals, par, tk = _beam_ref(logits[rows], prob[rows], beam_n, V)
        pr = par + i * beam_n
        assert torch.equal(tok.cpu()[rows], tk.to(torch.int32))
        assert torch.allclose(d["prob"].cpu()[rows], vals, rtol=1e-5, atol=0)
        assert torch.equal(hout.cpu()[rows, :t + 1], hist[pr, :t + 1])
        assert torch.equal(hout.cpu()[rows, t + 1], tk.to(torch.int32))
        assert torch.equal(sout.cpu()[rows, :t + 1], src[pr, :t + 1])
        assert torch.equal(sout.cpu()[rows, t + 1], torch.arange(i * beam_n, (i + 1) * beam_n, dtype=torch.int32))
        best = int(torch.argmax(vals))
        seq = torch.cat([hist[pr[best], 1:t + 1], tk[best:best + 1].to(torch.int32)])
        if int(tk[best]) == end:
            assert int(status[i]) == 1 and int(rlen[i]) == t
            assert torch.equal(result.cpu()[i, :t], seq[:-1])
        else:
            assert int(status[i]) == 0 and int(rlen[i]) == t + 1
            assert torch.equal(result.cpu()[i, :t + 1], seq)


def _pipeline(n_layers, vocab, image, seed, T):
    import fpnmt
    from fpnmt.layers import Init
    from utils.pipeline import Pipeline
    return Pipeline(max_seq_len=T, target_vocab_size=vocab, image_size=image, n_layers=n_layers, rate=0.0,
                    init=Init(torch.Generator().manual_seed(seed)), use_graph=False)


def test_batched_decode_matches_oracle_fp32():
    """Token ids of the batched, KV-cached, graph-replayed beam decode ==
    the CPU oracle running the reference's predict() literally (full-prefix
    recompute, beams of identical rows) on each image; 256^2 images so the
    cross-attention sees Lenc = 4 encoder positions."""
    import fpnmt
    from oracle import ref_cpu as R
    fpnmt.set_precision("fp32")
    T, vocab, image = 10, 200, 256
    pl = _pipeline(2, vocab, image, 13, T)
    sd = {k: v.detach().float().cpu().clone() for k, v in pl.transformer.state_dict().items()}
    cfg = dict(num_layers=2, num_heads=8, backbone="resnet50")
    g = torch.Generator().manual_seed(4)
    imgs = torch.rand(3, image, image, 3, generator=g) * 2 - 1
    ids = pl.predict_batch(imgs.to(DEV), T, beam_n=4)
    for i in range(3):
        ref = R.predict(sd, imgs[i], T, cfg, pl.start_token, pl.end_token, beam_n=4)
        assert ids[i] == ref.tolist(), (i, ids[i], ref.tolist())


def test_batched_decode_graph_matches_eager_bf16():
    import fpnmt
    fpnmt.set_precision("bf16")
    try:
        T, vocab, image = 12, 300, 224
        pl = _pipeline(2, vocab, image, 17, T)
        g = torch.Generator().manual_seed(6)
        imgs = (torch.rand(5, image, image, 3, generator=g) * 2 - 1).to(DEV)
        a = pl.predict_batch(imgs, T, beam_n=8, use_graph=False)
        b = pl.predict_batch(imgs, T, beam_n=8, use_graph=True)
        c = pl.predict_batch(imgs, T, beam_n=8, use_graph=True)  # replay of the captured graphs
        assert a == b == c
        assert all(len(x) <= T for x in a)
    finally:
        fpnmt.set_precision("fp32")
