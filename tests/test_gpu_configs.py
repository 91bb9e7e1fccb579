"""Parity at the BASELINE.json configurations themselves (not just small
shapes): C2 (R50-FPN + 6-layer transformer, 224^2, batch 32, V = 10 000), C3
(R101-FPN FeatureExtractor at 512^2, batch 64) and C5 (beam 8 batched decode,
256 images). GPU results in exact-fp32 mode are compared with the CPU oracle
(oracle/ref_cpu.py), which restates models/retinanet.py:266-307,
models/transformer.py:344-374 and utils/pipeline.py:50-57,82-154; the bf16
perf mode at the full batch is checked by stated properties against fp32.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
V_C2 = 10000


def _model(num_layers, vocab, image, seed, backbone="resnet50", rate=0.0):
    import fpnmt
    from fpnmt.layers import Init
    from models.transformer import Transformer
    fpnmt.set_precision("fp32")
    m = Transformer(num_layers, 512, 8, 2048, math.ceil(image / 16) ** 2, vocab, rate, max_seq_len=32,
                    backbone=backbone, init=Init(torch.Generator().manual_seed(seed)))
    sd = {k: v.detach().float().clone() for k, v in m.state_dict().items()}
    return m.to(DEV), sd, dict(num_layers=num_layers, num_heads=8, backbone=backbone)


def _captions(b, vocab, T=32, seed=1):
    """bench.py's synthetic captions: [<start>] + U{4..V-1} + [<end>], len U{8..32}, 0-padded."""
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(4, vocab, (b, T), generator=g)
    tok[:, 0] = 2
    lens = torch.randint(8, T + 1, (b,), generator=g)
    for i in range(b):
        tok[i, int(lens[i]) - 1] = 3
        tok[i, int(lens[i]):] = 0
    return tok


def _images(b, image, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(b, image, image, 3, generator=g) * 2 - 1


def _structured_images(b, image, seed=0):
    """b structurally different images in [-1, 1) (NHWC): smooth colour
    fields, gradients, stripes, checkerboards and rings with per-image
    orientation / frequency / colours, plus 5 % noise. U[-1, 1) noise images
    all look alike to the random frozen ResNet (their pyramids differ by
    texture only), so a model trained to caption them cannot tell them
    apart; these give each image features of its own."""
    g = torch.Generator().manual_seed(seed)
    y, x = torch.meshgrid(torch.linspace(-1, 1, image), torch.linspace(-1, 1, image), indexing="ij")
    out = torch.empty(b, image, image, 3)
    for i in range(b):
        col = torch.rand(2, 3, generator=g) * 2 - 1          # two colours
        th = float(torch.rand(1, generator=g)) * 3.14159
        f = 1.0 + 6.0 * float(torch.rand(1, generator=g))    # frequency
        u = x * torch.cos(torch.tensor(th)) + y * torch.sin(torch.tensor(th))
        kind = i % 5
        if kind == 0:
            t = (u + 1) / 2                                  # linear gradient
        elif kind == 1:
            t = (torch.sin(f * 3.14159 * u) > 0).float()     # stripes
        elif kind == 2:
            t = ((torch.floor((x + 1) * f) + torch.floor((y + 1) * f)) % 2)  # checkerboard
        elif kind == 3:
            t = (torch.sin(f * 3.14159 * (x * x + y * y).sqrt()) + 1) / 2    # rings
        else:
            t = torch.zeros_like(x) + float(torch.rand(1, generator=g))     # flat field
        img = col[0] * (1 - t)[..., None] + col[1] * t[..., None]
        img = img + 0.05 * (torch.rand(image, image, 3, generator=g) * 2 - 1)
        out[i] = img.clamp(-1, 0.9999)
    return out


def _oracle_logits(sd, img, tar, cfg, chunk=8):
    from oracle import ref_cpu as R
    torch.set_num_threads(min(16, torch.get_num_threads()))
    outs = []
    with torch.no_grad():
        for s in range(0, img.shape[0], chunk):
            t = tar[s:s + chunk]
            lg, _ = R.transformer(sd, img[s:s + chunk], t, True, R.create_masks(t), cfg)
            outs.append(lg)
    return torch.cat(outs)


# ------------------------------------------------------------------- C2
def test_c2_logits_and_loss_parity_fp32(parity_record):
    """C2 model and batch (6 layers, V = 10 000, 32 images of 224^2): fp32
    logits of every image within 1e-3 of the oracle, the masked-CE loss
    (utils/pipeline.py:50-57, mean over all 32 x 31 positions) within 1e-4."""
    from oracle import ref_cpu as R
    from fpnmt import ops
    from models.transformer import create_masks
    m, sd, cfg = _model(6, V_C2, 224, 1234)
    img, tok = _images(32, 224), _captions(32, V_C2)
    tar_inp, tar_real = tok[:, :-1], tok[:, 1:]
    with torch.no_grad():
        logits, _ = m(img.to(DEV), tar_inp.to(DEV), True, create_masks(tar_inp.to(DEV)))
        loss = float(ops.MaskedXentFn.apply(logits, tar_real.to(DEV)))
    ref = _oracle_logits(sd, img, tar_inp, cfg)
    d = (logits.cpu() - ref).abs()
    per_img = d.reshape(32, -1).amax(1)
    print(f"C2 fp32 logits: max|d| {float(d.max()):.2e} (images 0-1: {float(per_img[:2].max()):.2e}), "
          f"|logits| max {float(ref.abs().max()):.2f}")
    assert float(per_img[:2].max()) <= 1e-3
    assert float(d.max()) <= 1e-3
    loss_ref = float(R.masked_loss(tar_real, ref))
    print(f"C2 loss gpu {loss:.7f} oracle {loss_ref:.7f}")
    parity_record["c2_fp32_logits"] = {
        "images": 32, "max_abs_delta": float(d.max()), "per_image_max_abs_delta": [float(x) for x in per_img],
        "max_abs_logit": float(ref.abs().max()), "loss_gpu": loss, "loss_oracle": loss_ref,
        "loss_abs_delta": abs(loss - loss_ref), "bar_logits": 1e-3, "bar_loss": 1e-4}
    assert abs(loss - loss_ref) <= 1e-4


def test_c2_train_step_fp32_then_bf16():
    """The C2 training step itself (TrainEngine, batch 32): the fp32 step's
    loss equals the oracle's forward loss of the same parameters (step 0:
    only forward arithmetic differs), every parameter moves, and the bf16
    hipGraph step (the bench configuration, dropout 0.1) stays finite with a
    loss within 3 % of fp32's on the same batch."""
    from oracle import ref_cpu as R
    import fpnmt
    from fpnmt.train import TrainEngine
    from utils.utils import CustomSchedule
    img, tok = _images(32, 224, seed=2), _captions(32, V_C2, seed=3)
    m, sd, cfg = _model(6, V_C2, 224, 77)
    eng = TrainEngine(m, 1e-4, use_graph=False)
    p0 = eng.arena.flat.clone()
    loss = float(eng.step(img.to(DEV), tok.to(DEV)))
    ref = _oracle_logits(sd, img, tok[:, :-1], cfg)
    loss_ref = float(R.masked_loss(tok[:, 1:], ref))
    print(f"C2 fp32 train-step loss {loss:.7f} oracle {loss_ref:.7f}")
    assert abs(loss - loss_ref) <= 1e-4
    moved = (eng.arena.flat - p0).abs()
    frac = float((moved > 0).sum()) / float(sum(p.numel() for p in eng.arena.params))
    # Adam moves every element with a non-zero gradient. Structurally zero at
    # 224^2: the unused embedding rows, the empty P7 view's projections (Lk =
    # 0), the cross-attention Q/K (softmax over the single encoder position)
    print(f"fraction of parameters updated: {frac:.3f}")
    assert frac > 0.5, frac
    # bf16 perf mode, same model, hipGraph replay with dropout 0.1 (bench.py)
    mb, _, _ = _model(6, V_C2, 224, 77, rate=0.1)
    fpnmt.set_precision("bf16")
    try:
        engb = TrainEngine(mb, CustomSchedule(2048, 4000), use_graph=True)
        lb = [float(engb.step(img.to(DEV), tok.to(DEV))) for _ in range(3)]
    finally:
        fpnmt.set_precision("fp32")
    print(f"C2 bf16 graph steps: {lb}")
    assert all(math.isfinite(x) for x in lb)
    # lr(0) = 0: the first step leaves the weights unchanged, so the first two
    # losses differ only by dropout masks; the fp32 loss is the no-dropout value
    assert abs(lb[0] - loss) <= 0.03 * loss


def _rel_rms(a, b):
    return float((a - b).double().norm() / b.double().norm().clamp_min(1e-30))


# bf16 error bounds of the benchmarked arithmetic at C2 (bf16 operands and
# activations, fp32 accumulation; unit roundoff 2^-9 per rounding, ~20 chained
# roundings through R50-FPN + 6 transformer layers). Measured on MI355X
# (profiles/r06/parity_bf16.json): logits rel RMS 0.056, worst image 0.21 of
# its max |logit|, loss 1e-6 relative, transformer gradients rel RMS 0.075.
# The feature extractor's gradients are NOT pinned by bf16 at random init:
# per backward stage rel RMS 0.67-1.0, cosine 0.19-0.74 to the fp32 path's
# (profiles/r06/bf16_grad_probe.txt, bf16_grad_chain.txt). Localised: every
# forward activation is bf16-accurate (0.4-1 % rel) except the co-attention
# output of levels P4 / P6 (~10 %): their regression scores span ~300 with
# near-ties at the top, so softmax over positions acts as an argmax whose
# winner moves under 0.5 % score noise; the level gradients then differ by
# 40-80 %, upstream of which the FPN / res5 stages sit. The same error with
# every backward fusion off (not a fused-path artefact); rounding only the
# masters to bf16 in fp32 arithmetic already moves those stages by 28-52 %.
BF16_LOGIT_REL_RMS = 0.10       # ||logits_bf16 - logits_oracle||_2 / ||logits_oracle||_2 over the batch
BF16_LOGIT_IMG_MAXABS = 0.35    # per image: max |d| / max |logits_oracle| of that image
BF16_LOSS_REL = 1e-3            # masked-CE loss, relative
BF16_GRAD_REL_RMS_TRANSFORMER = 0.15  # one step's gradient, the transformer's arena range vs fp32
BF16_GRAD_REL_RMS_FE = 1.2      # each feature-extractor stage's range, relative RMS vs fp32
BF16_GRAD_COS_FE = 0.1          # ... and cosine similarity to the fp32 gradient, per stage


def test_c2_bf16_perf_path_vs_oracle(parity_record):
    """The benchmarked bf16 arithmetic at C2 (6 layers, V = 10 000, 32 images
    of 224^2; utils/pipeline.py:50-57) against the fp32 CPU oracle:
    logits relative RMS <= BF16_LOGIT_REL_RMS over the batch, per image
    max |d| <= BF16_LOGIT_IMG_MAXABS * max |logit| of that image, the loss
    within BF16_LOSS_REL; then one training step's gradients in bf16 against
    the fp32 path's on the same parameters and batch (dropout 0): relative
    RMS <= BF16_GRAD_REL_RMS_TRANSFORMER over the transformer's arena range;
    per feature-extractor stage range relative RMS <= BF16_GRAD_REL_RMS_FE
    and cosine similarity >= BF16_GRAD_COS_FE (the bounds' derivation is
    in the comment above them)."""
    from oracle import ref_cpu as R
    import fpnmt
    from fpnmt import ops
    from fpnmt.train import TrainEngine
    from models.transformer import create_masks
    m, sd, cfg = _model(6, V_C2, 224, 1234)
    img, tok = _images(32, 224), _captions(32, V_C2)
    tar_inp, tar_real = tok[:, :-1], tok[:, 1:]
    ref = _oracle_logits(sd, img, tar_inp, cfg)
    loss_ref = float(R.masked_loss(tar_real, ref))
    fpnmt.set_precision("bf16")
    try:
        with torch.no_grad():
            lg, _ = m(img.to(DEV), tar_inp.to(DEV), True, create_masks(tar_inp.to(DEV)))
            loss = float(ops.MaskedXentFn.apply(lg, tar_real.to(DEV)))
        lg = lg.float().cpu()
    finally:
        fpnmt.set_precision("fp32")
    rel = _rel_rms(lg, ref)
    d = (lg - ref).abs().reshape(32, -1)
    img_frac = (d.amax(1) / ref.abs().reshape(32, -1).amax(1)).tolist()
    loss_rel = abs(loss - loss_ref) / abs(loss_ref)
    # one step's gradients: bf16 vs fp32 on the same parameters and batch
    grads = {}
    for prec in ("fp32", "bf16"):
        mm, _, _ = _model(6, V_C2, 224, 1234)
        fpnmt.set_precision(prec)
        try:
            eng = TrainEngine(mm, 1e-4, use_graph=False)
            eng.step(img.to(DEV), tok.to(DEV))
            torch.cuda.synchronize()
            grads[prec] = eng.arena.grad.detach().cpu().clone()
            split_at = eng.split_at  # transformer parameters first, then the feature extractor
            stage_ranges = [r for r in eng.ranges[2:] if r[1] > r[0]]  # heads, FPN, C4-C5, C3-C4, input-C3
        finally:
            fpnmt.set_precision("fp32")
        del eng, mm
        torch.cuda.empty_cache()
    g32, g16 = grads["fp32"], grads["bf16"]
    rel_tr = _rel_rms(g16[:split_at], g32[:split_at])
    rel_fe = _rel_rms(g16[split_at:], g32[split_at:])
    cos = lambda a, b: float((a.double() @ b.double()) / (a.double().norm() * b.double().norm()).clamp_min(1e-300))
    stages = [{"range": list(r), "rel_rms": _rel_rms(g16[r[0]:r[1]], g32[r[0]:r[1]]),
               "cos": cos(g16[r[0]:r[1]], g32[r[0]:r[1]])} for r in stage_ranges]
    rec = {"images": 32, "logits_rel_rms": rel, "logits_per_image_maxabs_frac": img_frac,
           "loss_bf16": loss, "loss_oracle": loss_ref, "loss_rel": loss_rel,
           "grad_rel_rms_transformer": rel_tr, "grad_rel_rms_feature_extractor": rel_fe,
           "grad_feature_extractor_stages": stages,
           "bounds": {"logits_rel_rms": BF16_LOGIT_REL_RMS, "logits_img_maxabs": BF16_LOGIT_IMG_MAXABS,
                      "loss_rel": BF16_LOSS_REL, "grad_transformer": BF16_GRAD_REL_RMS_TRANSFORMER,
                      "grad_fe_stage_rel_rms": BF16_GRAD_REL_RMS_FE, "grad_fe_stage_cos": BF16_GRAD_COS_FE}}
    parity_record["c2_bf16_vs_oracle"] = rec
    print("C2 bf16 vs oracle:", {k: v for k, v in rec.items() if k != "logits_per_image_maxabs_frac"},
          f"max per-image frac {max(img_frac):.3e}")
    assert rel <= BF16_LOGIT_REL_RMS, rel
    assert max(img_frac) <= BF16_LOGIT_IMG_MAXABS, max(img_frac)
    assert loss_rel <= BF16_LOSS_REL, loss_rel
    assert rel_tr <= BF16_GRAD_REL_RMS_TRANSFORMER, rel_tr
    for st in stages:
        assert st["rel_rms"] <= BF16_GRAD_REL_RMS_FE and st["cos"] >= BF16_GRAD_COS_FE, st


# ------------------------------------------------------------------- C3
def _fe(depth, seed):
    import fpnmt
    from fpnmt.layers import Init
    from models.retinanet import FeatureExtractor
    fpnmt.set_precision("fp32")
    fe = FeatureExtractor(backbone=depth, init=Init(torch.Generator().manual_seed(seed)))
    sd = {"fe." + k: v.detach().float().clone() for k, v in fe.state_dict().items()}
    return fe.to(DEV), sd


def test_c3_r101_feature_extractor_512_fp32(parity_record):
    """C3's FeatureExtractor (ResNet-101 FPN, co-attention heads over P3-P7)
    at 512^2: the five level outputs of 2 images vs the oracle
    (retinanet.py:266-307 over keras-resnet ResNet101). The frozen
    identity-BN ResNet-101 grows activations with depth, so the bar is
    relative to each level's magnitude: 1e-4 of max |out|."""
    from oracle import ref_cpu as R
    fe, sd = _fe("resnet101", 101)
    img = _images(2, 512, seed=11)
    with torch.no_grad():
        outs = fe(img.to(DEV))
        ref = R.feature_extractor(sd, "fe", img, depth="resnet101")
    torch.cuda.synchronize()
    shapes = [(2, 32, 32, 512), (2, 16, 16, 512), (2, 8, 8, 512), (2, 4, 4, 512), (2, 2, 2, 512)]
    rec = {}
    for lvl, (o, r, s) in enumerate(zip(outs, ref, shapes)):
        assert tuple(o.shape) == s == tuple(r.shape), (lvl, o.shape, r.shape)
        err = float((o.cpu() - r).abs().max())
        mx = float(r.abs().max())
        print(f"C3 level P{lvl + 3}: max|d| {err:.3e}  max|ref| {mx:.3e}")
        rec[f"P{lvl + 3}"] = {"max_abs_delta": err, "max_abs_ref": mx, "rel": err / max(mx, 1e-30)}
    parity_record["c3_r101_512_fp32_levels"] = dict(rec, bar="1e-4 * max|ref| + 1e-6")
    for lvl, (o, r) in enumerate(zip(outs, ref)):
        err, mx = rec[f"P{lvl + 3}"]["max_abs_delta"], rec[f"P{lvl + 3}"]["max_abs_ref"]
        assert err <= 1e-4 * mx + 1e-6, lvl


def test_c3_bf16_batch64_properties():
    """The C3 configuration as benchmarked: bf16, batch 64, 512^2. The five
    FeatureExtractor outputs are finite, and the pyramid (ResNet-101 + FPN,
    P3-P7) of images 0-1 from the batch-64 bf16 run is within 5 % relative
    RMS of the fp32 path on the same weights. (The heads' outputs are not
    compared: with frozen identity BN the random-init score maps reach ~1e5,
    so the co-attention softmax is a hard arg-max over pixels that any
    bf16-level perturbation re-picks — a property of the model, which the
    fp32 test above pins at 1e-4.)"""
    import fpnmt
    from fpnmt import ops
    fe, _ = _fe("resnet101", 102)
    img = _images(64, 512, seed=12).to(DEV)
    with torch.no_grad():
        ref = [o.float() for o in fe.retinanet_model.pyramid(img[:2])]
        fpnmt.set_precision("bf16")
        try:
            outs = fe(img)
            pyr = fe.retinanet_model.pyramid(ops.cast(img, torch.bfloat16))
        finally:
            fpnmt.set_precision("fp32")
    torch.cuda.synchronize()
    for lvl, o in enumerate(outs):
        assert o.shape[0] == 64 and bool(torch.isfinite(o.float()).all()), lvl
    for lvl, (o, r) in enumerate(zip(pyr, ref)):
        assert o.shape[0] == 64 and bool(torch.isfinite(o.float()).all()), lvl
        rel = float((o[:2].float() - r).norm() / r.norm().clamp_min(1e-30))
        print(f"C3 bf16 pyramid P{lvl + 3}: rel RMS vs fp32 {rel:.3e}")
        assert rel <= 0.05, lvl


# ------------------------------------------------------------------- C5
def _oracle_predict_margins(sd, img, T, cfg, start, end, beam_n, detail=None):
    """oracle/ref_cpu.predict (utils/pipeline.py:82-154) with the relative
    gap between the kept and the first dropped candidate at every step, so
    a GPU/CPU divergence can be told apart from an fp32 near-tie. detail (a
    list) receives per step: the best beam's running probability after the
    step (pipeline.py:122,140; 0 once the product underflows, after which
    top_k only breaks ties among zeros) and the relative top-2 margin of
    the chosen token over its beam's runner-up, (p1 - p2) / p1."""
    from oracle import ref_cpu as R
    enc = R.encoder(sd, img[None], cfg).repeat(beam_n, 1, 1)
    V = sd["final_layer.kernel"].shape[1]
    out = torch.full((beam_n, 1), start, dtype=torch.int64)
    prob = torch.ones((beam_n, 1))
    margins, res = [], None
    for _ in range(T):
        lg, _ = R.transformer(sd, enc, out, False, R.create_look_ahead_mask(out.shape[1]), cfg)
        pr = torch.softmax(lg[:, -1, :], -1)
        cand = (pr * prob).reshape(-1)
        vals, idx = torch.sort(cand, descending=True, stable=True)
        top = float(vals[0])
        margins.append(abs(float(vals[beam_n - 1] - vals[beam_n])) / top if top > 0 else float("inf"))
        if detail is not None:
            # the token the best candidate extends its beam with vs that
            # beam's runner-up token (identical beams would tie each other)
            row = pr[int(idx[0]) // V].sort(descending=True).values
            detail.append({"best_beam_prob": top,
                           "top2_margin_rel": float((row[0] - row[1]) / row[0]) if row[0] > 0 else 0.0})
        vals, idx = vals[:beam_n], idx[:beam_n]
        ib = idx // V
        out = torch.cat([out[ib], (idx - ib * V)[:, None]], -1)
        prob = vals[:, None]
        res = out[int(torch.argmax(prob[:, 0]))]
        if int(res[-1]) == end:
            return res[1:-1].tolist(), margins
    return (res[1:-1] if int(res[-1]) == end else res[1:]).tolist(), margins


def _trained_pipeline(n_layers, vocab, T, n_img, seed, steps=300, lr=3e-4, n_captions=None, images="structured"):
    """lr: a constant or a utils.utils.CustomSchedule (the reference's warm-up
    schedule, on the device); n_captions: captions shared round-robin by the
    images (default one per image); images: "structured" (_structured_images:
    images the random frozen ResNet tells apart) or "noise" (U[-1, 1))."""
    return _trained_pipeline_impl(n_layers, vocab, T, n_img, seed, steps, lr, n_captions, images)


def _trained_pipeline_impl(n_layers, vocab, T, n_img, seed, steps, lr, n_captions=None, images="structured"):
    """A Pipeline whose model has memorised one caption per image: random-init
    weights give a near-uniform softmax whose running beam probability
    underflows to 0 within ~13 steps (every later token is then a tie among
    zeros), so the decode parity needs a model whose tokens are
    decided by its logits. n_img fixed images, each with its own caption
    <start> + (T - 3) random ids + <end> (+ one pad), trained with a
    constant-lr TrainEngine (bf16 graph steps, dropout 0) until its
    predictions are confident; returns (pipeline, images, captions, losses)
    with the fp32 parity mode set for the decode."""
    import fpnmt
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from utils.pipeline import Pipeline
    fpnmt.set_precision("bf16")
    pl = Pipeline(max_seq_len=T, target_vocab_size=vocab, image_size=224, n_layers=n_layers, rate=0.0,
                  init=Init(torch.Generator().manual_seed(seed)), use_graph=False)
    imgs = (_structured_images if images == "structured" else _images)(n_img, 224, seed=seed + 1)
    g = torch.Generator().manual_seed(seed + 2)
    tok = torch.zeros(n_img, T, dtype=torch.int64)
    nc = n_img if n_captions is None else n_captions
    caps = [torch.randint(4, vocab, (T - 3,), generator=g) for _ in range(nc)]
    for i in range(n_img):
        tok[i, 0] = pl.start_token
        tok[i, 1:T - 2] = caps[i % nc]
        tok[i, T - 2] = pl.end_token
    eng = TrainEngine(pl.transformer, lr, use_graph=True)
    di, dt = imgs.to(DEV), tok.to(DEV)
    losses = torch.stack([eng.step(di, dt).clone() for _ in range(steps)]).cpu().tolist()
    fpnmt.set_precision("fp32")
    return pl, imgs, tok, losses


def _decode_parity_trained(pl, imgs, tok, T, beam_n, cfg, key, parity_record, losses, batched=True, min_images=4,
                           min_memorised=0):
    """GPU decode of the trained model vs the oracle's literal predict():
    identical ids, and a record per image of the logit-decided steps (the
    best beam's running probability still > 0 and its top-2 candidates not
    tied), the distinct tokens and the top-2 margins."""
    sd = {k: v.detach().float().cpu().clone() for k, v in pl.transformer.state_dict().items()}
    if batched:
        ids = pl.predict_batch(imgs.to(DEV), T, beam_n=beam_n, use_graph=True)
    else:
        ids = [pl.predict(imgs[i].to(DEV), T)[0].cpu().tolist() for i in range(imgs.shape[0])]
    rec = {"train_loss_first_last": [losses[0], losses[-1]], "train_steps": len(losses), "images": []}
    ok = True
    with torch.no_grad():
        for i in range(imgs.shape[0]):
            detail = []
            ref, margins = _oracle_predict_margins(sd, imgs[i], T, cfg, pl.start_token, pl.end_token, beam_n, detail)
            decided = sum(1 for d in detail if d["best_beam_prob"] > 0 and d["top2_margin_rel"] > 1e-6)
            target = [int(t) for t in tok[i, 1:] if int(t) not in (0, pl.end_token)]
            rec["images"].append({
                "image": i, "identical": ids[i] == ref, "length": len(ref), "logit_decided_steps": decided,
                "distinct_tokens": len(set(ref)), "equals_memorised_caption": ref == target,
                "min_top2_margin_rel": min(d["top2_margin_rel"] for d in detail),
                "top2_margin_rel_per_step": [round(d["top2_margin_rel"], 6) for d in detail],
                "best_beam_prob_last": detail[-1]["best_beam_prob"], "gpu_ids": ids[i], "oracle_ids": ref})
            print(f"image {i}: identical {ids[i] == ref}, {decided} logit-decided steps, "
                  f"{len(set(ref))} distinct tokens, memorised {ref == target}")
            ok = ok and ids[i] == ref
    parity_record[key] = rec
    assert ok, [(r["gpu_ids"], r["oracle_ids"]) for r in rec["images"] if not r["identical"]]
    # discriminating: the tokens are decided by the logits, not by top_k's
    # tie-break among underflowed zeros (on at least min_images images; every
    # image's ids must be identical above)
    good = [r for r in rec["images"] if r["logit_decided_steps"] >= 24 and r["distinct_tokens"] >= 5]
    rec["images_logit_decided_ge24_distinct_ge5"] = len(good)
    assert len(good) >= min_images, [(r["logit_decided_steps"], r["distinct_tokens"]) for r in rec["images"]]
    # image-conditioned: images decoding their OWN memorised caption, and how
    # many different sequences the decode produced (one per image when the
    # tokens depend on the image; VERDICT r04 'weak' #1)
    mem = [r for r in rec["images"] if r["equals_memorised_caption"] and r["logit_decided_steps"] >= 24]
    rec["images_decoding_own_caption"] = len(mem)
    rec["distinct_decoded_sequences"] = len({tuple(r["oracle_ids"]) for r in rec["images"]})
    assert len(mem) >= min_memorised, (len(mem), min_memorised)
    assert rec["distinct_decoded_sequences"] >= min_memorised, rec["distinct_decoded_sequences"]


def test_c5_beam8_trained_decode_matches_oracle_fp32(parity_record):
    """C5's decode (beam 8, the C2 model: 6 layers, V = 10 000, 32 steps) of a
    model trained to give each of 6 structurally different images its OWN
    caption: the ids equal the oracle's literal predict(beam_n=8)
    (utils/pipeline.py:105-144) on all 6 images, >= 24 of their steps
    logit-decided, and >= 4 images decode their own memorised caption (so the
    decoded ids depend on the image: encoder and cross-attention included)."""
    from utils.utils import CustomSchedule
    T = 32
    # the 6-layer post-LN stack (fp32 and bf16 alike) collapses to the
    # caption's unigram distribution at a constant 1e-4 / 3e-4 or the warm-up
    # to 5e-4; the reference's CustomSchedule shape warming up over 400 steps
    # to 1e-4 memorises (tools/probes/train_c5.py, profiles/r04/train_c5.txt).
    # With _structured_images the 6 captions are learned apart: 6 / 6 images
    # decode their own caption after 1600 steps (loss 0.023,
    # tools/probes/train_cond.py, profiles/r05/train_cond.txt)
    pl, imgs, tok, losses = _trained_pipeline(6, V_C2, T, 6, seed=61, steps=1600, lr=CustomSchedule(156250, 400))
    assert losses[-1] < 0.5, f"6-layer model did not memorise its captions: loss {losses[0]:.3f} -> {losses[-1]:.3f}"
    cfg = dict(num_layers=6, num_heads=8, backbone="resnet50")
    _decode_parity_trained(pl, imgs, tok, T, 8, cfg, "c5_beam8_trained_fp32_vs_oracle", parity_record, losses,
                           min_memorised=4)


def test_greedy_trained_decode_matches_oracle_fp32(parity_record):
    """Pipeline.predict (BEAM_SEARCH_N = 4 identical beams == greedy,
    utils/pipeline.py:82-154) of a 2-layer model trained to give each of 4
    structurally different images its own caption, one image at a time,
    against the oracle's predict(beam_n=4): identical ids, and every image
    decodes its OWN caption (the ids depend on the image). With a constant
    3e-4 the 2-layer model reaches loss ~0.05 = ln(4) / 31, i.e. it cannot
    tell the images apart for the first token; the reference's warm-up
    schedule to 1e-4 separates them (4 / 4 after 1600 steps,
    tools/probes/train_cond.py 2L, profiles/r05/train_cond_2L.txt)."""
    from common.common_definitions import BEAM_SEARCH_N
    from utils.utils import CustomSchedule
    T = 32
    pl, imgs, tok, losses = _trained_pipeline(2, 1000, T, 4, seed=71, steps=1600, lr=CustomSchedule(156250, 400))
    cfg = dict(num_layers=2, num_heads=8, backbone="resnet50")
    _decode_parity_trained(pl, imgs, tok, T, BEAM_SEARCH_N, cfg, "greedy_2L_trained_fp32_vs_oracle", parity_record,
                           losses, batched=False, min_memorised=4)


def test_c5_beam8_decode_matches_oracle_fp32(parity_record):
    """C5's decode (beam 8, C2's model: 6 layers, V = 10 000, max_seq_len 32)
    on 4 images: token ids == the oracle's literal predict(beam_n=8). A
    divergence fails unless it lands on a step whose kept / first dropped
    candidates are tied to 1e-6 relative in fp32 (an fp32 tie that either
    side may break); every image's outcome, with the smallest candidate gap
    of its decode, goes to the parity record."""
    import fpnmt
    from fpnmt.layers import Init
    from utils.pipeline import Pipeline
    fpnmt.set_precision("fp32")
    T = 32
    pl = Pipeline(max_seq_len=T, target_vocab_size=V_C2, image_size=224, n_layers=6, rate=0.0,
                  init=Init(torch.Generator().manual_seed(31)), use_graph=False)
    sd = {k: v.detach().float().cpu().clone() for k, v in pl.transformer.state_dict().items()}
    cfg = dict(num_layers=6, num_heads=8, backbone="resnet50")
    imgs = _images(4, 224, seed=21)
    ids = pl.predict_batch(imgs.to(DEV), T, beam_n=8, use_graph=True)
    rec, fails = [], []
    with torch.no_grad():
        for i in range(4):
            detail = []
            ref, margins = _oracle_predict_margins(sd, imgs[i], T, cfg, pl.start_token, pl.end_token, 8, detail)
            ties = [j for j, mg in enumerate(margins) if mg <= 1e-6]
            # random-init weights: the running beam probability underflows
            # within ~13 steps; the later ids pin the reference's top_k
            # tie-break among zeros (the trained-model test below is the
            # logit-decided one)
            decided = sum(1 for d in detail if d["best_beam_prob"] > 0 and d["top2_margin_rel"] > 1e-6)
            if ids[i] != ref:
                k = next((j for j, (a, b) in enumerate(zip(ids[i], ref)) if a != b), min(len(ids[i]), len(ref)))
                print(f"image {i}: diverges at step {k}, oracle candidate gap {margins[k]:.2e}")
                rec.append({"image": i, "identical": False, "diverges_at_step": k, "gap_rel": margins[k],
                            "tie_steps": ties, "logit_decided_steps": decided, "gpu_ids": ids[i], "oracle_ids": ref})
                if margins[k] > 1e-6:
                    fails.append((i, k, margins[k]))
            else:
                print(f"image {i}: {len(ref)} ids identical (min gap {min(margins):.2e}, ties {ties})")
                rec.append({"image": i, "identical": True, "length": len(ref), "min_gap_rel": min(margins),
                            "tie_steps": ties, "logit_decided_steps": decided, "distinct_tokens": len(set(ref))})
    parity_record["c5_beam8_fp32_vs_oracle"] = rec
    assert not fails, fails


def test_c5_256_images_graph_equals_eager_bf16():
    """C5 as benchmarked: 256 images x beam 8 (2048 rows), bf16, one replayed
    hipGraph per decode step: ids identical to the eager (uncaptured) decode
    of the same model and images, twice (capture run and replay run)."""
    import fpnmt
    from fpnmt.layers import Init
    from utils.pipeline import Pipeline
    fpnmt.set_precision("bf16")
    try:
        T = 32
        pl = Pipeline(max_seq_len=T, target_vocab_size=V_C2, image_size=224, n_layers=6, rate=0.0,
                      init=Init(torch.Generator().manual_seed(32)), use_graph=False)
        imgs = _images(256, 224, seed=22).to(DEV)
        a = pl.predict_batch(imgs, T, beam_n=8, use_graph=False)
        b = pl.predict_batch(imgs, T, beam_n=8, use_graph=True)
        c = pl.predict_batch(imgs, T, beam_n=8, use_graph=True)
        assert len(a) == 256 and all(len(x) <= T for x in a)
        assert a == b == c
    finally:
        fpnmt.set_precision("fp32")
