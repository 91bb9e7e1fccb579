"""Diagnostic: where the bf16 training step's feature-extractor gradient
departs from the fp32 path's (C2 model, batch 32, one step, dropout 0).

Arms (each a fresh model of the same seed, one TrainEngine step):
  fp32          the reference arm
  fp32_w16      fp32 arithmetic on masters rounded to bf16 (the bf16 path's
                weight copies): the gradient's sensitivity to the weights'
                rounding alone
  bf16          the benchmarked arithmetic
  bf16_nofuse   bf16 with every backward fusion flag off (act' folds, summed
                consumer gradients, conv chains, deferred reductions)
  fp32_score16  fp32 arithmetic, the co-attention scores (the regression
                head's 1-channel output) rounded to bf16 before the softmax
Per arm vs fp32: relative RMS and cosine per exchange range and per
feature-extractor parameter tensor, and the fraction of the heads' 2x2
max-pool windows (after post_conv) whose argmax differs from fp32's.
  python tools/probes/bf16_grad_probe.py > out.txt"""
import json
import math
import os
import sys

sys.path[:0] = [os.path.join(os.getcwd(), "fpn-mt-image-captioning_amd"), os.getcwd(), os.path.join(os.getcwd(), "tests")]
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import ops  # noqa: E402
from fpnmt.train import TrainEngine  # noqa: E402
import test_gpu_configs as T  # noqa: E402

FLAGS = ["fuse_input_act", "fuse_block_act", "fuse_identity_residual", "fuse_grad_sums", "fuse_conv_chains",
         "defer_reductions", "fuse_residual_grads", "fuse_drop_ln", "fuse_ffn_act"]


def run(arm, img, tok):
    m, _, _ = T._model(6, T.V_C2, 224, 1234)
    if arm == "fp32_w16":
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(p.bfloat16().float())
    saved = {f: getattr(fpnmt.config, f) for f in FLAGS}
    if arm == "bf16_nofuse":
        for f in FLAGS:
            setattr(fpnmt.config, f, False)
    pools, scores = [], []
    orig = ops.max_pool2d_valid
    orig_ssm = ops.SpatialSoftmaxFn.apply

    def ssm(score, hs):
        scores.append(score.detach().float().cpu())
        if arm == "fp32_score16":
            score = score.bfloat16().float()
        return orig_ssm(score, hs)

    ops.SpatialSoftmaxFn.apply = ssm

    def rec(x, *a, **k):
        pools.append(x.detach().float().cpu())
        return orig(x, *a, **k)

    ops.max_pool2d_valid = rec
    import models.retinanet as MR
    MR.ops.max_pool2d_valid = rec
    fpnmt.set_precision("bf16" if arm.startswith("bf16") else "fp32")
    try:
        eng = TrainEngine(m, 1e-4, use_graph=False)
        loss = float(eng.step(img.cuda(), tok.cuda()))
        torch.cuda.synchronize()
        g = eng.arena.grad.detach().cpu().clone()
        names, offs = list(eng.arena.names), list(eng.arena.offsets)
        sizes = [p.numel() for p in eng.arena.params]
        ranges = list(eng.ranges)
    finally:
        fpnmt.set_precision("fp32")
        ops.max_pool2d_valid = orig
        MR.ops.max_pool2d_valid = orig
        ops.SpatialSoftmaxFn.apply = orig_ssm
        for f, v in saved.items():
            setattr(fpnmt.config, f, v)
    return dict(loss=loss, g=g, names=names, offs=offs, sizes=sizes, ranges=ranges, pools=pools, scores=scores)


def rel(a, b):
    return float((a - b).double().norm() / b.double().norm().clamp_min(1e-300))


def cos(a, b):
    return float((a.double() @ b.double()) / (a.double().norm() * b.double().norm()).clamp_min(1e-300))


def pool_argmax(x):
    n, h, w, c = x.shape
    x = x[:, :h // 2 * 2, :w // 2 * 2]
    x = x.reshape(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 5, 2, 4).reshape(n, h // 2, w // 2, c, 4)
    return x.argmax(-1)


def main():
    img, tok = T._images(32, 224), T._captions(32, T.V_C2)
    res = {a: run(a, img, tok) for a in ("fp32", "fp32_score16", "fp32_w16", "bf16", "bf16_nofuse")}
    ref = res["fp32"]
    out = {}
    for i, sc in enumerate(ref["scores"]):
        flat = sc.reshape(sc.shape[0], -1)
        spread = (flat.amax(1) - flat.amin(1))
        print(f"score level {i}: shape {tuple(sc.shape)} |score| max {float(sc.abs().max()):.3e}, "
              f"per-image max-min median {float(spread.median()):.3e}")
    for a in ("fp32_score16", "fp32_w16", "bf16", "bf16_nofuse"):
        r = res[a]
        rows = {"loss": r["loss"], "loss_fp32": ref["loss"], "ranges": []}
        for i, (s, e) in enumerate(r["ranges"]):
            if e > s:
                rows["ranges"].append({"range": i, "n": e - s, "rel_rms": rel(r["g"][s:e], ref["g"][s:e]),
                                       "cos": cos(r["g"][s:e], ref["g"][s:e])})
        per = []
        for n, o, sz in zip(r["names"], r["offs"], r["sizes"]):
            if not n.startswith("encoder.feature_extractor."):
                continue
            gr, gf = r["g"][o:o + sz], ref["g"][o:o + sz]
            if float(gf.norm()) == 0:
                continue
            per.append({"name": n[len("encoder.feature_extractor."):], "n": sz, "rel_rms": rel(gr, gf),
                        "cos": cos(gr, gf), "norm_fp32": float(gf.norm())})
        rows["fe_tensors"] = per
        flips = []
        for pa, pb in zip(r["pools"], ref["pools"]):
            if pa.shape == pb.shape and pa.numel():
                flips.append(float((pool_argmax(pa) != pool_argmax(pb)).float().mean()))
        rows["pool_argmax_flip_fraction_per_level"] = flips
        out[a] = rows
        print(f"== {a}: loss {r['loss']:.6f} (fp32 {ref['loss']:.6f}); pool argmax flips {[round(f, 4) for f in flips]}")
        for x in rows["ranges"]:
            print(f"   range {x['range']}: n {x['n']:>9}  rel_rms {x['rel_rms']:.4f}  cos {x['cos']:.4f}")
        per.sort(key=lambda x: x["cos"])
        print("   lowest-cosine feature-extractor tensors:")
        for x in per[:12]:
            print(f"     {x['name']:<60} n {x['n']:>8}  rel {x['rel_rms']:.3f}  cos {x['cos']:.3f}  |g| {x['norm_fp32']:.3e}")
        print("   highest-cosine:")
        for x in per[-5:]:
            print(f"     {x['name']:<60} n {x['n']:>8}  rel {x['rel_rms']:.3f}  cos {x['cos']:.3f}  |g| {x['norm_fp32']:.3e}")
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bf16_grad_probe.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
