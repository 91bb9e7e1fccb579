#!/usr/bin/env python3
"""Benchmark: training images/s of the FPN + multi-view-transformer training
step (BASELINE.json metric) on 1..N MI355X, one process per GPU.

Workload (BASELINE.json configs[1], "C2"): ResNet-50 FPN + 6-layer transformer,
224x224 images, per-GPU batch 32, captions T_pad=32 (decoder T=31), vocab
10000, bf16 MFMA compute with fp32 master weights / AMSGrad, dropout 0.1 —
the full step (forward, backward, per-tensor clip, AMSGrad, compute-weight
refresh; + RCCL gradient all-reduce for N>1) replayed as a hipGraph.
Synthetic data: images U[-1,1) (the mobilenet_v2
preprocess range), captions [<start>] + U{4..V-1}^(len-2) + [<end>], len ~
U{8..32}, zero padded; random-init weights (no checkpoints offline).

Extra objects on the JSON line:
  roofline      the dominant kernel (implicit-GEMM conv, the P3 subnet 3x3
                shape) timed live with HIP events on its stream
  cpu_baseline  the CPU oracle (oracle/ref_cpu.py, torch fp32) training step on
                this host's cores, rank 0 at N=1 only, bounded sample
  cpu_ref_logit_delta  max |logit_gpu(fp32 mode) - logit_cpu| on one image

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 under
torch.distributed.run (one rank per GPU, RCCL).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "training images/sec (FPN+transformer step) at 1/2/4/8 MI355X; CPU-ref logit Δ"
PEAK_BF16_TFLOPS = 2500.0
# the dominant kernel that roofline_probe times (the dispatch's choice for the
# P3 subnet conv at batch 32, csrc/gemm_dispatch.h pipe_cfg; the committed
# rocprofv3 summaries under profiles/ name it)
KERNEL_NAME = "gemm_pipe_lw_kernel<128,256,1,8,A_IM2COL,4,3,112>"
# analytic work: fwd MAC per image, R50-FPN + heads + 6L, 224, T=31, V=10k
FWD_GMAC_PER_IMG = 10.333
STEP_GFLOP_PER_IMG = 6 * FWD_GMAC_PER_IMG  # train = 3x fwd, 2 FLOP/MAC -> 62.0


def synthetic_batch(b, image, vocab, T, seed, device):
    g = torch.Generator().manual_seed(seed)
    img = torch.rand(b, image, image, 3, generator=g) * 2 - 1
    tok = torch.randint(4, vocab, (b, T), generator=g, dtype=torch.int64)
    tok[:, 0] = 2
    lens = torch.randint(8, T + 1, (b,), generator=g)
    for i in range(b):
        L = int(lens[i])
        tok[i, L - 1] = 3
        tok[i, L:] = 0
    return img.to(device), tok.to(torch.int32).to(device)


def roofline_probe(batch, iters=20, dtype=torch.bfloat16):
    """Dominant kernel: the 3x3 256->256 'same' conv on P3 (28x28 at 224^2) —
    the regression/classification subnet convs, the largest kernel family
    (SURVEY.md App. B). Timed with HIP events on the launching stream."""
    from fpnmt.layers import Conv2D
    conv = Conv2D(256, 256, 3, padding="same", activation="relu", kernel_initializer="normal").cuda()
    x = torch.randn(batch, 28, 28, 256, device="cuda").to(dtype)
    # `iters` back-to-back launches captured in one hipGraph (no host launch
    # gaps between them: eager launches read 2-2.5 us per launch above the
    # rocprofv3 average of the same kernel, round 6), the median of 5 timed
    # replays (after the step loop the clock can sit lower for a while)
    rounds = []
    with torch.no_grad():
        for _ in range(3):
            conv(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                conv(x)
        g.replay()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            g.replay()
            e1.record(st)
            torch.cuda.synchronize()
            rounds.append(e0.elapsed_time(e1) / iters)
    ms = sorted(rounds)[len(rounds) // 2]
    m, n, k = batch * 28 * 28, 256, 9 * 256
    flop = 2.0 * m * n * k
    achieved = flop / (ms * 1e-3) / 1e12
    # HBM bytes per launch from the committed PMC passes of this same kernel
    # and launch (pmc/roofline_pmc.json: rocprofv3 FETCH_SIZE / WRITE_SIZE,
    # gfx950-corrected); attached only when the record names this kernel
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "pmc", "roofline_pmc.json")
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))
            if rec.get("kernel") == KERNEL_NAME and rec.get("launch", "").endswith(f"M={m} N={n} K={k}"):
                traffic, traffic_src = rec.get("hbm_bytes_per_launch"), "pmc/roofline_pmc.json"
        except Exception:
            traffic = None
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
            "traffic_source": traffic_src, "algorithmic_bytes": 2 * (m * k // 9 + k * n + m * n),
            "kernel": KERNEL_NAME + " (implicit-GEMM conv fwd at a 112-row M step: 224 tiles, 8 MFMA waves of 112x32 (v_mfma_f32_16x16x32_bf16, LDS fragment reads only) + 4 loader waves owning the LDS-DMA of a 3-stage 128x256 ring, 16-B epilogue stores)",
            "launch": f"conv3x3 256->256 on {batch}x28x28, M={m} N={n} K={k}, {flop / 1e9:.1f} GFLOP/launch",
            "avg_launch_ms": round(ms, 4)}


def _graph_time(fn, iters):
    """Capture fn() once as a hipGraph, replay it iters times; ms per replay
    (HIP events on the replay stream)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        g.replay()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def headline_probe(batch=64, image=224, iters=10):
    """BASELINE north_star target: ResNet-50-FPN forward (backbone + FPN
    P3..P7, retinanet.py:105-141 on keras-resnet C3..C5), 224^2, batch 64,
    bf16, vs the dense bf16 MFMA peak. Work: 9.354 GFLOP/img (SURVEY §8d,
    analytic conv MACs x 2)."""
    from fpnmt.layers import Init
    from models.retinanet import FeatureExtractor
    fe = FeatureExtractor(backbone="resnet50", init=Init(torch.Generator().manual_seed(3))).cuda()
    x = (torch.rand(batch, image, image, 3, device="cuda") * 2 - 1).to(torch.bfloat16)
    with torch.no_grad():
        ms = _graph_time(lambda: fe.retinanet_model.pyramid(x), iters)
    gflop = 9.354 * batch
    tf = gflop / (ms * 1e-3) / 1e3
    return {"workload": f"ResNet-50-FPN forward (backbone + FPN P3-P7), {image}x{image}, batch {batch}, bf16, "
                        "hipGraph replay", "ms": round(ms, 3), "gflop": round(gflop, 1), "tflops": round(tf, 1),
            "mfma_frac": round(tf / PEAK_BF16_TFLOPS, 4), "images_per_s": round(batch / (ms * 1e-3), 1)}


def c3_probe(batch=64, image=512, iters=5):
    """BASELINE configs[2] (C3): ResNet-101 FPN FeatureExtractor forward at
    512^2, batch 64 — backbone, FPN, the shared 5-level heads and the
    co-attention over P3..P7. Work: 129.5 GFLOP/img."""
    from fpnmt.layers import Init
    from models.retinanet import FeatureExtractor
    fe = FeatureExtractor(backbone="resnet101", init=Init(torch.Generator().manual_seed(4))).cuda()
    x = torch.rand(batch, image, image, 3, device="cuda") * 2 - 1
    with torch.no_grad():
        ms = _graph_time(lambda: fe(x), iters)
    gflop = 129.5 * batch
    tf = gflop / (ms * 1e-3) / 1e3
    del fe
    return {"workload": f"C3: ResNet-101 FPN FeatureExtractor forward (backbone, FPN, 5-level heads, co-attention "
                        f"P3-P7), {image}x{image}, batch {batch}, bf16, hipGraph replay",
            "ms": round(ms, 3), "images_per_s": round(batch / (ms * 1e-3), 1), "tflops": round(tf, 1),
            "mfma_frac": round(tf / PEAK_BF16_TFLOPS, 4)}


def c5_probe(n_images=256, beam_n=8, T_max=32, image=224, layers=6, vocab=10000):
    """BASELINE configs[4] (C5): reference beam search (beam 8) batched over
    256 images — encoder once per image, then max_seq_len decode steps of
    2048 rows, each step one replayed hipGraph (KV cache, fpnmt_beam_step).
    Timed end to end (encoder + all steps) after one warm run; random-init
    weights rarely emit <end>, so all T_max steps run."""
    import fpnmt
    from fpnmt.decode import BeamDecoder
    from fpnmt.layers import Init
    from models.transformer import Transformer
    fpnmt.set_precision("bf16")
    tr = Transformer(layers, 512, 8, 2048, math.ceil(image / 16) ** 2, vocab, 0.0, max_seq_len=T_max,
                     init=Init(torch.Generator().manual_seed(6))).cuda()
    dec = BeamDecoder(tr, n_images, beam_n, T_max, 2, 3, use_graph=True)
    imgs = torch.rand(n_images, image, image, 3, device="cuda") * 2 - 1
    with torch.no_grad():
        dec.decode(imgs, check_every=0)  # captures the step graphs
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = dec.decode(imgs, check_every=0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    steps = T_max
    gflop_step = 2 * 27.1e-3 * n_images * beam_n  # 2 x 27.1 M MAC per row per step (6L, V=10k)
    del dec, tr
    torch.cuda.empty_cache()
    return {"workload": f"C5: beam-{beam_n} batched decode, {n_images} images {image}x{image}, R50-FPN + {layers}L, "
                        f"V={vocab}, {steps} steps, KV cache, hipGraph per step, bf16",
            "ms": round(dt * 1e3, 2), "images_per_s": round(n_images / dt, 1),
            "decode_steps": steps, "mean_len": round(sum(len(o) for o in out) / len(out), 2),
            "step_gflop": round(gflop_step, 1)}


def input_pipeline_probe(n=256, src=(480, 640), size=224, iters=20, decode_n=64, threads=16):
    """SURVEY §8f #2 (dataset.py:19-26): the batched resize + preprocess
    kernel over n resident decoded COCO-sized images (HIP events on the
    launching stream), the host JPEG decode rate on a thread pool, and the
    CPU restatement's resize + preprocess per image (oracle/image_ref.py)."""
    import io
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from PIL import Image
    from fpnmt import input_pipeline as IP
    from oracle import image_ref as OR
    rng = np.random.default_rng(7)
    base = rng.integers(0, 256, (src[0], src[1], 3), dtype=np.uint8)
    imgs = [np.roll(base, i, axis=1) for i in range(n)]
    pixels, items, max_w = IP.pack_images(imgs, pin=True)
    pd, idev = pixels.cuda(), items.cuda()
    out = torch.empty((n, size, size, 3), device="cuda")
    IP.resize_normalize_packed(pd, idev, n, max_w, size, size, out=out)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        IP.resize_normalize_packed(pd, idev, n, max_w, size, size, out=out)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    in_bytes = n * src[0] * src[1] * 3
    out_bytes = out.numel() * 4
    gbs = (in_bytes + out_bytes) / (ms * 1e-3) / 1e9
    # host decode of COCO-sized JPEGs
    jpgs = []
    for i in range(decode_n):
        b = io.BytesIO()
        Image.fromarray(imgs[i]).save(b, format="JPEG", quality=90)
        jpgs.append(b.getvalue())
    with ThreadPoolExecutor(threads) as pool:
        list(pool.map(IP.decode_image, jpgs[:threads]))
        t0 = time.perf_counter()
        list(pool.map(IP.decode_image, jpgs))
        dec_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    k = 8
    for i in range(k):
        OR.load_image_pixels(imgs[i], size)
    cpu_s = (time.perf_counter() - t0) / k
    return {"workload": f"resize (TF2 bilinear, half-pixel) + mobilenet preprocess, {n} decoded "
                        f"{src[0]}x{src[1]} RGB images -> ({n}, {size}, {size}, 3) fp32, one launch",
            "kernel_ms": round(ms, 4), "images_per_s": round(n / (ms * 1e-3), 1),
            "hbm": {"achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s", "frac": round(gbs / 8000.0, 4),
                    "bytes_per_launch": in_bytes + out_bytes,
                    "note": "algorithmic: every source byte once + fp32 output"},
            "host_jpeg_decode": {"images_per_s": round(decode_n / dec_s, 1), "threads": threads,
                                 "sample": f"{decode_n} JPEGs {src[0]}x{src[1]} q90, Pillow (libjpeg)"},
            "cpu_oracle_resize_ms_per_image": round(cpu_s * 1e3, 2)}


def cpu_model_name():
    """lscpu's "Model name" (from /proc/cpuinfo)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def c1_decode_latency(cores):
    """BASELINE configs[0] (C1) on the CPU oracle: R50-FPN + 2-layer
    transformer, 224^2, batch 1, greedy decode of at most 32 tokens (the
    oracle's greedy recomputes the full prefix each step, like the
    reference's predict()). ms per image."""
    from oracle import ref_cpu as R
    from fpnmt.layers import Init
    from models.transformer import Transformer
    torch.set_num_threads(cores)
    m = Transformer(2, 512, 8, 2048, 196, 10000, 0.0, max_seq_len=32, init=Init(torch.Generator().manual_seed(8)))
    sd = {k: v.float() for k, v in m.state_dict().items()}
    cfg = dict(num_layers=2, num_heads=8, backbone="resnet50")
    img = torch.rand(224, 224, 3, generator=torch.Generator().manual_seed(9)) * 2 - 1
    with torch.no_grad():
        R.greedy(sd, img, 2, cfg, 2, 3)  # warm
        t0 = time.time()
        ids = R.greedy(sd, img, 32, cfg, 2, 3)
        dt = time.time() - t0
    return {"ms_per_image": round(dt * 1e3, 1), "tokens": int(ids.numel()), "cores": cores,
            "workload": "C1: oracle/ref_cpu.py greedy decode, R50-FPN + 2L, 224x224, batch 1, <= 32 steps, "
                        "full-prefix recompute, fp32"}


def cpu_baseline(seconds_budget=20.0):
    """CPU oracle train step (fp32, torch eager on this host's cores) on a
    bounded sample of the same workload (batch 4)."""
    from oracle import ref_cpu as R
    from fpnmt.layers import Init
    from models.transformer import Transformer
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cores = max(1, min(cores, os.cpu_count() or 1))
    torch.set_num_threads(cores)
    m = Transformer(6, 512, 8, 2048, 196, 10000, 0.0, max_seq_len=32, init=Init(torch.Generator().manual_seed(5)))
    sd = {k: v.float() for k, v in m.state_dict().items()}
    trainable = {n for n, p in m.named_parameters()}
    cfg = dict(num_layers=6, num_heads=8, backbone="resnet50")
    b = 4
    img, tok = synthetic_batch(b, 224, 10000, 32, 99, "cpu")
    tok = tok.long()
    opt = R.KerasAMSGrad(sorted(trainable), [sd[n].shape for n in sorted(trainable)],
                         sparse=["decoder.embedding.embeddings"])
    params = dict(sd)

    def step():
        loss, _, grads, ess = R.loss_and_grads(params, img, tok, cfg, trainable)
        opt.apply(params, grads, R.custom_schedule, norms={"decoder.embedding.embeddings": ess})

    t0 = time.time()
    step()  # warmup
    first = time.time() - t0
    n = max(1, min(5, int(seconds_budget / max(first, 1e-3))))
    t0 = time.time()
    for _ in range(n):
        step()
    dt = time.time() - t0
    return {"value": round(b * n / dt, 3), "unit": "images/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model_name(),
            "sample": f"oracle/ref_cpu.py fp32 train step (fwd+bwd+Keras AMSGrad), same C2 model, batch {b}, "
                      f"{n} timed steps after 1 warmup ({dt:.1f} s)",
            "c1_decode": c1_decode_latency(cores)}


def step_probe(args, batch, precision, steps, warmup=2, split=False):
    """The training step at another per-GPU batch / precision (extra bench
    objects: C4's per-GPU batch 64 on one GPU, and the fp32 parity mode).
    split=True: the step C4 runs on every GPU (TrainEngine's world > 1 form:
    G1 forward + decoder backward, G2 encoder layers, one graph per feature-
    extractor stage, G3 update; the exchanges are empty at world 1), with one
    more step's per-graph timeline."""
    import fpnmt
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from models.transformer import Transformer
    from utils.utils import CustomSchedule
    prev = fpnmt.compute_dtype()
    fpnmt.set_precision(precision)
    try:
        model = Transformer(args.layers, 512, 8, 2048, math.ceil(args.image / 16) ** 2, args.vocab, args.dropout,
                            max_seq_len=32, backbone=args.backbone,
                            init=Init(torch.Generator().manual_seed(1234))).cuda()
        eng = TrainEngine(model, CustomSchedule(2048, 4000), use_graph=True, split_backward=split)
        img, tok = synthetic_batch(batch, args.image, args.vocab, 32, 2000, "cuda")
        for _ in range(warmup):
            eng.step(img, tok)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = eng.step(img, tok)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        out = {"per_gpu_batch": batch, "precision": precision, "ms_per_step": round(dt * 1e3, 3),
               "images_per_s": round(batch / dt, 2), "steps": steps, "loss": round(float(loss.item()), 5)}
        if split:
            eng.enable_timeline()
            eng.step(img, tok)
            tl = eng.timeline()[-1]
            eng.enable_timeline(False)
            prev_end, seg = 0.0, {}
            for g in tl["graphs"]:
                seg[g["name"]] = round(g["end_ms"] - prev_end, 4)
                prev_end = g["end_ms"]
            out["graphs"] = len(eng.graphs)
            out["graph_ms"] = seg  # per replayed graph (G1, G2, S1..S5, waits, G3), from the events between them
        del eng, model
        torch.cuda.empty_cache()
    finally:
        fpnmt.set_precision(prev)
    return out


def logit_delta(model, image=224):
    """fp32-mode GPU logits vs the CPU oracle on one image (same weights)."""
    import fpnmt
    from oracle import ref_cpu as R
    from models.transformer import create_masks
    prev = fpnmt.compute_dtype()
    fpnmt.set_precision("fp32")
    try:
        img, tok = synthetic_batch(1, image, 10000, 32, 7, "cuda")
        tar = tok[:, :-1]
        with torch.no_grad():  # inference split (training=False): no dropout, like the oracle
            enc = model.encoder(img, False, None)
            lg, _ = model(enc, tar, False, create_masks(tar))
        torch.cuda.synchronize()
        sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
        cfg = dict(num_layers=len(model.decoder.dec_layers), num_heads=8, backbone="resnet50")
        ref, _ = R.transformer(sd, img.cpu(), tar.cpu().long(), True, R.create_masks(tar.cpu().long()), cfg)
        return float((lg.cpu() - ref).abs().max()), float(ref.abs().max())
    finally:
        fpnmt.set_precision(prev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (weak scaling); default 32 on one GPU (C2), 64 per GPU on N > 1 "
                         "(C4: global 512 at 8 GPUs)")
    ap.add_argument("--bf16-buckets", action="store_true", help="all-reduce gradient buckets in bf16 (opt-in)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-only", action="store_true")
    ap.add_argument("--headline-only", action="store_true", help="ResNet-50-FPN fwd batch 64 only")
    ap.add_argument("--c3-only", action="store_true", help="C3 R101-FPN FeatureExtractor 512^2 only")
    ap.add_argument("--no-extra", action="store_true", help="skip the headline / C3 / C5 probes")
    ap.add_argument("--c5-only", action="store_true", help="C5 batched beam decode only")
    ap.add_argument("--input-only", action="store_true", help="input pipeline (resize + preprocess) only")
    ap.add_argument("--backbone", default="resnet50")
    ap.add_argument("--side-wgrad", default=None, choices=["off", "dense", "all"],
                    help="weight gradients on a second stream (default: fpnmt.config.side_wgrad)")
    ap.add_argument("--fuse-identity", default=None, choices=["on", "off"],
                    help="identity-bottleneck gradient sum in the bwd-data epilogue (default: fpnmt.config.fuse_identity_residual)")
    ap.add_argument("--fuse-block-act", default=None, choices=["on", "off"],
                    help="previous bottleneck's ReLU' in the identity block's bwd-data epilogue (default: fpnmt.config.fuse_block_act)")
    ap.add_argument("--fuse-prep", default=None, choices=["on", "off"],
                    help="compute-copy refresh inside the AMSGrad kernel (default: fpnmt.config.fuse_optimizer_prep)")
    ap.add_argument("--defer", default=None, choices=["on", "off"],
                    help="batched deferred gradient reductions (default: fpnmt.config.defer_reductions)")
    ap.add_argument("--zero-grad-grid", type=int, default=None,
                    help="workgroups of the side-stream gradient-arena fill beside the forward; 0 = inline "
                         "(default: fpnmt.config.zero_grad_overlap_grid)")
    ap.add_argument("--early-update", default=None, choices=["on", "off"],
                    help="transformer's optimizer part beside the feature extractor's backward "
                         "(default: fpnmt.config.early_update)")
    ap.add_argument("--timeline", default=None,
                    help="N > 1: directory for each rank's exchange timeline (rank<r>.json) of one extra step")
    args = ap.parse_args()

    import fpnmt
    from fpnmt import dist as fdist
    fpnmt._lib.assert_in_tree()
    rank, world, local = fdist.init_from_env()  # FPNMT_DIST_BACKEND=gloo: a one-GPU rehearsal of N > 1
    backend = torch.distributed.get_backend() if world > 1 else None
    torch.cuda.set_device(fdist.device_for_local_rank(local))
    fpnmt.set_precision(args.precision)
    if args.side_wgrad is not None:
        fpnmt.config.side_wgrad = False if args.side_wgrad == "off" else args.side_wgrad
    if args.defer is not None:
        fpnmt.config.defer_reductions = args.defer == "on"
    if args.early_update is not None:
        fpnmt.config.early_update = args.early_update == "on"
    if args.zero_grad_grid is not None:
        fpnmt.config.zero_grad_overlap_grid = args.zero_grad_grid
    if args.fuse_prep is not None:
        fpnmt.config.fuse_optimizer_prep = args.fuse_prep == "on"
    if args.fuse_identity is not None:
        fpnmt.config.fuse_identity_residual = args.fuse_identity == "on"
    if args.fuse_block_act is not None:
        fpnmt.config.fuse_block_act = args.fuse_block_act == "on"
    if args.batch is None:
        args.batch = 32 if world == 1 else 64

    if args.roofline_only:
        r = roofline_probe(args.batch)
        print(json.dumps({"roofline": r}))
        return
    if args.c5_only:
        print(json.dumps({"c5_decode": c5_probe()}))
        return
    if args.headline_only:
        print(json.dumps({"headline_r50fpn_fwd": headline_probe()}))
        return
    if args.input_only:
        print(json.dumps({"input_pipeline": input_pipeline_probe()}))
        return
    if args.c3_only:
        print(json.dumps({"c3_fe_fwd": c3_probe()}))
        return

    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from models.transformer import Transformer
    from utils.utils import CustomSchedule

    T_pad = 32
    model = Transformer(args.layers, 512, 8, 2048, math.ceil(args.image / 16) ** 2, args.vocab, args.dropout,
                        max_seq_len=T_pad, backbone=args.backbone,
                        init=Init(torch.Generator().manual_seed(1234))).cuda()
    eng = TrainEngine(model, CustomSchedule(2048, 4000), use_graph=not args.no_graph,
                      bucket_dtype=torch.bfloat16 if args.bf16_buckets else None)
    img, tok = synthetic_batch(args.batch, args.image, args.vocab, T_pad, 1000 + rank, "cuda")

    for _ in range(args.warmup):
        eng.step(img, tok)
    torch.cuda.synchronize()
    if world > 1:
        fdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = eng.step(img, tok)
    torch.cuda.synchronize()
    if world > 1:
        fdist.barrier()
    torch.cuda.synchronize()
    dt = fdist.allreduce_max_scalar(time.perf_counter() - t0)
    loss_v = float(loss.item()) if loss is not None else float("nan")
    timeline = None
    if world > 1 and eng.split and eng.use_graph:
        # one more (untimed) replayed step with HIP events around every stage
        # graph and every range's exchange: the per-rank overlap picture
        eng.enable_timeline()
        eng.step(img, tok)
        timeline = eng.timeline()[-1]
        eng.enable_timeline(False)
        if args.timeline:
            os.makedirs(args.timeline, exist_ok=True)
            with open(os.path.join(args.timeline, f"rank{rank}.json"), "w") as f:
                json.dump(timeline, f)
        ends = {g["name"]: g["end_ms"] for g in timeline["graphs"]}
        last_stage = max(v for k, v in ends.items() if k.startswith(("G1", "G2", "S")))
        exposed = fdist.allreduce_max_scalar(ends["waits"] - last_stage)
        timeline["exposed_exchange_ms_max_over_ranks"] = round(exposed, 4)

    out = None
    if rank == 0:
        ms = dt / args.steps * 1e3
        value = world * args.batch * args.steps / dt
        step_tflops = STEP_GFLOP_PER_IMG * args.batch / (ms * 1e-3) / 1e3
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if args.precision == "bf16" else "fp32",
            "data": "synthetic: U[-1,1) 224x224 images, random-token captions (T_pad 32), random-init weights",
            "config": {"workload": (f"{'C2' if world == 1 else 'C4'}: ResNet-50 FPN + {args.layers}-layer "
                                    f"transformer, {args.image}x{args.image}, per-GPU batch {args.batch}, T=31, "
                                    f"V={args.vocab}, full training step (fwd+bwd+clip+AMSGrad), dropout "
                                    f"{args.dropout}, hipGraph replay"
                                    + ("" if world == 1 else
                                       (", RCCL all-reduce per backward stage, overlapped" if backend == "nccl" else
                                        f", {backend} all-reduce per backward stage (one-GPU rehearsal, "
                                        "not a scaling point)"))),
                       "per_gpu_batch": args.batch,
                       "global_batch": args.batch * world, "seq_len": T_pad - 1,
                       "parallelism": f"dp{world}"},
            "loss": round(loss_v, 5),
            "step_tflops": round(step_tflops, 2),
            "step_mfma_frac": round(step_tflops / PEAK_BF16_TFLOPS, 4),
        }
    if rank == 0 and timeline is not None:
        out["exchange_timeline_rank0"] = timeline
    if rank == 0 and world == 1:
        out["roofline"] = roofline_probe(args.batch)

        if not args.no_cpu_baseline:
            try:
                out["cpu_ref_logit_delta"], out["cpu_ref_logit_absmax"] = logit_delta(model, args.image)
            except Exception as e:  # report, never hide
                out["cpu_ref_logit_delta"] = f"error: {e}"
            out["cpu_baseline"] = cpu_baseline()
        if not args.no_extra:
            del eng, model
            torch.cuda.empty_cache()
            # C4's per-GPU work (batch 64) on one GPU: the N=1 point of a
            # weak-scaling curve at the multi-GPU default batch
            out["c4_per_gpu_b64"] = step_probe(args, 64, "bf16", 10)
            # the form C4 actually runs per GPU (8 graph replays per step)
            sp = step_probe(args, 64, "bf16", 10, split=True)
            sp["overhead_vs_single_graph"] = round(sp["ms_per_step"] / out["c4_per_gpu_b64"]["ms_per_step"] - 1, 4)
            out["c4_split_step_b64"] = sp
            out["fp32_mode_step"] = step_probe(args, args.batch, "fp32", 5, warmup=3)
            out["headline_r50fpn_fwd"] = headline_probe()
            out["c3_fe_fwd"] = c3_probe()
            out["c5_decode"] = c5_probe()
            out["input_pipeline"] = input_pipeline_probe()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
