"""Model-level parity on the GPU against the CPU oracle (oracle/ref_cpu.py):
fp32 logits within 1e-3, train-step loss / gradients / updated parameters,
greedy-decode token ids bit-exact (with the top-2 margin reported), the
hipGraph-replayed step equal to the eager step, and the bf16 perf mode
staying close to fp32.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _build(num_layers=2, vocab=500, image=224, max_seq_len=32, seed=1234, backbone="resnet50", rate=0.0):
    import fpnmt
    from fpnmt.layers import Init
    from models.transformer import Transformer
    fpnmt.set_precision("fp32")
    torch.manual_seed(seed)
    m = Transformer(num_layers, 512, 8, 2048, math.ceil(image / 16) ** 2, vocab, rate, max_seq_len=max_seq_len,
                    backbone=backbone, init=Init(torch.Generator().manual_seed(seed)))
    sd = {k: v.detach().float().clone() for k, v in m.state_dict().items()}
    return m.to(DEV), sd, dict(num_layers=num_layers, num_heads=8, backbone=backbone)


def _inputs(b=2, image=224, vocab=500, T=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    img = torch.rand(b, image, image, 3, generator=g) * 2 - 1
    tok = torch.randint(4, vocab, (b, T), generator=g)
    tok[:, 0] = 2
    for i in range(b):
        L = int(torch.randint(8, T + 1, (1,), generator=g))
        tok[i, L - 1] = 3
        tok[i, L:] = 0
    return img, tok


def test_forward_logits_parity_fp32():
    from oracle import ref_cpu as R
    from models.transformer import create_masks
    m, sd, cfg = _build()
    img, tok = _inputs()
    tar = tok[:, :-1]
    with torch.no_grad():
        logits, w = m(img.to(DEV), tar.to(DEV), True, create_masks(tar.to(DEV)))
    ref, wr = R.transformer(sd, img, tar, True, R.create_masks(tar), cfg)
    torch.cuda.synchronize()
    err = float((logits.cpu() - ref).abs().max())
    print(f"fp32 logit max|delta| = {err:.3e}")
    assert err <= 1e-3
    for key in wr:
        assert float((w[key].cpu() - wr[key]).abs().max()) <= 1e-4, key


@pytest.mark.parametrize("image", [128, 224])
def test_train_step_parity_fp32(image, parity_record):
    """Loss, every parameter gradient and the parameters after two AMSGrad
    steps. Gradients are anchored on an fp64 run of the oracle: the GPU fp32
    error must be within 3x (bulk; 10x at the max) the fp32 noise floor — the
    larger error of two fp32 oracle runs, the second on the input perturbed by
    ~1 ulp — the frozen-BN ResNet's backbone gradients are ill-conditioned
    enough that fp32 on any device is ~1e-2 off fp64 at 224^2
    (tests/test_gpu_parts.py)."""
    _train_step_parity(1, 300, image, parity_record, f"train_step_1L_V300_{image}")


@pytest.mark.timeout(1200)
def test_train_step_parity_c2_model_fp32(parity_record):
    """The same two-step check on the full C2 model (ResNet-50 FPN + 6-layer
    transformer, V = 10 000, 224^2) at batch 2: every one of its parameter
    gradients against the fp64 oracle, and the parameters after two AMSGrad
    steps (utils/pipeline.py:64-80, Keras AMSGrad + per-tensor clipnorm).

    The bulk (90th-percentile) bar is taken over three inputs — the test's
    and two copies perturbed by ~1 ulp — on both sides: the median of the
    GPU's errors within 3x the median of the fp32 oracle's (+1e-5 of max).
    At the single original input the GPU's P4-path bias gradients sat 8.5x
    above the oracle's (round 3); tools/probes/p4_chain.py traced that to ONE
    scalar, the co-attention score gradient at the near-one-hot softmax peak
    of level P4, whose error comes from the upstream gradient's routing
    through 2x2 max pools that are fp32 ties (fp64 top-2 gaps ~1e-14: the
    GPU and the CPU break ~120 of them differently), not from any kernel's
    arithmetic (the spatial-softmax backward is within 3e-8 of fp64 on the
    same operands; every forward tensor is more accurate than the CPU
    oracle's); at the perturbed inputs the GPU's error on the same gradients
    is 0.4-1.2x the oracle's (profiles/r04/p4_chain.txt)."""
    _train_step_parity(6, 10000, 224, parity_record, "train_step_c2_6L_V10000_224_b2", n_inputs=3)


def _perturbed(img, seed):
    """img with every element moved by ~1 ulp (random sign)."""
    gp = torch.Generator().manual_seed(seed)
    sgn = torch.randint(0, 2, img.shape, generator=gp).float() * 2 - 1
    return img * (1 + sgn * 2.0 ** -23)


def _train_step_parity(num_layers, vocab, image, parity_record, key, bulk_floor=1e-5, n_inputs=1):
    from oracle import ref_cpu as R
    from fpnmt.train import TrainEngine
    lr = 1e-4
    m, sd, cfg = _build(num_layers=num_layers, vocab=vocab, image=image)
    trainable = [n for n, p in m.named_parameters() if p.requires_grad]
    img, tok = _inputs(b=2, vocab=vocab, image=image)
    rec = {"params": len(trainable)}
    inputs = [img] + [_perturbed(img, 77 + j) for j in range(n_inputs - 1)]
    gpu_sets = None
    if n_inputs > 1:
        # GPU gradients at every input from the initial parameters (an lr-0
        # engine leaves them unchanged); the live engine below starts afresh
        eng0 = TrainEngine(m, 0.0, use_graph=False)
        gpu_sets = []
        for x in inputs:
            eng0.step(x.to(DEV), tok.to(DEV))
            torch.cuda.synchronize()
            gpu_sets.append({n: p.grad.detach().cpu().double().clone() for n, p in m.named_parameters()})
        del eng0
    eng = TrainEngine(m, lr, use_graph=False)  # constant lr: the schedule's first steps are ~0
    emb = "decoder.embedding.embeddings"
    opts = {dt: R.KerasAMSGrad(trainable, [sd[n].shape for n in trainable], sparse=[emb], dtype=dt)
            for dt in (torch.float32, torch.float64)}
    params = {dt: {k: v.to(dt).clone() for k, v in sd.items()} for dt in opts}
    for step in range(2):
        ref = {dt: R.loss_and_grads(params[dt], img.to(dt), tok, cfg, set(trainable)) for dt in opts}
        loss = eng.step(img.to(DEV), tok.to(DEV))
        torch.cuda.synchronize()
        loss_ref, loss64 = float(ref[torch.float32][0]), float(ref[torch.float64][0])
        if step == 0:  # identical parameters: only forward arithmetic differs
            assert abs(float(loss) - loss_ref) <= 1e-4 * max(1.0, abs(loss_ref)), step
        else:  # after an update the fp32 trajectories themselves differ: anchor on fp64
            assert abs(float(loss) - loss64) <= 3 * abs(loss_ref - loss64) + 2e-4 * max(1.0, abs(loss64)), step
        if step == 0:
            g32, g64 = ref[torch.float32][2], ref[torch.float64][2]
            # fp32 noise floor of this model at this input: the fp32 oracle
            # again on the image perturbed by ~1 ulp (random sign). The
            # frozen-BN ResNet / co-attention softmax amplify rounding-level
            # forward differences (ReLU kinks, near-tied pools, summation
            # order) into the gradients; one fp32 run can land close to fp64
            # by chance, so the max anchor is the largest of the fp32 errors
            # (n_inputs > 1: the bulk bar compares medians over the inputs)
            cpu_sets = [g32] + [R.loss_and_grads(params[torch.float32], x, tok, cfg, set(trainable))[2]
                                for x in (inputs[1:] if n_inputs > 1 else [_perturbed(img, 77)])]
            if gpu_sets is not None:
                # the live engine's first step reproduces the lr-0 engine's (bitwise determinism)
                assert all(torch.equal(gpu_sets[0][n], p.grad.detach().cpu().double())
                           for n, p in m.named_parameters())
            rows, bulk = [], []
            zero = {}  # structurally-zero gradients: absolute errors (relative ones are noise / ~0)
            for (n, p) in m.named_parameters():
                t = g64[n]
                mx = float(t.abs().max())
                # absolute errors; the 1e-7 floor covers structurally-zero
                # gradients (e.g. the regression-head bias, whose output only
                # enters a shift-invariant spatial softmax: true grad 0)
                dg = (p.grad.detach().cpu().double() - t).abs()
                dc = torch.stack([(cs[n].double() - t).abs() for cs in cpu_sets]).amax(0)
                eg, ec = float(dg.max()), float(dc.max())
                if mx < 1e-7:
                    zero[n] = {"fp64_max_abs": mx, "gpu_max_abs": eg, "cpu_fp32_max_abs": ec}
                # max error: a ReLU kink or a max-pool near-tie decided the
                # other way than fp64 (a ~1e-6 forward difference) reroutes
                # one output channel's gradient, i.e. a whole weight-gradient
                # column; which of two fp32 runs hits one is chance. The max
                # bar leaves room for that; the bulk (90th percentile) bar is
                # the 3x-the-fp32-oracle one.
                rows.append((eg - 10 * ec - 1e-2 * mx - 1e-7, eg / max(mx, 1e-30), ec / max(mx, 1e-30), n))
                if t.numel() >= 16:
                    def p90(d, big):
                        return float(torch.quantile(d.flatten().float(), 0.9)) if d.numel() < 2 ** 24 else big
                    if gpu_sets is None:
                        qg, qc = p90(dg, eg), p90(dc, ec)
                    else:  # medians over the inputs, on both sides
                        qg = sorted(p90((gs[n] - t).abs(), eg) for gs in gpu_sets)[n_inputs // 2]
                        qc = sorted(p90((cs[n].double() - t).abs(), ec) for cs in cpu_sets)[n_inputs // 2]
                    bulk.append((qg - 3 * qc - bulk_floor * mx - 1e-8, qg / max(mx, 1e-30), qc / max(mx, 1e-30), n))
            rows.sort(reverse=True)
            bulk.sort(reverse=True)
            for r in sorted(rows, key=lambda r: -r[1])[:3]:
                print("grad max rel err vs fp64: gpu %.2e  cpu32 %.2e  %s" % r[1:])
            for r in sorted(bulk, key=lambda r: -r[1])[:3]:
                print("grad p90 rel err vs fp64: gpu %.2e  cpu32 %.2e  %s" % r[1:])
            for r in bulk[:8]:  # closest to the bar (excess over 3x the fp32 oracle)
                print("grad p90 excess %.2e: gpu %.2e  cpu32 %.2e  %s" % r)
            rec["loss_step0_gpu"], rec["loss_step0_oracle32"] = float(loss), loss_ref
            # relative errors (of the tensor's max |fp64 grad|) over the tensors
            # with a nonzero gradient; the structurally-zero ones (attention
            # key biases under the shift-invariant softmax, the regression-head
            # bias) recorded by absolute error
            rec["grad_max_rel_err_vs_fp64_worst"] = [
                {"param": r[3], "gpu": r[1], "cpu_fp32": r[2]}
                for r in sorted(rows, key=lambda r: -r[1]) if r[3] not in zero][:5]
            rec["grad_p90_rel_err_vs_fp64_worst"] = [
                {"param": r[3], "gpu": r[1], "cpu_fp32": r[2]}
                for r in sorted(bulk, key=lambda r: -r[1]) if r[3] not in zero][:5]
            rec["grad_structurally_zero"] = zero
            rec["grad_tensors_checked"] = len(rows)
            rec["bulk_bar"] = (f"p90 gpu <= 3 x p90 cpu_fp32 + {bulk_floor:g} x max, "
                               + ("one input" if n_inputs == 1 else f"medians over {n_inputs} inputs (1 ulp perturbed)"))
            assert rows[0][0] <= 0.0, rows[0]
            assert bulk[0][0] <= 0.0, bulk[0]
        for dt, o in opts.items():
            o.apply(params[dt], ref[dt][2], lambda it: lr, norms={emb: ref[dt][3]})
    # Adam normalises each element, so ill-conditioned gradient elements can
    # move by up to ~2*alpha apart between ANY two fp32 runs: require the
    # elementwise bound, and the mean deviation from the fp64 trajectory to be
    # within 3x that of the fp32 CPU oracle.
    alphas = [lr * math.sqrt(1 - 0.98 ** t) / (1 - 0.9 ** t) for t in (1, 2)]
    bound = 2.0 * sum(alphas)
    dev_g, dev_c, tot = 0.0, 0.0, 0
    for n, p in m.named_parameters():
        t = params[torch.float64][n]
        pg = p.detach().cpu().double()
        assert float((pg - params[torch.float32][n].double()).abs().max()) <= bound, n
        dev_g += float((pg - t).abs().sum())
        dev_c += float((params[torch.float32][n].double() - t).abs().sum())
        tot += p.numel()
    print(f"mean |param - fp64 trajectory|: gpu {dev_g / tot:.3e}  cpu32 {dev_c / tot:.3e}")
    rec["params_after_2_steps_mean_abs_dev_vs_fp64"] = {"gpu": dev_g / tot, "cpu_fp32": dev_c / tot}
    parity_record[key] = rec
    assert dev_g <= 3 * dev_c + 1e-9 * tot


def test_greedy_decode_parity_fp32(parity_record):
    from oracle import ref_cpu as R
    from utils.pipeline import Pipeline
    import fpnmt
    fpnmt.set_precision("fp32")
    from fpnmt.layers import Init
    pl = Pipeline(max_seq_len=12, target_vocab_size=200, image_size=224, n_layers=2, rate=0.0,
                  init=Init(torch.Generator().manual_seed(7)), use_graph=False)
    sd = {k: v.detach().float().cpu().clone() for k, v in pl.transformer.state_dict().items()}
    cfg = dict(num_layers=2, num_heads=8, backbone="resnet50")
    g = torch.Generator().manual_seed(3)
    for i in range(2):
        img = torch.rand(224, 224, 3, generator=g) * 2 - 1
        ids, _ = pl.predict(img.to(DEV), 12)
        ref = R.predict(sd, img, 12, cfg, 2, 3)
        greedy = R.greedy(sd, img, 12, cfg, 2, 3)
        assert torch.equal(ref, greedy)  # reference beam procedure == greedy
        parity_record.setdefault("greedy_2L_V200_ids", []).append(
            {"image": i, "gpu": ids.cpu().tolist(), "oracle": ref.tolist(), "identical": ids.cpu().tolist() == ref.tolist()})
        assert ids.cpu().tolist() == ref.tolist(), (ids.tolist(), ref.tolist())


def test_graph_step_matches_eager():
    """The replayed hipGraph step reproduces the eager step. Both engines are
    put in the identical state (parameters, AMSGrad m/v/v-hat, step counter)
    before every step and compared one step at a time: the loss of the same
    parameters, and the parameter update. The frozen-BN ResNet is chaotic
    over several steps (fp32 split-K atomics noise grows ~10x per step), so a
    free-running multi-step comparison would measure that chaos, not the
    graph; a missed, stale or doubled update would be of the order of the
    update itself."""
    from fpnmt.train import TrainEngine
    from fpnmt import layers as flayers
    m_e, _, _ = _build(num_layers=1, vocab=300, seed=11)
    m_g, _, _ = _build(num_layers=1, vocab=300, seed=11)
    E = TrainEngine(m_e, 1e-6, use_graph=False)
    G = TrainEngine(m_g, 1e-6, use_graph=True)
    img, tok = _inputs(b=2, vocab=300, seed=5)
    img, tok = img.to(DEV), tok.to(DEV)
    state = ("flat", "m", "v", "vhat", "step")
    for i in range(4):
        if i:
            with torch.no_grad():
                for nme in state:
                    getattr(G.arena, nme).copy_(getattr(E.arena, nme))
            flayers.prepare_all(G.model)  # refresh G's compute copies in place
            # allocation noise between replays: a graph that reads memory it
            # does not own (or relies on a node that does not re-run, e.g. a
            # captured hipMemsetAsync) picks up these 1e30s
            junk = [torch.full((1 << 26,), 1e30, device=DEV) for _ in range(8)]
            torch.cuda.synchronize()
            del junk
        p0 = E.arena.flat.detach().clone()
        le = float(E.step(img, tok))
        lg = float(G.step(img, tok))
        torch.cuda.synchronize()
        de = E.arena.flat - p0
        dg = G.arena.flat - p0
        upd = float(de.abs().mean())
        err = float((de - dg).abs().mean())
        print(f"step {i}: loss eager {le:.7f} graph {lg:.7f}; mean |update| {upd:.3e}, mean |d update| {err:.3e}")
        assert abs(le - lg) <= 1e-5 * max(1.0, abs(le)), (i, le, lg)
        assert upd > 0
        assert err <= 0.02 * upd, (i, upd, err)
        assert torch.equal(E.arena.step, G.arena.step)


def test_split_backward_step_matches_single_graph():
    """The data-parallel step structure (G1 forward + transformer backward,
    G2 feature-extractor backward, G3 update; what overlaps the RCCL
    all-reduce with backward at world > 1) run at world 1 equals the single
    graph step, one step at a time from identical state."""
    from fpnmt.train import TrainEngine
    from fpnmt import layers as flayers
    m_a, _, _ = _build(num_layers=1, vocab=300, seed=12)
    m_b, _, _ = _build(num_layers=1, vocab=300, seed=12)
    A = TrainEngine(m_a, 1e-6, use_graph=True)
    B = TrainEngine(m_b, 1e-6, use_graph=True, split_backward=True)
    assert B.split and not A.split and A.arena.names == B.arena.names
    img, tok = _inputs(b=2, vocab=300, seed=6)
    img, tok = img.to(DEV), tok.to(DEV)
    for i in range(4):
        if i:
            with torch.no_grad():
                for nme in ("flat", "m", "v", "vhat", "step"):
                    getattr(B.arena, nme).copy_(getattr(A.arena, nme))
            flayers.prepare_all(B.model)
        p0 = A.arena.flat.detach().clone()
        la = float(A.step(img, tok))
        lb = float(B.step(img, tok))
        torch.cuda.synchronize()
        da, db = A.arena.flat - p0, B.arena.flat - p0
        upd = float(da.abs().mean())
        err = float((da - db).abs().mean())
        print(f"step {i}: loss {la:.7f} / {lb:.7f}; mean |update| {upd:.3e}, mean |d update| {err:.3e}")
        assert abs(la - lb) <= 1e-5 * max(1.0, abs(la))
        assert upd > 0 and err <= 0.02 * upd


def test_fp32_logits_after_graph_bf16_steps():
    """bench.py's parity leg: bf16 hipGraph training steps, then the first
    fp32 forward of the same model (fresh fp32 compute copies, incl. the
    stacked operands of the grouped projections) against the CPU oracle on
    the model's own state dict (fp32 logits within 1e-3)."""
    import fpnmt
    from oracle import ref_cpu as R
    from fpnmt.train import TrainEngine
    from models.transformer import create_masks
    m, _, cfg = _build(num_layers=1, vocab=300, seed=21, rate=0.1)
    fpnmt.set_precision("bf16")
    try:
        eng = TrainEngine(m, 1e-4, use_graph=True)
        img, tok = _inputs(b=4, vocab=300, seed=8)
        for _ in range(3):
            eng.step(img.to(DEV), tok.to(DEV))
        torch.cuda.synchronize()
        fpnmt.set_precision("fp32")
        img1, tok1 = _inputs(b=1, vocab=300, seed=9)
        tar = tok1[:, :-1]
        with torch.no_grad():
            enc = m.encoder(img1.to(DEV), False, None)
            lg, _ = m(enc, tar.to(DEV), False, create_masks(tar.to(DEV)))
        sd = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
        ref, _ = R.transformer(sd, img1, tar, True, R.create_masks(tar), cfg)
        err = float((lg.cpu() - ref).abs().max())
        print(f"fp32 logits after graph steps: max |d| {err:.2e} (|logits| {float(ref.abs().max()):.2f})")
        assert err <= 1e-3
    finally:
        fpnmt.set_precision("fp32")


def test_bf16_step_close_to_fp32():
    from fpnmt.train import TrainEngine
    import fpnmt
    res = {}
    for prec in ("fp32", "bf16"):
        m, sd, cfg = _build(num_layers=1, vocab=300, seed=21)
        fpnmt.set_precision(prec)
        eng = TrainEngine(m, 1e-4, use_graph=(prec == "bf16"))
        img, tok = _inputs(b=4, vocab=300, seed=9)
        res[prec] = [float(eng.step(img.to(DEV), tok.to(DEV))) for _ in range(3)]
    fpnmt.set_precision("fp32")
    print("fp32", res["fp32"], "bf16", res["bf16"])
    for a, b in zip(res["fp32"], res["bf16"]):
        assert math.isfinite(b) and abs(a - b) <= 0.03 * abs(a)


@pytest.mark.parametrize("arena", [False, True])
def test_fused_projections_match_unfused(arena):
    """Grouped projection GEMMs (fpnmt.config.fuse_projections) give the same
    loss and gradients as one Dense per projection, with the parameters in
    separate tensors (per-member fallbacks) and in a group-ordered arena
    (one bias column-sum / one batched bwd-filter GEMM per group)."""
    import fpnmt
    from fpnmt.arena import ParamArena
    from fpnmt.layers import group_param_order
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    res = {}
    for fuse in (False, True):
        m, sd, cfg = _build(num_layers=2, vocab=300, image=128, seed=3)
        if arena:
            named = group_param_order(m, [(n, p) for n, p in m.named_parameters() if p.requires_grad])
            ParamArena(named, DEV, sparse_names=["decoder.embedding.embeddings"])
        fpnmt.config.fuse_projections = fuse
        try:
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
        finally:
            fpnmt.config.fuse_projections = True
        res[fuse] = (float(loss), {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()
                                   if p.grad is not None})
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) <= 1e-5 * max(1.0, abs(l0))
    # a projection of the empty (0x0) view gets no gradient tensor on one path
    # and an all-zero one on the other: compare over the union, missing = 0
    for n in set(g0) ^ set(g1):
        t = g0.get(n, g1.get(n))
        assert float(t.abs().max()) == 0.0, n
        g0.setdefault(n, torch.zeros_like(t))
        g1.setdefault(n, torch.zeros_like(t))
    worst = max(((float((g1[n] - g0[n]).abs().max()) - 1e-3 * float(g0[n].abs().max()) - 1e-7), n) for n in g0)
    assert worst[0] <= 0, worst


@pytest.mark.parametrize("prec,graph", [("fp32", False), ("bf16", True)])
def test_train_step_bitwise_deterministic(prec, graph):
    """Every gradient reduction of the step (split-K weight gradients, bias /
    LayerNorm column sums, embedding scatter, CE loss, per-tensor norms) is
    fixed-order: the same step from the same state gives bitwise-identical
    parameters, AMSGrad state and loss, eager and graph-replayed."""
    import fpnmt
    from fpnmt.train import TrainEngine
    m, _, _ = _build(num_layers=2, vocab=300, seed=41, rate=0.1 if graph else 0.0)  # eager: fresh dropout seeds per call
    fpnmt.set_precision(prec)
    try:
        eng = TrainEngine(m, 1e-4, use_graph=graph)
        img, tok = _inputs(b=4, vocab=300, seed=10)
        img, tok = img.to(DEV), tok.to(DEV)
        eng.step(img, tok)  # warm (first call is eager; captures on the next when graph)
        names = ("flat", "m", "v", "vhat", "step")
        s0 = {n: getattr(eng.arena, n).clone() for n in names}
        runs = []
        for _ in range(2):
            with torch.no_grad():
                for n in names:
                    getattr(eng.arena, n).copy_(s0[n])
            from fpnmt import layers as flayers
            flayers.prepare_all(m)
            loss = eng.step(img, tok).clone()
            torch.cuda.synchronize()
            runs.append((loss, {n: getattr(eng.arena, n).clone() for n in names}))
        (l0, a0), (l1, a1) = runs
        assert torch.equal(l0, l1), (float(l0), float(l1))
        for n in names:
            assert torch.equal(a0[n], a1[n]), n
        assert not torch.equal(a0["flat"], s0["flat"])  # the step did update
    finally:
        fpnmt.set_precision("fp32")


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_fused_conv_chains_bitwise_equal(prec):
    """ops.conv_chain (bottleneck 2a->2b->2c, submodel convs -> heads, grouped
    over the levels) fuses each intermediate's ReLU derivative into the
    bwd-data epilogue: loss and every gradient equal the layer-by-layer
    Conv2dFn / ConvGroupedFn path bit for bit."""
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    fpnmt.set_precision(prec)
    res = {}
    fpnmt.config.fuse_identity_residual = False  # an autograd add on both sides (own test below)
    try:
        for fuse in (False, True):
            m, _, _ = _build(num_layers=2, vocab=300, image=128, seed=3)
            fpnmt.config.fuse_conv_chains = fuse
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_conv_chains = True
        fpnmt.config.fuse_identity_residual = True
        fpnmt.set_precision("fp32")
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1), (float(l0), float(l1))
    assert set(g0) == set(g1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_identity_residual_gradient_fused(prec):
    """keras-resnet identity bottlenecks (models/resnet.py: x is conv 2a's
    input and 2c's residual): x's two gradients summed in 2a's bwd-data
    epilogue (fpnmt_conv2d_bwd_data_res) equal bwd-data + the autograd add:
    bit for bit in fp32 (one fp32 rounding either way), within bf16 rounding
    of the sum in bf16 (one rounding instead of two)."""
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    fpnmt.set_precision(prec)
    res = {}
    try:
        for fuse in (False, True):
            m, _, _ = _build(num_layers=1, vocab=300, image=128, seed=5)
            fpnmt.set_precision(prec)
            fpnmt.config.fuse_identity_residual = fuse
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_identity_residual = True
        fpnmt.set_precision("fp32")
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)  # forward unchanged
    bb = [n for n in g0 if "backbone" in n]
    assert bb
    for n in g0:
        if prec == "fp32":
            assert torch.equal(g0[n], g1[n]), n
        else:
            d = float((g0[n] - g1[n]).abs().max())
            mx = float(g0[n].abs().max())
            assert d <= 3e-2 * max(mx, 1e-30) + 1e-30, (n, d, mx)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_block_act_fused_bitwise_equal(prec, monkeypatch):
    """The previous bottleneck's output ReLU' applied in the identity block's
    fused bwd-data epilogue (fpnmt_conv2d_bwd_data_res_act; the producing
    chain then skips its act_bwd pass) gives the same gradients as the
    separate pass, bit for bit in both precisions (a 0/1 factor after the
    same rounding), and the fused form is actually taken."""
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    calls = {}
    real_call = ops.call

    def counting_call(name, *a):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *a)

    monkeypatch.setattr(ops, "call", counting_call)
    res, counts = {}, {}
    try:
        for fuse in (False, True):
            calls.clear()
            m, _, _ = _build(num_layers=1, vocab=300, image=128, seed=5)
            fpnmt.set_precision(prec)
            fpnmt.config.fuse_block_act = fuse
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            counts[fuse] = dict(calls)
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_block_act = True
        fpnmt.set_precision("fp32")
    fused = counts[True].get("fpnmt_conv2d_bwd_data_res_act", 0)
    assert fused >= 8, counts[True]  # every identity block after another bottleneck (R50: 12)
    assert counts[True].get("fpnmt_act_bwd", 0) == counts[False].get("fpnmt_act_bwd", 0) - fused
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_input_act_fused_equal(prec, monkeypatch):
    """A conv's input that is another conv's ReLU output (the ResNet stage
    outputs C2..C5 under the next stage's strided projection block and the FPN
    laterals, the stem under its max pool, P6_conv under its pool): every
    consumer multiplies its contribution by that ReLU' in its bwd-data
    epilogue (fpnmt_conv2d_bwd_data_mask, accumulating and scattered too) or
    in the pool's backward (fpnmt_maxpool2d_bwd_act), and the producer skips
    its act_bwd pass. Loss and every gradient equal the unfused path in value
    (torch.equal: a masked zero may carry the other sign), in both precisions."""
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    calls = {}
    real_call = ops.call

    def counting_call(name, *a):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *a)

    monkeypatch.setattr(ops, "call", counting_call)
    res, counts = {}, {}
    try:
        for fuse in (False, True):
            calls.clear()
            m, _, _ = _build(num_layers=1, vocab=300, image=128, seed=7)
            fpnmt.set_precision(prec)
            fpnmt.config.fuse_input_act = fuse
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            counts[fuse] = dict(calls)
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_input_act = True
        fpnmt.set_precision("fp32")
    masked = counts[True].get("fpnmt_conv2d_bwd_data_mask", 0)
    # R50: C2 (2 strided consumers), C3 / C4 (2 strided + the lateral), C5 (lateral)
    assert masked >= 8, counts[True]
    assert counts[True].get("fpnmt_maxpool2d_bwd_act", 0) >= 2, counts[True]  # stem, P6_conv, coatt conv
    assert counts[True].get("fpnmt_conv2d_bwd_data_grouped_mask", 0) >= 2, counts[True]  # both head chains
    saved = counts[False].get("fpnmt_act_bwd", 0) - counts[True].get("fpnmt_act_bwd", 0)
    assert saved >= 6, (counts[False].get("fpnmt_act_bwd"), counts[True].get("fpnmt_act_bwd"))
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)
    assert set(g0) == set(g1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("split,mode", [(False, "dense"), (True, "dense"), (False, "all")])
def test_side_stream_wgrad_bitwise_equal(split, mode):
    """Weight gradients on the side stream (fpnmt.config.side_wgrad, forked and
    joined inside the captured backward) give the same step as the
    single-stream backward, bit for bit: parameters, AMSGrad state, loss."""
    import fpnmt
    from fpnmt import layers as flayers
    from fpnmt.train import TrainEngine
    img, tok = _inputs(b=4, vocab=300, seed=12)
    img, tok = img.to(DEV), tok.to(DEV)
    fpnmt.set_precision("bf16")
    res = {}
    try:
        fpnmt.config.defer_reductions = False  # single-stream: it turns the side stream off
        for side in (False, mode):
            fpnmt.config.side_wgrad = side
            m, _, _ = _build(num_layers=2, vocab=300, seed=43, rate=0.1)
            eng = TrainEngine(m, 1e-4, use_graph=True, split_backward=split)
            losses = [eng.step(img, tok).clone() for _ in range(3)]  # eager, capture + replay, replay
            torch.cuda.synchronize()
            res[side] = (torch.stack(losses), {n: getattr(eng.arena, n).clone() for n in ("flat", "m", "v", "vhat")})
            del eng, m
            flayers.invalidate_weights()
    finally:
        fpnmt.config.side_wgrad = False
        fpnmt.config.defer_reductions = True
        fpnmt.set_precision("fp32")
    (l0, a0), (l1, a1) = res[False], res[mode]
    assert torch.equal(l0, l1), (l0, l1)
    for n in a0:
        assert torch.equal(a0[n], a1[n]), n


@pytest.mark.parametrize("split,arena", [(False, None), (True, None), (False, 1 << 20)])
def test_deferred_reductions_bitwise_equal(split, arena):
    """fpnmt_defer_begin/_flush (the TrainEngine's backward: split-K weight-
    gradient reduces and bias / LayerNorm column sums queued and batched at
    the end of each backward graph) give the immediate-mode step bit for bit
    over eager, captured and replayed steps. arena: a 1 MiB deferred arena,
    so most slabs and partials fall back to the process scratch and their
    sums run immediately between queued ones (the fallback's
    colsum touches the queue first)."""
    import fpnmt
    from fpnmt import _lib
    from fpnmt import layers as flayers
    from fpnmt.train import TrainEngine
    img, tok = _inputs(b=4, vocab=300, seed=13)
    img, tok = img.to(DEV), tok.to(DEV)
    fpnmt.set_precision("bf16")
    res = {}
    saved = (_lib.DEFER_BYTES, dict(_lib._defer))
    if arena is not None:
        _lib.DEFER_BYTES = arena
        _lib._defer.clear()
    try:
        for defer in (False, True):
            fpnmt.config.defer_reductions = defer
            m, _, _ = _build(num_layers=2, vocab=300, seed=44, rate=0.1)
            eng = TrainEngine(m, 1e-4, use_graph=True, split_backward=split)
            losses = [eng.step(img, tok).clone() for _ in range(3)]
            torch.cuda.synchronize()
            res[defer] = (torch.stack(losses), {n: getattr(eng.arena, n).clone() for n in ("flat", "m", "v", "vhat")})
            del eng, m
            flayers.invalidate_weights()
    finally:
        fpnmt.config.defer_reductions = True
        fpnmt.set_precision("fp32")
        _lib.DEFER_BYTES = saved[0]
        _lib._defer.clear()
        _lib._defer.update(saved[1])
    (l0, a0), (l1, a1) = res[False], res[True]
    assert torch.equal(l0, l1), (l0, l1)
    for n in a0:
        assert torch.equal(a0[n], a1[n]), n


def test_zero_grad_overlap_bitwise_equal():
    """The gradient arena's zero fill as a small-grid trickle on a side stream
    beside the forward (config.zero_grad_overlap_grid, joined before the
    backward) gives the inline fill's losses, weights and optimizer state bit
    for bit over eager, captured and replayed steps; the arena really is
    zeroed every step (a poisoned arena changes nothing)."""
    import fpnmt
    from fpnmt import layers as flayers
    from fpnmt.train import TrainEngine
    img, tok = _inputs(b=4, vocab=300, seed=19)
    img, tok = img.to(DEV), tok.to(DEV)
    fpnmt.set_precision("bf16")
    res = {}
    keep = fpnmt.config.zero_grad_overlap_grid
    try:
        for grid in (0, 7):
            fpnmt.config.zero_grad_overlap_grid = grid
            m, _, _ = _build(num_layers=2, vocab=300, seed=46, rate=0.1)
            eng = TrainEngine(m, 1e-4, use_graph=True)
            eng.arena.grad.fill_(3.0)  # stale gradients must not leak into step 1
            losses = [eng.step(img, tok).clone() for _ in range(3)]
            torch.cuda.synchronize()
            res[grid] = (torch.stack(losses), {n: getattr(eng.arena, n).clone() for n in ("flat", "m", "v", "vhat")})
            del eng, m
            flayers.invalidate_weights()
    finally:
        fpnmt.config.zero_grad_overlap_grid = keep
        fpnmt.set_precision("fp32")
    (l0, a0), (l1, a1) = res[0], res[7]
    assert torch.equal(l0, l1), (l0, l1)
    for n in a0:
        assert torch.equal(a0[n], a1[n]), n


def test_early_update_bitwise_equal():
    """The transformer's clip + AMSGrad on a second stream from inside the
    backward (config.early_update: ops.transformer_grads_barrier ->
    TrainEngine._early_update, the feature extractor's part at the end) gives
    the one-launch update's losses, weights and optimizer state bit for bit
    over eager, captured and replayed steps, and the early part really ran
    (the barrier's callback fired once per step, on the leading blocks)."""
    import fpnmt
    from fpnmt import layers as flayers
    from fpnmt.train import TrainEngine
    img, tok = _inputs(b=4, vocab=300, seed=17)
    img, tok = img.to(DEV), tok.to(DEV)
    fpnmt.set_precision("bf16")
    res, fired = {}, {}
    try:
        for early in (False, True):
            fpnmt.config.early_update = early
            m, _, _ = _build(num_layers=2, vocab=300, seed=45, rate=0.1)
            eng = TrainEngine(m, 1e-4, use_graph=True)
            assert 0 < eng.early_blocks < eng.arena.nblocks
            calls = []
            orig = eng._early_update
            eng._early_update = lambda: (calls.append(1), orig())
            losses = [eng.step(img, tok).clone() for _ in range(3)]
            torch.cuda.synchronize()
            fired[early] = len(calls)
            res[early] = (torch.stack(losses), {n: getattr(eng.arena, n).clone() for n in ("flat", "m", "v", "vhat")},
                          int(eng.arena.step.item()))
            del eng, m
            flayers.invalidate_weights()
    finally:
        fpnmt.config.early_update = False
        fpnmt.set_precision("fp32")
    # eager step + the capture run the Python callback; replays run the graph
    assert fired[False] == 0 and fired[True] == 2, fired
    (l0, a0, s0), (l1, a1, s1) = res[False], res[True]
    assert s0 == s1 == 3
    assert torch.equal(l0, l1), (l0, l1)
    for n in a0:
        assert torch.equal(a0[n], a1[n]), n


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_drop_ln_fused_bitwise_equal(prec, monkeypatch):
    """The dropout backward of every `LN(res + dropout(dense))` sublayer end
    written by the LayerNorm backward (fpnmt_layernorm_bwd_drop; the Dense
    then skips its act_bwd pass) gives the same loss and gradients as the
    separate pass, bit for bit in both precisions (the same mask applied to
    the same stored dx), and the fused form is actually taken: decoder
    mha1 / mha2 / ffn2 and encoder ffn2 per layer."""
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    calls = {}
    real_call = ops.call

    def counting_call(name, *a):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *a)

    monkeypatch.setattr(ops, "call", counting_call)
    res, counts = {}, {}
    try:
        for fuse in (False, True):
            calls.clear()
            m, _, _ = _build(num_layers=2, vocab=300, image=128, seed=5, rate=0.1)
            fpnmt.set_precision(prec)
            fpnmt.config.fuse_drop_ln = fuse
            ops.runtime.reset_sites()
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            counts[fuse] = dict(calls)
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_drop_ln = True
        fpnmt.set_precision("fp32")
    fused = counts[True].get("fpnmt_layernorm_bwd_drop", 0)
    assert fused == 2 * 3 + 2 * 1, counts[True]
    assert counts[False].get("fpnmt_layernorm_bwd_drop", 0) == 0
    assert counts[True].get("fpnmt_act_bwd", 0) == counts[False].get("fpnmt_act_bwd", 0) - fused
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)
    assert set(g0) == set(g1)
    bad = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_view_norms_fused_match_per_view(prec, monkeypatch):
    """The Encoder's five view LayerNorms (+ posenc, dropout) as one launch per
    pass (fpnmt_layernorm_views_fwd / _bwd) against one LayerNormFn +
    DropoutFn per view: same loss and gradients bit for bit (same rows, same
    masks), except the shared LayerNorm's gamma / beta, whose five per-view
    column sums may be added in another order (fp32 rounding only); and the
    grouped form replaces the 10 + 10 per-view launches. The Decoder's
    embedding dropout (same flag) runs inside the embedding launches.""" 
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    calls = {}
    real_call = ops.call

    def counting_call(name, *a):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *a)

    monkeypatch.setattr(ops, "call", counting_call)
    res, counts = {}, {}
    try:
        for fuse in (False, True):
            calls.clear()
            m, _, _ = _build(num_layers=2, vocab=300, image=128, seed=5, rate=0.1)
            fpnmt.set_precision(prec)
            fpnmt.config.fuse_view_norms = fuse
            ops.runtime.reset_sites()
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            counts[fuse] = dict(calls)
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_view_norms = True
        fpnmt.set_precision("fp32")
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)
    assert set(g0) == set(g1)
    for n in g0:
        if n.startswith("encoder.layernorm1."):
            d = float((g0[n] - g1[n]).abs().max())
            assert d <= 1e-6 * float(g0[n].abs().max()) + 1e-30, (n, d)
        else:
            assert torch.equal(g0[n], g1[n]), n
    assert counts[True].get("fpnmt_layernorm_views_fwd", 0) == 1
    assert counts[True].get("fpnmt_layernorm_views_bwd", 0) == 1
    # at 128^2 the views are 8x8, 4x4, 2x2, 1x1 and 0x0 (no dropout launch):
    # 4 forward + 4 backward dropout launches folded into the grouped passes,
    # and the decoder embedding's 2 into the embedding launches
    assert counts[False].get("fpnmt_dropout", 0) == 10
    assert counts[True].get("fpnmt_dropout", 0) == 0
    assert counts[True].get("fpnmt_embed_posenc_fwd_drop", 0) == 1


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_ffn_act_fused_matches(prec, monkeypatch):
    """ffn1's LeakyReLU backward applied in ffn2's bwd-data epilogue
    (fpnmt_gemm_act_in; ffn1 then skips its act_bwd pass) against the
    separate pass: every gradient bit for bit in fp32 (one fp32 product
    either way), within one bf16 rounding of the masked product in bf16;
    the fused form taken for every encoder and decoder layer."""
    import fpnmt
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    calls = {}
    real_call = ops.call

    def counting_call(name, *a):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *a)

    monkeypatch.setattr(ops, "call", counting_call)
    res, counts = {}, {}
    try:
        for fuse in (False, True):
            calls.clear()
            m, _, _ = _build(num_layers=2, vocab=300, image=128, seed=9, rate=0.1)
            fpnmt.set_precision(prec)
            fpnmt.config.fuse_ffn_act = fuse
            ops.runtime.reset_sites()
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            loss.backward()
            torch.cuda.synchronize()
            counts[fuse] = dict(calls)
            res[fuse] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None})
    finally:
        fpnmt.config.fuse_ffn_act = True
        fpnmt.set_precision("fp32")
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)
    assert set(g0) == set(g1)
    # structurally-zero gradients (the attention K-projection biases: a
    # shift of every key leaves the softmax unchanged) are rounding noise in
    # bf16: their bar is relative to the model's gradient scale
    # bf16 rounding differences of the encoder-output gradient reach the
    # frozen-BN backbone, whose backward is ill-conditioned (DESIGN.md §6:
    # cancellation amplifies them element-wise), so the feature extractor is
    # held to a norm-wise bar over its whole gradient and the transformer's
    # tensors, where the fused epilogue runs, element-wise per tensor
    gmax = max(float(g.abs().max()) for g in g0.values())
    fe_d = fe_n = 0.0
    for n in g0:
        if prec == "fp32":
            assert torch.equal(g0[n], g1[n]), n
        elif ".feature_extractor." in n:
            fe_d += float(((g0[n] - g1[n]) ** 2).sum())
            fe_n += float((g0[n] ** 2).sum())
        else:
            d = float((g0[n] - g1[n]).abs().max())
            mx = float(g0[n].abs().max())
            assert d <= 3e-2 * max(mx, 1e-3 * gmax), (n, d, mx)
    assert fe_d ** 0.5 <= 5e-2 * fe_n ** 0.5, (fe_d ** 0.5, fe_n ** 0.5)
    fused = counts[True].get("fpnmt_gemm_act_in", 0)
    assert fused == 2 + 2, counts[True]  # ffn2 of every encoder and decoder layer
    assert counts[True].get("fpnmt_act_bwd", 0) == counts[False].get("fpnmt_act_bwd", 0) - fused


def test_deferred_dense_wgrads_match_immediate():
    """Inside a deferred-reduction region the transformer's Dense weight
    gradients (bf16) are queued and run at the flush as grouped whole-K tile
    launches (gemm_wg_jobs_kernel): the same gradients as the immediate
    launches up to fp32 summation order (and no stale operand: the queued
    GEMMs' inputs are held until the flush)."""
    import fpnmt
    from fpnmt import _lib as L
    from fpnmt import ops
    from models.transformer import create_masks
    img, tok = _inputs(b=2, vocab=300, image=128)
    res = {}
    try:
        for defer in (False, True):
            m, _, _ = _build(num_layers=2, vocab=300, image=128, seed=7)
            fpnmt.set_precision("bf16")
            tar_inp, tar_real = tok[:, :-1].to(DEV), tok[:, 1:].to(DEV)
            logits, _ = m(img.to(DEV), tar_inp, True, create_masks(tar_inp))
            loss = ops.MaskedXentFn.apply(logits, tar_real)
            with L.deferred_reductions(defer):
                loss.backward()
            torch.cuda.synchronize()
            res[defer] = (loss.detach().clone(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                                  if p.grad is not None})
    finally:
        fpnmt.set_precision("fp32")
    (l0, g0), (l1, g1) = res[False], res[True]
    assert torch.equal(l0, l1)
    assert set(g0) == set(g1)
    dense = [n for n in g0 if n.endswith(".kernel") and ("encoder.enc_layers" in n or "decoder." in n
                                                         or "final_layer" in n)]
    assert len(dense) >= 20, dense
    worst = []
    for n in g0:
        d = float((g0[n] - g1[n]).abs().max())
        mx = float(g0[n].abs().max())
        worst.append((d / max(mx, 1e-30), n))
        assert d <= 1e-4 * mx + 1e-30, (n, d, mx)
    print("largest relative difference", max(worst))


@pytest.mark.parametrize("graph", [False, True])
def test_fused_optimizer_prep_bitwise_equal(graph):
    """fpnmt_amsgrad_step_prep writes the bf16 compute copies (OHWI and
    flipped, frozen-BN scale folded) of the updated conv / dense kernels from
    the optimizer pass itself: masters, AMSGrad state, loss and EVERY compute
    copy equal the separate refresh pass (fpnmt_weight_prep_batched) bit for
    bit, over two steps (utils/pipeline.py:78)."""
    import fpnmt
    from fpnmt import layers as flayers
    from fpnmt.train import TrainEngine
    fpnmt.set_precision("bf16")
    try:
        results = []
        for fused in (True, False):
            fpnmt.config.fuse_optimizer_prep = fused
            m, _, _ = _build(num_layers=2, vocab=300, seed=43, rate=0.0)
            fpnmt.set_precision("bf16")  # _build leaves fp32 set
            eng = TrainEngine(m, 1e-4, use_graph=graph)
            img, tok = _inputs(b=2, vocab=300, seed=12)
            img, tok = img.to(DEV), tok.to(DEV)
            losses = [eng.step(img, tok).clone() for _ in range(3)]
            torch.cuda.synchronize()
            fp = flayers.fused_prep(m, eng.arena)
            if fused:
                assert fp is not None and len(fp.layers) > 20, "most kernels should take the fused path"
            copies = {}
            for i, lyr in enumerate(flayers.weight_layers(m)):
                for dt, (wf, wb) in lyr._copies.items():
                    copies[(i, str(dt))] = (wf.clone(), wb.clone())
            results.append((losses, eng.arena.flat.clone(), eng.arena.vhat.clone(), copies))
        (l0, f0, h0, c0), (l1, f1, h1, c1) = results
        for a, b in zip(l0, l1):
            assert torch.equal(a, b)
        assert torch.equal(f0, f1) and torch.equal(h0, h1)
        assert c0.keys() == c1.keys()
        for k in c0:
            assert torch.equal(c0[k][0], c1[k][0]), ("ohwi", k)
            assert torch.equal(c0[k][1], c1[k][1]), ("flip", k)
    finally:
        fpnmt.config.fuse_optimizer_prep = True
        fpnmt.set_precision("fp32")
