"""MobileNetV2 backbone — the reference FeatureExtractor's default
(models/retinanet.py:274, models/mobilenet.py:43-72).

CPU: the architecture against Keras' published MobileNetV2(alpha=1.0,
include_top=False) parameter counts, tap shapes, and the oracle's BN
semantics. GPU: the BatchNorm / depthwise kernels against torch fp32, and the
FeatureExtractor / training step against the oracle (oracle/ref_cpu.py,
mobilenet_v2 + batch_norm)."""
import math

import pytest
import torch

DEV = "cuda"


# --------------------------------------------------------------------- CPU
def test_param_counts_match_keras_summary():
    """keras.applications.MobileNetV2(alpha=1.0, include_top=False,
    weights=None).summary(): 2,257,984 params = 2,223,872 trainable (conv /
    depthwise kernels, BN gamma / beta) + 34,112 non-trainable (BN moving
    mean / variance)."""
    from models.mobilenet import MobileNetV2Backbone
    m = MobileNetV2Backbone()
    assert sum(p.numel() for p in m.parameters()) == 2223872
    assert sum(b.numel() for b in m.buffers()) == 34112


@pytest.mark.parametrize("image", [224, 512])
def test_oracle_tap_shapes(image):
    """block_5_add (H/8, 32), block_12_add (H/16, 96), out_relu (H/32, 1280)."""
    from fpnmt.layers import Init
    from models.mobilenet import MobileNetV2Backbone
    from oracle import ref_cpu as R
    m = MobileNetV2Backbone(init=Init(torch.Generator().manual_seed(0)))
    sd = {"b." + k: v for k, v in m.state_dict().items()}
    with torch.no_grad():
        outs = R.mobilenet_v2(sd, "b", torch.rand(1, image, image, 3) * 2 - 1, training=True)
    assert [tuple(o.shape) for o in outs] == [(1, image // 8, image // 8, 32), (1, image // 16, image // 16, 96),
                                              (1, image // 32, image // 32, 1280)]


def test_oracle_batchnorm_semantics():
    """Training-mode Keras BN: normalise with the biased batch variance, move
    the averages toward the Bessel-corrected one (momentum 0.999)."""
    from oracle import ref_cpu as R
    g = torch.Generator().manual_seed(1)
    x = torch.randn(3, 5, 4, 8, generator=g) * 2 + 1
    sd = {"bn.gamma": torch.rand(8, generator=g) + 0.5, "bn.beta": torch.randn(8, generator=g),
          "bn.moving_mean": torch.zeros(8), "bn.moving_variance": torch.ones(8)}
    st = {}
    y = R.batch_norm(sd, "bn", x, True, st)
    flat = x.reshape(-1, 8)
    mu, var = flat.mean(0), flat.var(0, unbiased=False)
    assert torch.allclose(y.reshape(-1, 8), (flat - mu) / torch.sqrt(var + 1e-3) * sd["bn.gamma"] + sd["bn.beta"],
                          atol=1e-5)
    assert torch.allclose(st["bn.moving_mean"], 0.001 * mu, atol=1e-7)
    assert torch.allclose(st["bn.moving_variance"], 0.999 + 0.001 * flat.var(0, unbiased=True), atol=1e-6)


# --------------------------------------------------------------------- GPU
def _close(a, b, dt, tol32=2e-5, tol16=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    tol = tol32 if dt == torch.float32 else tol16
    assert float((a - b).abs().max()) <= tol * max(1.0, float(b.abs().max())), float((a - b).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act,res", [("relu6", False), (None, True), (None, False)])
def test_batchnorm_train_fwd_bwd(dt, act, res):
    from fpnmt.layers import BatchNormalization
    g = torch.Generator().manual_seed(2)
    n, h, w, c = 4, 9, 11, 48
    bn = BatchNormalization(c).to(DEV)
    with torch.no_grad():
        bn.gamma.copy_(torch.rand(c, generator=g) + 0.5)
        bn.beta.copy_(torch.randn(c, generator=g))
    x = (torch.randn(n, h, w, c, generator=g) * 3 + 2).to(dt).to(DEV).requires_grad_(True)
    r = torch.randn(n, h, w, c, generator=g).to(dt).to(DEV).requires_grad_(True) if res else None
    y = bn(x, True, act, r)
    # torch fp32 restatement
    xf = x.detach().float().requires_grad_(True)
    rf = r.detach().float().requires_grad_(True) if res else None
    gm = bn.gamma.detach().clone().requires_grad_(True)
    bt = bn.beta.detach().clone().requires_grad_(True)
    fl = xf.reshape(-1, c)
    mu, var = fl.mean(0), fl.var(0, unbiased=False)
    yr = ((fl - mu) / torch.sqrt(var + 1e-3) * gm + bt).reshape(xf.shape)
    if act == "relu6":
        yr = torch.clamp(yr, 0, 6)
    if res:
        yr = yr + rf
    _close(y, yr, dt)
    gy = torch.randn(yr.shape, generator=g)
    y.backward(gy.to(dt).to(DEV))
    yr.backward(gy.to(dt).float().to(DEV))
    torch.cuda.synchronize()
    _close(x.grad, xf.grad, dt, 1e-4, 5e-2)
    _close(bn.gamma.grad, gm.grad, dt, 1e-4, 5e-2)
    _close(bn.beta.grad, bt.grad, dt, 1e-4, 5e-2)
    if res:
        _close(r.grad, rf.grad, dt)
    # moving statistics moved once
    _close(bn.moving_mean, 0.001 * mu.detach(), dt, 1e-6, 1e-4)
    _close(bn.moving_variance, 0.999 + 0.001 * fl.detach().var(0, unbiased=True), dt, 1e-6, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,stride,pads", [((2, 14, 14, 96), 1, (1, 1, 1, 1)), ((3, 14, 12, 32), 2, (0, 1, 0, 1)),
                                               ((2, 7, 7, 16), 2, (0, 1, 0, 1)), ((1, 5, 6, 8), 1, (1, 1, 1, 1))])
def test_depthwise_fwd_bwd(dt, shape, stride, pads):
    import torch.nn.functional as F
    from fpnmt.layers import DepthwiseConv2D, Init
    n, h, w, c = shape
    dw = DepthwiseConv2D(c, 3, stride, pads, init=Init(torch.Generator().manual_seed(3))).to(DEV)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(shape, generator=g).to(dt).to(DEV).requires_grad_(True)
    y = dw(x)
    xf = x.detach().float().requires_grad_(True)
    kf = dw.kernel.detach().clone().requires_grad_(True)
    xt = F.pad(xf.permute(0, 3, 1, 2), (pads[2], pads[3], pads[0], pads[1]))
    yr = F.conv2d(xt, kf.permute(2, 3, 0, 1), stride=stride, groups=c).permute(0, 2, 3, 1)
    assert y.shape == yr.shape
    _close(y, yr, dt)
    gy = torch.randn(yr.shape, generator=g)
    y.backward(gy.to(dt).to(DEV))
    yr.backward(gy.to(dt).float().to(DEV))
    torch.cuda.synchronize()
    _close(x.grad, xf.grad, dt)
    _close(dw.kernel.grad, kf.grad, dt, 1e-4, 5e-2)


def _fe(seed=0):
    import fpnmt
    from fpnmt.layers import Init
    from models.retinanet import FeatureExtractor
    fpnmt.set_precision("fp32")
    fe = FeatureExtractor(backbone="mobilenet224_1.0", init=Init(torch.Generator().manual_seed(seed)))
    sd = {"fe." + k: v.detach().float().clone() for k, v in fe.state_dict().items()}
    return fe.to(DEV), sd


@pytest.mark.gpu
@pytest.mark.parametrize("training", [True, False])
def test_feature_extractor_matches_oracle_fp32(training):
    """FeatureExtractor(backbone='mobilenet224_1.0') level outputs (and, in
    training mode, every BN's updated moving statistics) vs the oracle."""
    from oracle import ref_cpu as R
    fe, sd = _fe(5)
    img = torch.rand(2, 224, 224, 3, generator=torch.Generator().manual_seed(6)) * 2 - 1
    st = {}
    with torch.no_grad():
        outs = fe(img.to(DEV), training=training)
        ref = R.feature_extractor(sd, "fe", img, "mobilenet224_1.0", training=training, stats=st)
    torch.cuda.synchronize()
    for lvl, (o, r) in enumerate(zip(outs, ref)):
        assert o.shape == r.shape
        if r.numel():
            err = float((o.cpu() - r).abs().max())
            print(f"P{lvl + 3}: max|d| {err:.2e} max|ref| {float(r.abs().max()):.2e}")
            assert err <= 1e-4 * float(r.abs().max()) + 1e-30, lvl  # relative: untrained levels are tiny
    if training:
        msd = fe.state_dict()
        assert len(st) == 2 * 52  # 52 BN layers
        for k, v in st.items():
            got = msd[k[len("fe."):]].cpu()
            assert torch.allclose(got, v, atol=1e-5, rtol=1e-4), k


@pytest.mark.gpu
def test_backbone_grads_vs_fp64():
    """Training-mode BN (batch statistics), ReLU6, depthwise and 1x1 convs
    backward through the whole MobileNetV2 backbone (loss = random
    projections of C3, C4, C5), anchored on an fp64 oracle run: per tensor,
    the GPU fp32 error norm ||g - g64|| / ||g64|| within 3x the fp32
    oracle's own (+1e-5). (Norms, not max elements: batch-statistics BN
    backward subtracts channel means of g and g*xhat, so single elements are
    cancellations.) The FPN / heads' backward over this backbone is the
    ResNet path's (tests/test_gpu_parts.py); through the whole feature
    extractor the fp32 comparison is dominated by ReLU masks of the
    near-zero FPN activations that flip between any two fp32 runs."""
    from oracle import ref_cpu as R
    fe, sd = _fe(7)
    bb = fe.retinanet_model.backbone
    bb.bn_training = True
    g = torch.Generator().manual_seed(8)
    img = torch.rand(2, 128, 128, 3, generator=g) * 2 - 1
    outs = bb(img.to(DEV))[1:]
    ws = [torch.randn(o.shape, generator=g) for o in outs]
    sum((o * w.to(DEV)).sum() for o, w in zip(outs, ws)).backward()
    res = {}
    for dt in (torch.float32, torch.float64):
        params = {k: v.to(dt).clone().requires_grad_(True) for k, v in sd.items()}
        ro = R.mobilenet_v2(params, "fe.retinanet_model.backbone", img.to(dt), training=True)
        sum((o * w.to(dt)).sum() for o, w in zip(ro, ws)).backward()
        res[dt] = params
    worst = []
    for n, p in bb.named_parameters():
        t = res[torch.float64]["fe.retinanet_model.backbone." + n].grad
        nrm = float(t.norm())
        eg = float((p.grad.detach().cpu().double() - t).norm()) / nrm
        ec = float((res[torch.float32]["fe.retinanet_model.backbone." + n].grad.double() - t).norm()) / nrm
        worst.append((eg - 3 * ec, eg, ec, n))
    worst.sort(reverse=True)
    for w in worst[:4]:
        print("rel err norm vs fp64: gpu %.2e cpu32 %.2e %s" % w[1:])
    assert worst[0][1] <= 3 * worst[0][2] + 1e-5, worst[0]


@pytest.mark.gpu
def test_train_step_and_decode_with_mobilenet():
    """The reference's default model end to end: the fp32 training step's
    loss equals the oracle's (BN in training mode), a bf16 hipGraph step stays
    finite, and greedy decode (BN on moving statistics) matches the oracle's
    predict()."""
    import fpnmt
    from oracle import ref_cpu as R
    from fpnmt.layers import Init
    from fpnmt.train import TrainEngine
    from models.transformer import Transformer
    fpnmt.set_precision("fp32")
    m = Transformer(1, 512, 8, 2048, math.ceil(224 / 16) ** 2, 300, 0.0, max_seq_len=16,
                    backbone="mobilenet224_1.0", init=Init(torch.Generator().manual_seed(9)))
    sd = {k: v.detach().float().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    g = torch.Generator().manual_seed(10)
    img = torch.rand(2, 224, 224, 3, generator=g) * 2 - 1
    tok = torch.randint(4, 300, (2, 16), generator=g)
    tok[:, 0] = 2
    tok[1, 9] = 3
    tok[1, 10:] = 0
    cfg = dict(num_layers=1, num_heads=8, backbone="mobilenet224_1.0")
    eng = TrainEngine(m, 1e-4, use_graph=False)
    loss = float(eng.step(img.to(DEV), tok.to(DEV)))
    with torch.no_grad():
        lg, _ = R.transformer(sd, img, tok[:, :-1], True, R.create_masks(tok[:, :-1]), cfg)
    loss_ref = float(R.masked_loss(tok[:, 1:], lg))
    print(f"mobilenet train-step loss {loss:.6f} oracle {loss_ref:.6f}")
    assert abs(loss - loss_ref) <= 1e-4 * max(1.0, abs(loss_ref))
    # greedy decode on the updated model (moving statistics moved by the step)
    sd2 = {k: v.detach().float().cpu().clone() for k, v in m.state_dict().items()}
    from utils.pipeline import Pipeline
    x1 = img[0]
    with torch.no_grad():
        enc = m.encoder(x1[None].to(DEV), False, None)
        encr = R.encoder(sd2, x1[None], cfg)
    assert float((enc.cpu() - encr).abs().max()) <= 1e-4 * max(1.0, float(encr.abs().max()))
    fpnmt.set_precision("bf16")
    try:
        engb = TrainEngine(m, 1e-4, use_graph=True)
        lb = [float(engb.step(img.to(DEV), tok.to(DEV))) for _ in range(3)]
    finally:
        fpnmt.set_precision("fp32")
    assert all(math.isfinite(v) for v in lb), lb
