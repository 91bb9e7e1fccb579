"""Fused ResNet identity bottleneck (fpnmt_bottleneck_fwd, csrc/bottleneck.hip):
keras-resnet bottleneck_2d blocks 1.. (reference models/resnet.py:99-112)
as one launch with the 64 / 128-channel intermediates in LDS, inference only.

- against an fp32 CPU reference of the same block (torch conv2d on the folded
  bf16 weights, the two intermediates rounded to bf16 as both GPU paths store
  them), random frozen-BN statistics (non-trivial scale and shift), images at
  the top / bottom / side borders (the zero-padded halo);
- against the unfused three-launch path on a batch that gives the persistent
  blocks several tiles each (the DMA unit stream across tiles);
- the whole ResNet-50-FPN pyramid (bench.py headline_probe's work) with and
  without the fused blocks;
- the fused path stays off whenever a gradient is needed, for other shapes
  and dtypes (the caller's three convs run instead)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(56, 256, 64), (28, 512, 128)]  # (h = w, c, cm): res2, res3 at 224^2


def _block(c, cm, seed):
    import fpnmt
    from fpnmt.layers import Init, invalidate_weights
    from models.resnet import Bottleneck2D
    blk = Bottleneck2D(c, cm, stage=1, block=1, init=Init(torch.Generator().manual_seed(seed)))
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for conv in (blk.conv2a, blk.conv2b, blk.conv2c):
            k = conv.filters
            conv.bn_gamma.copy_(0.5 + torch.rand(k, generator=g))
            conv.bn_beta.copy_(0.2 * torch.randn(k, generator=g))
            conv.bn_mean.copy_(0.1 * torch.randn(k, generator=g))
            conv.bn_var.copy_(0.5 + torch.rand(k, generator=g))
            conv.refresh_bn()
    invalidate_weights()
    fpnmt.set_precision("bf16")
    return blk.to(DEV)


def _unfused(blk, x):
    import fpnmt
    fpnmt.config.fuse_bottleneck = False
    try:
        with torch.no_grad():
            return blk(x)
    finally:
        fpnmt.config.fuse_bottleneck = True


def _cpu_reference(blk, x):
    """fp32 CPU restatement on the GPU path's operands: the folded bf16 OHWI
    compute weights, fp32 folded biases, intermediates rounded to bf16."""
    import torch.nn.functional as F
    from fpnmt.ops import _f32_bias

    def w_oihw(conv):
        wf, _ = conv.compute_weights(torch.bfloat16)  # flat OHWI
        o, kh, kw, i = conv.filters, conv.kh, conv.kw, conv.in_channels
        return wf.float().cpu().view(o, kh, kw, i).permute(0, 3, 1, 2).contiguous()

    xc = x.float().cpu().permute(0, 3, 1, 2)
    a = F.conv2d(xc, w_oihw(blk.conv2a)) + _f32_bias(blk.conv2a).cpu()[None, :, None, None]
    a = a.clamp_min(0).bfloat16().float()
    b = F.conv2d(a, w_oihw(blk.conv2b), padding=1) + _f32_bias(blk.conv2b).cpu()[None, :, None, None]
    b = b.clamp_min(0).bfloat16().float()
    c = F.conv2d(b, w_oihw(blk.conv2c)) + _f32_bias(blk.conv2c).cpu()[None, :, None, None]
    return (c + xc).clamp_min(0).permute(0, 2, 3, 1)


def _x(n, h, c, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, h, h, c, generator=g)).bfloat16().to(DEV)


@pytest.mark.parametrize("h,c,cm", SHAPES)
def test_bottleneck_fused_vs_fp32_reference(h, c, cm):
    from fpnmt import ops
    blk = _block(c, cm, seed=5)
    x = _x(2, h, c, seed=6)
    with torch.no_grad():
        y = ops.bottleneck_fused(blk, x)
    assert y is not None, "the fused kernel did not take a supported shape"
    torch.cuda.synchronize()
    ref = _cpu_reference(blk, x)
    yf = y.float().cpu()
    err = (yf - ref).abs()
    scale = float(ref.abs().max())
    # bf16 output rounding (2^-8 relative) plus fp32 summation order; the
    # intermediates are rounded at the same points on both sides
    print(f"fused bottleneck {h}x{h}x{c}/{cm}: max|d| {float(err.max()):.3e} of max|y| {scale:.3e}, "
          f"mean|d| {float(err.mean()):.3e}")
    assert float(err.max()) <= 1e-2 * scale
    # the output's own bf16 rounding is ~2^-9 of |y| on average
    assert float(err.mean()) <= 4e-3 * float(ref.abs().mean())
    # every output pixel written (an unwritten border would hold empty_like garbage)
    assert bool(torch.isfinite(yf).all())


@pytest.mark.parametrize("h,c,cm", SHAPES)
def test_bottleneck_fused_equals_unfused_many_tiles(h, c, cm):
    """A batch whose tiles outnumber the 256 persistent blocks (res2: 16
    images = 448 tiles, res3: 40 images = 280 tiles): the same values as the
    three-launch path to bf16 rounding."""
    from fpnmt import ops
    n = 16 if h == 56 else 40
    blk = _block(c, cm, seed=7)
    x = _x(n, h, c, seed=8)
    with torch.no_grad():
        y = ops.bottleneck_fused(blk, x)
    assert y is not None
    yu = _unfused(blk, x)
    d = (y.float() - yu.float()).abs()
    scale = float(yu.float().abs().max())
    print(f"fused vs unfused {n}x{h}x{h}x{c}: max|d| {float(d.max()):.3e} of {scale:.3e}, "
          f"frac > 1 % of max {float((d > 1e-2 * scale).float().mean()):.2e}")
    assert float(d.max()) <= 2e-2 * scale
    assert float(d.mean()) <= 4e-3 * float(yu.float().abs().mean())


def test_bottleneck_fused_only_when_supported():
    import fpnmt
    from fpnmt import ops
    blk = _block(256, 64, seed=9)
    x = _x(1, 56, 256, seed=10)
    with torch.enable_grad():
        xr = x.clone().requires_grad_(True)
        assert ops.bottleneck_fused(blk, xr) is None  # a gradient is needed: the three convs
    with torch.no_grad():
        assert ops.bottleneck_fused(blk, x.float()) is None  # fp32 parity mode
        assert ops.bottleneck_fused(blk, _x(1, 28, 256, seed=11)) is None  # no kernel for 28x28x256/64
        assert ops.bottleneck_fused(blk, x) is not None
    fpnmt.set_precision("bf16")


def test_r50fpn_pyramid_fused_equals_unfused():
    """bench.py's headline work (ResNet-50 + FPN P3-P7, 224^2, bf16): the five
    fused identity blocks (res2b, c; res3b, c, d) against the unfused path."""
    import fpnmt
    from fpnmt.layers import Init
    from models.retinanet import FeatureExtractor
    fpnmt.set_precision("bf16")
    fe = FeatureExtractor(backbone="resnet50", init=Init(torch.Generator().manual_seed(3))).to(DEV)
    g = torch.Generator().manual_seed(4)
    x = (torch.rand(8, 224, 224, 3, generator=g) * 2 - 1).bfloat16().to(DEV)
    with torch.no_grad():
        fused = fe.retinanet_model.pyramid(x)
        fpnmt.config.fuse_bottleneck = False
        try:
            plain = fe.retinanet_model.pyramid(x)
        finally:
            fpnmt.config.fuse_bottleneck = True
    for lvl, (a, b) in enumerate(zip(fused, plain)):
        rel = float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))
        print(f"P{lvl + 3}: rel RMS fused vs unfused {rel:.3e}")
        assert rel <= 5e-2, lvl
