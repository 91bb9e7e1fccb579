"""Per-kernel numerics on the GPU: every libfpnmt op against a plain PyTorch
fp32 reference of the same op (and the oracle's TF-semantics helpers), in the
exact-fp32 MFMA mode (tight tolerance) and the bf16 mode (bf16 tolerance).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _tol(dt):
    return (2e-4, 2e-4) if dt == torch.float32 else (3e-2, 3e-2)


def _close(a, b, dt, scale=None):
    a, b = a.detach().float(), b.detach().float()
    assert a.shape == b.shape, (a.shape, b.shape)
    if a.numel() == 0:
        return
    rtol, atol = _tol(dt)
    s = scale if scale is not None else max(1.0, float(b.abs().max()))
    err = float((a - b).abs().max()) if a.numel() else 0.0
    assert err <= atol * s + rtol * 0, f"max err {err:.3e} (scale {s:.3e})"


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mnk", [(1, 1, 1), (31, 33, 17), (64, 64, 64), (200, 130, 96), (992, 512, 512),
                                 (257, 1000, 72), (4, 2048, 512)])
@pytest.mark.parametrize("trans", [(0, 0), (0, 1), (1, 1), (1, 0)])
def test_gemm_modes(dt, mnk, trans):
    from fpnmt import _lib as L
    m, n, k = mnk
    ta, tb = trans
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n * 3 + k)
    A = torch.randn(m, k, generator=g).to(DEV)
    B = torch.randn(k, n, generator=g).to(DEV)
    bias = torch.randn(n, generator=g).to(DEV)
    a_st = (A.t().contiguous() if ta else A).to(dt)
    b_st = (B.contiguous() if tb else B.t().contiguous()).to(dt)
    C = torch.empty(m, n, dtype=dt, device=DEV)
    d = L.GemmDesc()
    d.m, d.n, d.k, d.batch, d.batch_inner, d.dtype = m, n, k, 1, 1, L.dtype_code(dt)
    d.a_trans, d.b_trans = ta, tb
    d.lda = m if ta else k
    d.ldb = n if tb else k
    d.ldc = d.ldr = n
    d.alpha, d.act, d.act_alpha, d.accumulate, d.c_f32, d.split_k = 1.0, L.ACT_LEAKY, 0.2, 0, 0, 1
    L.call("fpnmt_gemm", d, a_st.data_ptr(), b_st.data_ptr(), C.data_ptr(), None, bias.data_ptr(), None,
           L.stream_ptr())
    ref = F.leaky_relu(A.to(dt).float() @ B.to(dt).float() + bias, 0.2)
    torch.cuda.synchronize()
    _close(C, ref, dt, scale=max(1.0, math.sqrt(k)))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_atomic_splitk_and_epilogue(dt):
    from fpnmt import _lib as L
    m, n, k = 96, 80, 4096
    A = torch.randn(k, m, device=DEV).to(dt)  # stored K x M (a_trans)
    B = torch.randn(k, n, device=DEV).to(dt)  # stored K x N (b_trans)
    C = torch.ones(m, n, device=DEV)
    sc = torch.rand(n, device=DEV) + 0.5
    d = L.GemmDesc()
    d.m, d.n, d.k, d.batch, d.batch_inner, d.dtype = m, n, k, 1, 1, L.dtype_code(dt)
    d.a_trans, d.b_trans, d.lda, d.ldb, d.ldc, d.ldr = 1, 1, m, n, n, n
    d.alpha, d.act, d.accumulate, d.c_f32, d.split_k = 0.5, 0, 2, 1, 0
    L.call("fpnmt_gemm", d, A.data_ptr(), B.data_ptr(), C.data_ptr(), sc.data_ptr(), None, None, L.stream_ptr())
    ref = 1 + 0.5 * (A.float().t() @ B.float()) * sc
    torch.cuda.synchronize()
    _close(C, ref, dt, scale=64.0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_batched_residual(dt):
    from fpnmt import _lib as L
    Bo, Hi, m, n, k = 3, 4, 31, 64, 64
    A = torch.randn(Bo, m, Hi * k, device=DEV).to(dt)
    Bm = torch.randn(Bo, n, Hi * k, device=DEV).to(dt)
    R = torch.randn(Bo, Hi, m, n, device=DEV).to(dt)
    C = torch.empty(Bo, Hi, m, n, device=DEV, dtype=torch.float32)
    d = L.GemmDesc()
    d.m, d.n, d.k, d.batch, d.batch_inner, d.dtype = m, n, k, Bo * Hi, Hi, L.dtype_code(dt)
    d.a_trans, d.b_trans = 0, 0
    d.lda, d.ldb, d.ldc, d.ldr = Hi * k, Hi * k, n, n
    d.a_so, d.a_si, d.b_so, d.b_si = m * Hi * k, k, n * Hi * k, k
    d.c_so, d.c_si, d.r_so, d.r_si = Hi * m * n, m * n, Hi * m * n, m * n
    d.alpha, d.act, d.accumulate, d.c_f32, d.split_k = 0.125, 1, 0, 1, 1
    L.call("fpnmt_gemm", d, A.data_ptr(), Bm.data_ptr(), C.data_ptr(), None, None, R.data_ptr(), L.stream_ptr())
    Ah = A.float().reshape(Bo, m, Hi, k).permute(0, 2, 1, 3)
    Bh = Bm.float().reshape(Bo, n, Hi, k).permute(0, 2, 1, 3)
    ref = F.relu(0.125 * Ah @ Bh.transpose(-1, -2) + R.float())
    torch.cuda.synchronize()
    _close(C, ref, dt, scale=8.0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(32, 512, 6144, 1), (17, 100, 3000, 3), (64, 512, 2048, 1), (40, 64, 1024, 2)])
def test_gemm_small_split_k(dt, shape):
    """Small-M GEMMs split K across blocks through the process workspace: the
    partial tiles are summed in split order, so two runs are bit-identical,
    and bias / residual / activation are applied once by the last block."""
    from fpnmt import _lib as L
    m, n, k, nb = shape
    g = torch.Generator().manual_seed(m + n + k)
    A = torch.randn(nb, m, k, generator=g).to(dt).to(DEV)
    Bm = torch.randn(nb, n, k, generator=g).to(dt).to(DEV)
    R = torch.randn(nb, m, n, generator=g).to(dt).to(DEV)
    bias = torch.randn(n, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        C = torch.empty(nb, m, n, dtype=dt, device=DEV)
        d = L.GemmDesc()
        d.m, d.n, d.k, d.batch, d.batch_inner, d.dtype = m, n, k, nb, 1, L.dtype_code(dt)
        d.lda, d.ldb, d.ldc, d.ldr = k, k, n, n
        d.a_so, d.b_so, d.c_so, d.r_so = m * k, n * k, m * n, m * n
        d.alpha, d.act, d.act_alpha, d.accumulate, d.c_f32, d.split_k = 0.5, L.ACT_LEAKY, 0.2, 0, 0, 1
        L.call("fpnmt_gemm", d, A.data_ptr(), Bm.data_ptr(), C.data_ptr(), None, bias.data_ptr(), R.data_ptr(),
               L.stream_ptr())
        outs.append(C)
    ref = F.leaky_relu(0.5 * A.float() @ Bm.float().transpose(1, 2) + bias + R.float(), 0.2)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    _close(outs[0], ref, dt, scale=max(1.0, math.sqrt(k)))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,acc", [((992, 512, 10000), 0), ((1568, 512, 6144), 1), ((288, 512, 6144), 0)])
def test_gemm_long_k_rows(dt, shape, acc):
    """Long-K row GEMMs over a few hundred to a few thousand rows (the decoder's
    vocabulary-wide dgrad, M = 992, K = 10 000 — K not a multiple of 64; the
    views' grouped K/V projection dgrads, K = 6144): 128x128 tiles split over
    K through the workspace, summed in split order with the full epilogue
    (bias, residual, activation, or C += for accumulate 1); run to run the
    same bits."""
    from fpnmt import _lib as L
    m, n, k = shape
    g = torch.Generator().manual_seed(m + k)
    A = torch.randn(m, k, generator=g).to(dt).to(DEV)
    Bm = torch.randn(n, k, generator=g).to(dt).to(DEV)
    R = torch.randn(m, n, generator=g).to(dt).to(DEV)
    C0 = torch.randn(m, n, generator=g).to(dt).to(DEV)
    bias = torch.randn(n, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        C = C0.clone()
        d = L.GemmDesc()
        d.m, d.n, d.k, d.batch, d.batch_inner, d.dtype = m, n, k, 1, 1, L.dtype_code(dt)
        d.lda, d.ldb, d.ldc, d.ldr = k, k, n, n
        if acc:
            d.alpha, d.act, d.act_alpha, d.accumulate, d.c_f32, d.split_k = 0.5, 0, 0.0, 1, 0, 1
            L.call("fpnmt_gemm", d, A.data_ptr(), Bm.data_ptr(), C.data_ptr(), None, None, None, L.stream_ptr())
        else:
            d.alpha, d.act, d.act_alpha, d.accumulate, d.c_f32, d.split_k = 0.5, L.ACT_LEAKY, 0.2, 0, 0, 1
            L.call("fpnmt_gemm", d, A.data_ptr(), Bm.data_ptr(), C.data_ptr(), None, bias.data_ptr(), R.data_ptr(),
                   L.stream_ptr())
        outs.append(C)
    prod = 0.5 * A.float() @ Bm.float().t()
    ref = C0.float() + prod if acc else F.leaky_relu(prod + bias + R.float(), 0.2)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    _close(outs[0], ref, dt, scale=max(1.0, math.sqrt(k)))


# ------------------------------------------------------------------ conv
CONV_CASES = [
    # n, h, w, c, k, r, stride, padding
    (2, 9, 9, 64, 32, 3, 1, "same"),
    (2, 14, 14, 256, 256, 3, 1, "same"),
    (3, 7, 7, 512, 256, 1, 1, "same"),
    (2, 28, 28, 64, 128, 1, 2, "valid"),
    (2, 4, 4, 256, 64, 1, 2, "valid"),  # tiny strided 1x1: dgrad = row-scatter GEMM with M = 8
    (2, 2, 2, 512, 256, 1, 1, "same"),  # M = 8 rows
    (2, 32, 32, 3, 64, 7, 2, (3, 3, 3, 3)),
    (2, 12, 12, 32, 16, 3, 1, (1, 1, 1, 1)),
    (2, 5, 5, 256, 1, 3, 1, "same"),
    (1, 1, 1, 256, 512, 3, 1, "same"),
    (2, 3, 5, 24, 40, 3, 1, "same"),
    # large enough for the pipelined LDS-DMA kernel (bf16): 128x256, 256x128, 256x64 tiles
    (16, 28, 28, 128, 256, 3, 1, "same"),
    (16, 56, 56, 64, 64, 3, 1, "same"),
    (16, 28, 28, 256, 512, 1, 1, "same"),
    # strided 1x1 projection shortcuts (res3a / res4a): the dgrad's row scatter on
    # the LDS-DMA pipe kernels + scatter_rows_kernel (round 6)
    (4, 56, 56, 256, 512, 1, 2, "valid"),
    (8, 28, 28, 512, 1024, 1, 2, "valid"),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(dt, case):
    from fpnmt.layers import Conv2D
    from oracle import ref_cpu as R
    n, h, w, c, k, r, s, pad = case
    torch.manual_seed(sum(case[:6]))
    layer = Conv2D(c, k, r, strides=s, padding=pad, activation="relu", kernel_initializer="glorot_uniform").to(DEV)
    with torch.no_grad():
        layer.bias.normal_(0, 0.1)
    x = torch.randn(n, h, w, c, device=DEV).to(dt)
    res = None
    # big cases: fp64 CPU reference (the GPU fp32 conv reference may pick
    # Winograd for 3x3, ~1e-3 relative error — above this test's fp32 bar)
    big = n * h * w * c * k * r * r > 10 ** 8
    rdt, rdev = (torch.float64, "cpu") if big else (torch.float32, DEV)
    x_ref = x.to(rdt).to(rdev).clone().requires_grad_(True)
    need_dx = s == 1 or r == 1  # strided k>1 convs only occur on the image (no dgrad)
    x_in = x.clone().requires_grad_(need_dx)
    y = layer(x_in)
    pads = layer.pads_for(h, w)
    kern = layer.kernel.detach().to(dt).to(rdt).to(rdev).clone().requires_grad_(True)
    bias = layer.bias.detach().to(rdt).to(rdev).clone().requires_grad_(True)
    # the ReLU derivative is taken at the GPU's own outputs: where the
    # pre-activation is within rounding of 0 (a few of the ~3M outputs of the
    # big cases) the two sides may pick opposite sides of the kink, which
    # would move a whole dx row by |gy * w| and say nothing about the kernel
    pre = R.conv2d(x_ref, kern, bias, s, pads)
    y_ref = pre * (y.detach() > 0).to(rdt).to(rdev)
    _close(y, F.relu(pre).to(DEV), dt, scale=max(1.0, math.sqrt(r * r * c) * 0.3))
    gy = torch.randn(y_ref.shape, device=DEV)
    y.backward(gy.to(dt))
    y_ref.backward(gy.to(rdt).to(rdev))
    torch.cuda.synchronize()
    sc_x = max(1.0, math.sqrt(r * r * k))
    if need_dx:
        _close(x_in.grad, x_ref.grad.to(DEV), dt, scale=sc_x)
    sc_w = max(1.0, math.sqrt(n * y.shape[1] * y.shape[2]) * 2)
    _close(layer.kernel.grad, kern.grad.to(DEV), dt, scale=sc_w)
    _close(layer.bias.grad, bias.grad.to(DEV), dt, scale=sc_w)


# 3x3 stride-1 'same' convs over the shapes of the LDS-DMA pipe kernels'
# im2col tiles: one / several 64-channel K-tiles per tap, W = 62 (the widest
# padded row), non-square grids, tiles straddling images; under-filled grids
# take the split-K (fp32 slabs + ordered reduce) forms, held to the same bar.
CONV3X3_CASES = [
    (32, 28, 28, 256, 256),
    (16, 56, 56, 64, 64),
    (16, 56, 56, 128, 128),
    (9, 62, 62, 64, 128),
    (16, 40, 60, 64, 128),
    (64, 14, 14, 256, 256),
    # under-filled grids (the register-staged split-K kernels, same bar)
    (32, 14, 14, 256, 256),
    (32, 7, 7, 512, 512),
    (64, 14, 14, 128, 128),
]


@pytest.mark.parametrize("case", CONV3X3_CASES)
def test_conv3x3_same_bf16(case):
    """bf16 3x3 'same' conv forward and bwd-data (pipe / split-K kernels) against an
    fp32 im2col (unfold) reference of the same bf16-rounded operands: every
    element within one bf16 rounding of the output (+1e-4 of the range), so a
    single wrong or missing tap (~0.3 here) cannot hide."""
    import fpnmt
    from fpnmt.layers import Conv2D
    fpnmt.set_precision("bf16")
    n, h, w, c, k = case
    torch.manual_seed(n + h + w + c + k)
    layer = Conv2D(c, k, 3, padding="same", activation=None, kernel_initializer="glorot_uniform").to(DEV)
    with torch.no_grad():
        layer.bias.normal_(0, 0.1)
    x = torch.randn(n, h, w, c, device=DEV).to(torch.bfloat16)
    xi = x.clone().requires_grad_(True)
    y = layer(xi)
    gy = torch.randn(y.shape, device=DEV).to(torch.bfloat16)
    y.backward(gy)
    torch.cuda.synchronize()
    wq = layer.kernel.detach().to(torch.bfloat16).float()  # HWIO
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    cols = F.unfold(xr, 3, padding=1)  # (n, c*9, h*w), index c*9 + r*3 + s
    w2 = wq.permute(3, 2, 0, 1).reshape(k, c * 9)
    yr = (w2 @ cols).reshape(n, k, h, w).permute(0, 2, 3, 1) + layer.bias.detach().float()
    yr.backward(gy.float())

    def check(a, b):
        a, b = a.detach().float(), b.detach().float()
        err = (a - b).abs()
        bound = 2.0 ** -8 * b.abs() + 1e-4 * float(b.abs().max())
        bad = int((err > bound).sum())
        assert bad == 0, f"{bad} elements off, worst {float(err.max()):.3e} at |ref| max {float(b.abs().max()):.3e}"

    check(y, yr)
    check(xi.grad, xr.grad.permute(0, 2, 3, 1))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_frozen_bn_residual(dt):
    from fpnmt.layers import Conv2D
    torch.manual_seed(3)
    layer = Conv2D(64, 128, 1, padding="valid", activation="relu", use_bias=False, frozen_bn=True).to(DEV)
    with torch.no_grad():
        layer.bn_gamma.uniform_(0.5, 1.5)
        layer.bn_beta.normal_()
        layer.bn_mean.normal_()
        layer.bn_var.uniform_(0.5, 2)
        layer.refresh_bn()
    x = torch.randn(2, 6, 6, 64, device=DEV).to(dt).requires_grad_(True)
    res = torch.randn(2, 6, 6, 128, device=DEV).to(dt).requires_grad_(True)
    y = layer(x, residual=res)
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True)
    kern = layer.kernel.detach().clone().requires_grad_(True)
    sc = layer.bn_gamma / torch.sqrt(layer.bn_var + 1e-5)
    wq = (kern * sc).to(dt).float() if dt != torch.float32 else kern * sc
    yr = F.relu(torch.einsum("nhwc,ck->nhwk", xr, wq[0, 0]) + (layer.bn_beta - layer.bn_mean * sc) + rr)
    _close(y, yr, dt, scale=8.0)
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    torch.cuda.synchronize()
    _close(x.grad, xr.grad, dt, scale=12.0)
    _close(res.grad, rr.grad, dt, scale=4.0)
    _close(layer.kernel.grad, kern.grad, dt, scale=12.0)


@pytest.mark.parametrize("case", [(3, 37, 37, 64, (3, 3, 3, 3), "relu"), (2, 224, 224, 64, (3, 3, 3, 3), "relu"),
                                  (1, 30, 45, 128, (2, 3, 2, 3), None), (1, 7, 7, 64, (3, 3, 3, 3), "relu")])
def test_stem_conv_frozen_bn(case):
    """conv_stem.hip (7x7/2 over 3 channels, bf16): tiles with partial rows /
    columns, 2 channel chunks, asymmetric pads; fp64 reference on the same
    bf16-rounded operands, so the bar is the output's own bf16 rounding."""
    from fpnmt.layers import Conv2D
    from oracle import ref_cpu as R
    n, h, w, k, pad, act = case
    torch.manual_seed(n * h + k)
    layer = Conv2D(3, k, 7, strides=2, padding=pad, activation=act, use_bias=False, frozen_bn=True).to(DEV)
    with torch.no_grad():
        layer.bn_gamma.uniform_(0.5, 1.5)
        layer.bn_beta.normal_()
        layer.bn_mean.normal_()
        layer.bn_var.uniform_(0.5, 2)
        layer.refresh_bn()
    x = (torch.rand(n, h, w, 3, device=DEV) * 2 - 1).to(torch.bfloat16)
    with torch.no_grad():
        y = layer(x)
    sc = (layer.bn_gamma / torch.sqrt(layer.bn_var + 1e-5)).detach()
    wq = (layer.kernel.detach() * sc).to(torch.bfloat16).double().cpu()
    shift = (layer.bn_beta - layer.bn_mean * sc).detach().double().cpu()
    ref = R.conv2d(x.double().cpu(), wq, shift, 2, layer.pads_for(h, w))
    if act == "relu":
        ref = F.relu(ref)
    assert y.shape == ref.shape
    err = (y.double().cpu() - ref).abs()
    bar = ref.abs() * 2.0 ** -8 + 1e-3
    assert bool((err <= bar).all()), f"max err {float(err.max()):.3e}"


# ------------------------------------------------------------- pooling etc
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_maxpool(dt):
    from fpnmt import ops
    from oracle import ref_cpu as R
    for shape in [(2, 7, 7, 16), (2, 6, 8, 8), (1, 1, 1, 8), (2, 112, 112, 64)]:
        x = torch.randn(*shape, device=DEV).to(dt).requires_grad_(True)
        xr = x.detach().float().requires_grad_(True)
        for fn, rf in [(ops.max_pool2d_valid, R.maxpool_valid), (lambda t: ops.max_pool2d_same(t, 3, 2), R.maxpool_same)]:
            if x.grad is not None:
                x.grad = None
                xr.grad = None
            y = fn(x)
            yr = rf(xr)
            _close(y, yr, dt)
            if y.numel():
                g = torch.randn_like(yr)
                y.backward(g.to(dt))
                yr.backward(g)
                _close(x.grad, xr.grad, dt, scale=4.0)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_maxpool_bwd_recompute_and_ties(dt):
    """bwd from x (no argmax) == bwd from the fwd argmax; ties go to the first
    tap in window order (values quantised so ties are common)."""
    from fpnmt import _lib as L
    from fpnmt import ops
    for shape, c_ok in [((2, 15, 15, 64), True), ((2, 9, 11, 6), False)]:
        n, h, w, c = shape
        x = (torch.randint(0, 3, shape, device=DEV).float()).to(dt)
        ho, wo = (h + 1) // 2, (w + 1) // 2
        pt, pl = ((ho - 1) * 2 + 3 - h) // 2, ((wo - 1) * 2 + 3 - w) // 2
        y = torch.empty(n, ho, wo, c, device=DEV, dtype=dt)
        am = torch.empty(n, ho, wo, c, device=DEV, dtype=torch.uint8)
        L.call("fpnmt_maxpool2d_fwd", L.dtype_code(dt), n, h, w, c, 3, 3, 2, 2, pt, pl, ho, wo,
               L.ptr(x), L.ptr(y), L.ptr(am), L.stream_ptr())
        dy = torch.randn(n, ho, wo, c, device=DEV).to(dt)
        dx1, dx2 = torch.empty_like(x), torch.empty_like(x)
        L.call("fpnmt_maxpool2d_bwd", L.dtype_code(dt), n, h, w, c, 3, 3, 2, 2, pt, pl, ho, wo,
               L.ptr(x), L.ptr(am), L.ptr(dy), L.ptr(dx1), L.stream_ptr())
        L.call("fpnmt_maxpool2d_bwd", L.dtype_code(dt), n, h, w, c, 3, 3, 2, 2, pt, pl, ho, wo,
               L.ptr(x), None, L.ptr(dy), L.ptr(dx2), L.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dx1, dx2)
        # CPU: first max in window order
        xc, ac = x.float().cpu(), am.cpu().long()
        xp = torch.nn.functional.pad(xc.permute(0, 3, 1, 2), (pl, 3 * 1, pt, 3), value=float("-inf"))
        for i in range(3):
            for j in range(3):
                tap = xp[:, :, i:i + 2 * ho:2, j:j + 2 * wo:2].permute(0, 2, 3, 1)
                first = (ac == i * 3 + j)
                assert torch.equal(tap[first], y.float().cpu()[first])
                earlier = ac > i * 3 + j  # taps before the argmax must be strictly smaller
                assert bool((tap[earlier] < y.float().cpu()[earlier]).all())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("sizes", [(7, 14, 28), (16, 32, 64), (4, 7, 13), (1, 1, 2)])
def test_fpn_topdown(dt, sizes):
    from fpnmt import ops
    from oracle import ref_cpu as R
    h5, h4, h3 = sizes
    n, c = 2, 64
    l5 = torch.randn(n, h5, h5, c, device=DEV).to(dt).requires_grad_(True)
    l4 = torch.randn(n, h4, h4, c, device=DEV).to(dt).requires_grad_(True)
    l3 = torch.randn(n, h3, h3, c, device=DEV).to(dt).requires_grad_(True)
    p4m, p3m = ops.FpnTopDownFn.apply(l5, l4, l3)
    r5, r4, r3 = [t.detach().float().requires_grad_(True) for t in (l5, l4, l3)]
    q4 = R.upsample_like(r5, r4) + r4
    q3 = R.upsample_like(q4, r3) + r3
    _close(p4m, q4, dt, scale=4)
    _close(p3m, q3, dt, scale=4)
    g4, g3 = torch.randn_like(q4), torch.randn_like(q3)
    torch.autograd.backward([p4m, p3m], [g4.to(dt), g3.to(dt)])
    torch.autograd.backward([q4, q3], [g4, g3])
    for a, b in [(l5.grad, r5.grad), (l4.grad, r4.grad), (l3.grad, r3.grad)]:
        _close(a, b, dt, scale=16)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_spatial_softmax(dt):
    from models.coattention import CoAttention_CNN
    from oracle import ref_cpu as R
    m = CoAttention_CNN()
    for (n, h, w, c) in [(2, 28, 28, 256), (3, 1, 1, 256), (2, 3, 5, 64)]:
        s = torch.randn(n, h, w, 1, device=DEV).to(dt).requires_grad_(True)
        hs = torch.randn(n, h, w, c, device=DEV).to(dt).requires_grad_(True)
        y = m(s, hs)
        sr, hr = s.detach().float().requires_grad_(True), hs.detach().float().requires_grad_(True)
        yr = R.coattention(sr, hr)
        _close(y, yr, dt, scale=1)
        g = torch.randn_like(yr)
        y.backward(g.to(dt))
        yr.backward(g)
        _close(s.grad, sr.grad, dt, scale=2)
        _close(hs.grad, hr.grad, dt, scale=1)


@pytest.mark.parametrize("gap", [4.0, 9.0, 14.0])
def test_spatial_softmax_peaked_bwd_vs_fp64(gap):
    """The P4-level co-attention of the C2 parity case (round-4 probe,
    tools/probes/p4_chain.py): regression scores of magnitude ~300 over a
    14x14 level make the spatial softmax nearly one-hot (1 - a_peak ~
    e^-gap), and the score gradient at the peak, a (da_p - sum a da), is a
    cancellation of two nearly equal terms. Against fp64 arithmetic on the
    same fp32 operands, the GPU backward (fp64 accumulation of da and of the
    weighted sum over the fp32 softmax it stored) must be at least as
    accurate as the fp32 reference formula (torch fp32 softmax backward,
    what TF computes): error <= 3x the fp32 oracle's + 1e-7 of max."""
    from models.coattention import CoAttention_CNN
    from oracle import ref_cpu as R
    m = CoAttention_CNN()
    g = torch.Generator().manual_seed(int(gap))
    n, h, w, c = 2, 14, 14, 256
    score = torch.randn(n, h, w, 1, generator=g) * 100.0
    score[0, 7, 7, 0] = score[0].max() + gap
    score[1, 3, 9, 0] = score[1].max() + gap
    hs = torch.randn(n, h, w, c, generator=g) * 400.0
    dctx = torch.randn(n, h, w, c, generator=g) * 1e-4
    s_d, hs_d = score.to(DEV).requires_grad_(True), hs.to(DEV).requires_grad_(True)
    m(s_d, hs_d).backward(dctx.to(DEV))
    torch.cuda.synchronize()
    grads = {}
    for dt in (torch.float64, torch.float32):
        sr = score.to(dt).requires_grad_(True)
        R.coattention(sr, hs.to(dt)).backward(dctx.to(dt))
        grads[dt] = sr.grad.double()
    ref = grads[torch.float64]
    mx = float(ref.abs().max())
    eg = float((s_d.grad.cpu().double() - ref).abs().max()) / mx
    ec = float((grads[torch.float32] - ref).abs().max()) / mx
    print(f"peaked spatial softmax (gap {gap}): score-gradient max rel err vs fp64 gpu {eg:.2e} cpu32 {ec:.2e}")
    assert eg <= 3 * ec + 1e-7, (eg, ec)


def test_coattention_known_answer():
    """coattention.py:44-51 sample: uniform score over 7x7 -> ctx = hs / 49."""
    from models.coattention import CoAttention_CNN
    score = torch.ones(1, 7, 7, 1, device=DEV)
    hs = torch.arange(147, dtype=torch.float32, device=DEV).reshape(1, 7, 7, 3)
    out = CoAttention_CNN()(score, hs)
    torch.cuda.synchronize()
    ref = torch.tensor([2.9387755, 2.9591837, 2.9795918])
    assert torch.allclose(out[0, 6, 6].cpu(), ref, atol=1e-6)


# ------------------------------------------------------------- attention
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 8, 31, 31, 64, "causal"), (3, 8, 1, 196, 64, None), (2, 8, 31, 1, 64, None),
                                   (2, 8, 16, 1024, 64, None), (2, 8, 1, 0, 64, None), (2, 2, 40, 40, 32, "causal"),
                                   # one-query (fused) path: Lk 1 / 9 / 49, key padding mask, H < 8, D < 64,
                                   # and Lk above the fused kernel's LDS limit (general path)
                                   (5, 8, 1, 1, 64, None), (3, 8, 1, 9, 64, "keypad"), (4, 8, 1, 49, 64, None),
                                   (2, 3, 1, 70, 32, "keypad"), (2, 8, 1, 1024, 64, None),
                                   # one-query multi-wave path (bf16, D 64, Lk >= 128): ragged tail, masked
                                   (3, 8, 1, 130, 64, None), (3, 8, 1, 784, 64, "keypad"),
                                   # fused short-sequence path (Lq, Lk <= 32, D <= 64): ragged sizes,
                                   # odd D, key padding broadcast over queries, the 32 x 32 limit
                                   (3, 8, 7, 5, 64, "keypad"), (2, 3, 32, 32, 32, "causal"),
                                   (2, 8, 20, 9, 48, None), (1, 1, 2, 32, 8, "keypad"), (3, 4, 33, 32, 64, None),
                                   # the MFMA form of that path (bf16, D 64): full 32 x 32 and ragged masked
                                   (3, 8, 32, 32, 64, "causal"), (2, 8, 13, 17, 64, "keypad")])
def test_attention(dt, shape):
    from fpnmt import ops
    from oracle import ref_cpu as R
    B, H, Lq, Lk, D, mk = shape
    q = torch.randn(B, Lq, H * D, device=DEV).to(dt).requires_grad_(True)
    k = torch.randn(B, Lk, H * D, device=DEV).to(dt).requires_grad_(True)
    v = torch.randn(B, Lk, H * D, device=DEV).to(dt).requires_grad_(True)
    mask = None
    if mk == "causal":
        tok = torch.randint(1, 50, (B, Lq), device=DEV)
        tok[0, Lq - 5:] = 0
        mask = R.create_masks(tok.cpu()).to(DEV)
    elif mk == "keypad":
        mask = (torch.rand(B, 1, 1, Lk, generator=torch.Generator().manual_seed(Lk)) < 0.3).float().to(DEV)
        mask[..., 0] = 0.0  # at least one key kept per row
    out, w = ops.AttentionFn.apply(q, k, v, mask, H, 1.0 / math.sqrt(D))
    qr, kr, vr = [t.detach().float().requires_grad_(True) for t in (q, k, v)]
    sp = lambda x: x.reshape(B, -1, H, D).permute(0, 2, 1, 3)
    o_r, w_r = R.scaled_dot_product_attention(sp(qr), sp(kr), sp(vr), mask)
    o_r = o_r.permute(0, 2, 1, 3).reshape(B, Lq, H * D)
    _close(out, o_r, dt, scale=2)
    _close(w, w_r, dt, scale=1)
    g = torch.randn_like(o_r)
    out.backward(g.to(dt))
    o_r.backward(g)
    torch.cuda.synchronize()
    _close(q.grad, qr.grad, dt, scale=4)
    if Lk:
        _close(k.grad, kr.grad, dt, scale=4)
        _close(v.grad, vr.grad, dt, scale=4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("lks", [(196, 49, 9, 0), (784, 196, 49, 9), (130, 1, 0, 64)])
def test_attention_views_grouped(dt, lks):
    """fpnmt_attention_fwd_views / _bwd_views (the EncoderLayer's per-view
    attentions of the baseline's one query row, one launch in bf16 incl. a
    keyless 0x0 view) against the oracle's attention per view, and fp32 (the
    per-view fallback) likewise."""
    from fpnmt import ops
    from oracle import ref_cpu as R
    B, H, D = 3, 8, 64
    g = torch.Generator(device=DEV).manual_seed(sum(lks))
    q = (torch.randn(B, 1, H * D, device=DEV, generator=g)).to(dt)
    ks = [torch.randn(B, lk, H * D, device=DEV, generator=g).to(dt) for lk in lks]
    vs = [torch.randn(B, lk, H * D, device=DEV, generator=g).to(dt) for lk in lks]
    O = torch.empty(B, len(lks) * H * D, device=DEV, dtype=dt)
    outs = [O[:, i * H * D:(i + 1) * H * D].view(B, 1, H * D) for i in range(len(lks))]
    states = ops._attn_fwd_views([(q, k, v) for k, v in zip(ks, vs)], None, H, 1.0 / math.sqrt(D), outs)
    dO = torch.randn(B, len(lks) * H * D, device=DEV, generator=g)
    grads = ops._attn_bwd_views([(st[0], st[1], st[2], st[3], st[4], st[6]) for st in states],
                                [dO[:, i * H * D:(i + 1) * H * D].to(dt).view(B, 1, H * D) for i in range(len(lks))])
    torch.cuda.synchronize()
    sp = lambda x: x.reshape(B, -1, H, D).permute(0, 2, 1, 3)  # noqa: E731
    for i, (k, v) in enumerate(zip(ks, vs)):
        qr, kr, vr = [t.detach().float().requires_grad_(True) for t in (q, k, v)]
        o_r, w_r = R.scaled_dot_product_attention(sp(qr), sp(kr), sp(vr), None)
        o_r = o_r.permute(0, 2, 1, 3).reshape(B, 1, H * D)
        if lks[i] == 0:
            assert float(outs[i].float().abs().max()) == 0.0
            assert float(grads[3 * i].float().abs().max()) == 0.0
            continue
        _close(outs[i], o_r, dt, scale=2)
        _close(states[i][4][..., :lks[i]], w_r, dt, scale=1)
        o_r.backward(dO[:, i * H * D:(i + 1) * H * D].to(dt).float().view(B, 1, H * D))
        _close(grads[3 * i], qr.grad, dt, scale=4)
        _close(grads[3 * i + 1], kr.grad, dt, scale=4)
        _close(grads[3 * i + 2], vr.grad, dt, scale=4)


@pytest.mark.parametrize("b,T,idt", [(32, 32, torch.int64), (3, 2, torch.int64), (5, 17, torch.int32),
                                     (32, 32, torch.int32)])
def test_decoder_targets(b, T, idt):
    """fpnmt_decoder_targets == tok[:, :-1], tok[:, 1:], create_masks(tar_inp)
    (utils/pipeline.py:66-69, transformer.py:42-67), bit for bit, from a
    row-strided int64 batch with padding."""
    from fpnmt import ops
    from oracle import ref_cpu as R
    g = torch.Generator().manual_seed(b * T)
    full = torch.randint(1, 9000, (b, T + 3), generator=g)
    for i in range(b):
        full[i, int(torch.randint(1, T + 1, (1,), generator=g)):] = 0
    tok = full.to(idt).to(DEV)[:, :T]  # row stride T + 3
    tin, tout, mask = ops.decoder_targets(tok)
    torch.cuda.synchronize()
    ref = full[:, :T]
    assert tin.dtype == torch.int32 and torch.equal(tin.cpu().long(), ref[:, :-1])
    assert torch.equal(tout.cpu().long(), ref[:, 1:])
    assert torch.equal(mask.cpu(), R.create_masks(ref[:, :-1]).float())


# ----------------------------------------------------- layernorm / embed
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(3, 17, 512), (64, 33, 512), (5, 9, 300), (4, 7, 1000), (2, 5, 1024), (3, 3, 8)])
def test_layernorm(dt, shape):
    from fpnmt.layers import LayerNormalization
    from oracle import ref_cpu as R
    b, t, d = shape
    ln = LayerNormalization(d).to(DEV)
    with torch.no_grad():
        ln.gamma.uniform_(0.5, 1.5)
        ln.beta.normal_()
    for use_res, use_pe in [(False, False), (True, False), (False, True)]:
        ln.gamma.grad = None
        ln.beta.grad = None
        x = (torch.randn(b, t, d, device=DEV) * 3 + 1).to(dt).requires_grad_(True)
        r = torch.randn(b, t, d, device=DEV).to(dt).requires_grad_(True) if use_res else None
        pe = torch.randn(40, d, device=DEV) if use_pe else None
        y = ln(x, residual=r, pe=pe)
        xr = x.detach().float().requires_grad_(True)
        rr = r.detach().float().requires_grad_(True) if use_res else None
        gm = ln.gamma.detach().clone().requires_grad_(True)
        bt = ln.beta.detach().clone().requires_grad_(True)
        yr = R.layer_norm(xr + rr if use_res else xr, gm, bt)
        if use_pe:
            yr = yr + pe[:t]
        _close(y, yr, dt, scale=4)
        g = torch.randn_like(yr)
        y.backward(g.to(dt))
        yr.backward(g)
        torch.cuda.synchronize()
        _close(x.grad, xr.grad, dt, scale=4)
        if use_res:
            _close(r.grad, rr.grad, dt, scale=4)
        _close(ln.gamma.grad, gm.grad, dt, scale=16)
        _close(ln.beta.grad, bt.grad, dt, scale=16)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_embedding_posenc(dt):
    from fpnmt.layers import Embedding
    emb = Embedding(100, 512).to(DEV)
    pe = torch.randn(32, 512, device=DEV)
    tok = torch.randint(0, 100, (4, 31), device=DEV)
    tok[0, :5] = 7  # duplicates
    y = emb(tok, pe, dt)
    ref = emb.embeddings.detach()[tok] + pe[:31]
    _close(y, ref, dt)
    g = torch.randn(4, 31, 512, device=DEV).to(dt)
    y.backward(g)
    dref = torch.zeros(100, 512, device=DEV).index_add_(0, tok.reshape(-1), g.float().reshape(-1, 512))
    torch.cuda.synchronize()
    _close(emb.embeddings.grad, dref, dt, scale=4)


def test_embedding_bwd_deterministic_and_norm():
    """C2-sized decoder input (32 x 31 positions, many duplicate and padding
    ids): the scatter-free backward sums each id's rows in position order
    (bitwise repeatable), and the IndexedSlices norm^2 (one row per position,
    duplicates counted) lands in the sumsq slot."""
    from fpnmt.layers import Embedding
    emb = Embedding(10000, 512).to(DEV)
    pe = torch.randn(32, 512, device=DEV)
    g0 = torch.Generator().manual_seed(3)
    tok = torch.randint(4, 60, (32, 31), generator=g0)
    tok[:, 20:] = 0
    tok = tok.to(DEV)
    g = torch.randn(32, 31, 512, generator=g0).to(DEV)
    grads, norms = [], []
    for _ in range(2):
        emb.embeddings.grad = None
        emb.sumsq_slot = torch.zeros(1, device=DEV)
        emb(tok, pe, torch.float32).backward(g)
        torch.cuda.synchronize()
        grads.append(emb.embeddings.grad.clone())
        norms.append(emb.sumsq_slot.clone())
    dref = torch.zeros(10000, 512, dtype=torch.float64).index_add_(0, tok.reshape(-1).cpu(),
                                                                   g.double().reshape(-1, 512).cpu())
    assert float((grads[0].double().cpu() - dref).abs().max()) <= 1e-4
    assert torch.equal(grads[0], grads[1]) and torch.equal(norms[0], norms[1])
    assert abs(float(norms[0]) - float((g.double() ** 2).sum())) <= 1e-5 * float((g.double() ** 2).sum())


def test_xent():
    from fpnmt import ops
    from oracle import ref_cpu as R
    logits = (torch.randn(4, 31, 1000, device=DEV) * 3).requires_grad_(True)
    lab = torch.randint(0, 1000, (4, 31), device=DEV)
    lab[1, 10:] = 0
    loss = ops.MaskedXentFn.apply(logits, lab)
    lr_ = logits.detach().clone().requires_grad_(True)
    ref = R.masked_loss(lab, lr_)
    loss.backward()
    ref.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(ref)) < 1e-5
    assert float((logits.grad - lr_.grad).abs().max()) < 1e-6


@pytest.mark.parametrize("const_lr", [None, 1e-2])
def test_amsgrad_matches_keras(const_lr):
    from fpnmt.arena import ParamArena
    from oracle import ref_cpu as R
    from utils.utils import CustomSchedule
    torch.manual_seed(0)
    ps = [("a", torch.nn.Parameter(torch.randn(300, 7))), ("emb", torch.nn.Parameter(torch.randn(50, 16))),
          ("c", torch.nn.Parameter(torch.randn(5)))]
    init = {n: p.detach().clone() for n, p in ps}
    ar = ParamArena(ps, DEV, sparse_names=["emb"])
    opt = R.KerasAMSGrad([n for n, _ in ps], [p.shape for _, p in ps], sparse=["emb"])
    sched = CustomSchedule(2048, 4000) if const_lr is None else const_lr
    lr_fn = sched if const_lr is None else (lambda it: const_lr)
    params = {n: v.clone() for n, v in init.items()}
    for step in range(3):
        grads = {n: torch.randn(p.shape) * (5 if n == "a" else 0.1) for n, p in ps}
        ar.zero_grad()
        for (n, p) in ps:
            p.grad.copy_(grads[n].to(DEV))
        emb_ss = float((grads["emb"].double() ** 2).sum()) * 1.7  # caller-supplied IndexedSlices norm
        ar.sumsq_slot(ps[1][1]).fill_(emb_ss)
        ar.amsgrad_step(sched)
        opt.apply(params, grads, lr_fn, norms={"emb": emb_ss})
    torch.cuda.synchronize()
    assert int(ar.step.item()) == 3
    for n, p in ps:
        assert torch.allclose(p.detach().cpu(), params[n], atol=1e-6, rtol=1e-5), n


def test_amsgrad_grad_scale_equals_averaged_grads():
    """DP folding: a SUM all-reduce over W ranks followed by grad_scale = 1/W
    (the embedding's caller-supplied IndexedSlices norm^2 scaled by 1/W^2)
    gives the same update as the averaged gradient."""
    from fpnmt.arena import ParamArena
    torch.manual_seed(1)
    W = 4
    out = []
    for scale in (1.0, 1.0 / W):
        ps = [("a", torch.nn.Parameter(torch.ones(1000))), ("emb", torch.nn.Parameter(torch.ones(64, 8)))]
        ar = ParamArena(ps, DEV, sparse_names=["emb"])
        g = torch.Generator().manual_seed(5)
        ga, ge = torch.randn(1000, generator=g), torch.randn(64, 8, generator=g)
        ess = float((ge.double() ** 2).sum()) * 1.3
        mult = 1.0 if scale == 1.0 else W
        for _ in range(2):
            ar.zero_grad()
            ps[0][1].grad.copy_((ga * mult).to(DEV))
            ps[1][1].grad.copy_((ge * mult).to(DEV))
            ar.sumsq_slot(ps[1][1]).fill_(ess * mult * mult)
            ar.amsgrad_step(1e-2, grad_scale=scale)
        torch.cuda.synchronize()
        out.append(ar.flat.detach().clone())
    assert float((out[0] - out[1]).abs().max()) <= 1e-6


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,c", [(992, 2048), (6272, 512), (25088, 256), (37, 12), (5, 3), (3000, 64)])
def test_act_bwd_bias_grad(dt, rows, c):
    """dz = dy * leaky'(y) and db += colsum(dz), with the caller's workspace
    and without it (the process scratch): per-chunk partials summed in chunk
    order either way, so the two agree bitwise."""
    from fpnmt import _lib as L
    g = torch.Generator().manual_seed(rows + c)
    dy = torch.randn(rows, c, generator=g).to(dt).to(DEV)
    y = torch.randn(rows, c, generator=g).to(dt).to(DEV)
    dz_ref = dy.float() * torch.where(y.float() > 0, 1.0, 0.2)
    db_ref = dz_ref.to(dt).float().sum(0).double()
    dbs = []
    for use_ws in (True, False):
        dz = torch.empty_like(dy)
        db = torch.full((c,), 0.5, device=DEV)
        ws = None
        if use_ws:
            ws = torch.empty(max(L.lib.fpnmt_act_bwd_ws_bytes(L.dtype_code(dt), rows, c) // 4, 1), device=DEV)
        L.call("fpnmt_act_bwd", L.dtype_code(dt), rows, c, L.ACT_CODES["leaky_relu"], 0.2, L.ptr(dy), L.ptr(y),
               L.ptr(dz), L.ptr(db), L.ptr(ws), 0.0, 0, None, L.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dz, dz_ref.to(dt))
        err = float((db.double().cpu() - 0.5 - db_ref.cpu()).abs().max())
        assert err <= 1e-5 * float(dz_ref.abs().sum(0).max()) + 1e-6, (use_ws, err)
        dbs.append(db)
    assert torch.equal(dbs[0], dbs[1])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows", [32, 992, 6272])
def test_dense_fused_dropout_residual(dt, rows):
    """Dense(x, dropout=p, residual=R) = R + dropout(x W + b) in the GEMM
    epilogue; the backward recomputes the same mask inside act_bwd: dbias,
    dW and dx all follow the kept set observed in the forward output."""
    import fpnmt
    from fpnmt import ops
    from fpnmt.layers import Dense
    fpnmt.ops.runtime.seed_tensor = torch.zeros(1, dtype=torch.int64, device=DEV)
    p = 0.25
    layer = Dense(512, 512).to(DEV)
    with torch.no_grad():
        layer.bias.normal_()
    x = torch.randn(rows, 512, device=DEV).to(dt).requires_grad_(True)
    R = torch.randn(rows, 512, device=DEV).to(dt).requires_grad_(True)
    y = layer(x, dropout=p, residual=R)
    # the kernel multiplies by the dt-rounded weights
    lin = (x.detach().float() @ layer.kernel.detach().to(dt).float() + layer.bias.detach())
    z = (y.detach().float() - R.detach().float())
    keep = z != 0
    frac = float(keep.float().mean())
    assert abs(frac - (1 - p)) < 0.02, frac
    tol = 1e-4 if dt == torch.float32 else 0.05
    assert float(((z - lin / (1 - p)) * keep).abs().max()) <= tol * (1 + float(lin.abs().max()))
    g = torch.randn(rows, 512, device=DEV).to(dt)
    y.backward(g)
    torch.cuda.synchronize()
    dz = g.float() * keep / (1 - p)
    assert torch.equal(R.grad, g)
    gb = layer.bias.grad.detach()
    # in bf16 a kept element whose |x W + b| is below half an ulp of R leaves
    # y == R, so `keep` (inferred from the output) can miss it: such elements
    # bound the extra bias-gradient difference
    amb = (~keep) & (lin.abs() <= 2.0 ** -6 * (R.detach().float().abs() + 1e-30)) if dt != torch.float32 else ~keep & False
    slack = (amb.float() * g.float().abs() / (1 - p)).sum(0)
    assert bool(((gb - dz.to(dt).float().sum(0)).abs() <= 1e-3 * float(dz.abs().sum(0).max()) + 1e-4 + slack).all())
    amb_g = amb.float() * g.float().abs() / (1 - p)
    rt = 1e-4 if dt == torch.float32 else 0.03
    dx_ref = dz.to(dt).float() @ layer.kernel.detach().t()
    slack_dx = amb_g @ layer.kernel.detach().abs().t()
    assert bool(((x.grad.float() - dx_ref).abs() <= rt * float(dx_ref.abs().max()) + slack_dx).all())
    dw_ref = x.detach().float().t() @ dz.to(dt).float()
    slack_dw = x.detach().float().abs().t() @ amb_g
    assert bool(((layer.kernel.grad - dw_ref).abs() <= rt * float(dw_ref.abs().max()) + slack_dw).all())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,fin,fout", [(8192, 512, 512), (6272, 512, 2048), (4000, 1024, 256)])
def test_dense_large(dt, rows, fin, fout):
    """Row-major Dense big enough for the pipelined kernel (bf16): forward with
    bias + leaky ReLU, bwd-data, bwd-filter and bias grads vs torch fp32."""
    from fpnmt.layers import Dense
    torch.manual_seed(rows + fin)
    layer = Dense(fin, fout, activation="leaky_relu").to(DEV)
    with torch.no_grad():
        layer.bias.normal_()
    x = torch.randn(rows, fin, device=DEV).to(dt).requires_grad_(True)
    y = layer(x)
    kern = layer.kernel.detach().clone().requires_grad_(True)
    bias = layer.bias.detach().clone().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    yr = F.leaky_relu(xr @ kern.to(dt).float() + bias, 0.2)
    _close(y, yr, dt, scale=max(1.0, math.sqrt(fin) * 0.3))
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    torch.cuda.synchronize()
    _close(x.grad, xr.grad, dt, scale=max(1.0, math.sqrt(fout)))
    _close(layer.kernel.grad, kern.grad, dt, scale=max(1.0, math.sqrt(rows) * 2))
    _close(layer.bias.grad, bias.grad, dt, scale=max(1.0, math.sqrt(rows) * 2))


@pytest.mark.parametrize("case", ["1x1s2", "1x1s2-linear", "empty-keys-attention"])
def test_captured_backward_replay_safe(case):
    """A captured backward re-zeroes what it accumulates into on EVERY replay
    (zero fills are kernel nodes: captured hipMemsetAsync nodes were measured
    not to, tools/probes/conv_noise.py) and reads no memory outside its graph:
    replays after 1e30 allocation noise equal the eager result."""
    import fpnmt
    from fpnmt.layers import Conv2D
    from fpnmt.train import capture_sequence
    fpnmt.set_precision("fp32")
    torch.manual_seed(1)
    out = {}
    if case.startswith("1x1s2"):
        layer = Conv2D(256, 128, 1, strides=2, padding="valid", activation=None if "linear" in case else "relu",
                       use_bias=False, frozen_bn=True).to(DEV)
        x = torch.randn(2, 28, 28, 256, device=DEV).requires_grad_(True)

        def run():
            x.grad = None
            layer.kernel.grad = None
            y = layer(x)
            (y * y).sum().backward()
            out["a"], out["b"] = x.grad.clone(), layer.kernel.grad.clone()
    else:
        from fpnmt import ops
        q = torch.randn(2, 3, 64, device=DEV).requires_grad_(True)
        k = torch.randn(2, 0, 64, device=DEV).requires_grad_(True)
        v = torch.randn(2, 0, 64, device=DEV).requires_grad_(True)

        def run():
            q.grad = None
            o, _ = ops.AttentionFn.apply(q, k, v, None, 1, 0.125)
            (o.float() + 1).sum().backward()
            out["a"], out["b"] = q.grad.clone(), o.detach().clone()
    run()
    torch.cuda.synchronize()
    ref = {kk: vv.clone() for kk, vv in out.items()}
    g = capture_sequence([run])[0]
    for _ in range(2):
        junk = [torch.full((1 << 26,), 1e30, device=DEV) for _ in range(4)]
        torch.cuda.synchronize()
        del junk
        g.replay()
        torch.cuda.synchronize()
        for kk in ref:
            assert float((out[kk] - ref[kk]).abs().max()) <= 1e-5 * max(1.0, float(ref[kk].abs().max())), kk


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_weight_prep_batched_layouts(dt):
    """fpnmt_weight_prep_batched (one launch over a model's weight layers):
    OHWI and flipped copies of convs (frozen BN scale folded, partial
    32-tiles) and Dense layers, bit-exact against torch permutes."""
    from fpnmt.layers import Conv2D, Dense, WeightPrepPlan
    torch.manual_seed(11)
    model = torch.nn.ModuleList([
        Conv2D(37, 70, 3, padding="same", use_bias=False, frozen_bn=True),
        Dense(100, 33), Conv2D(64, 64, 1), Conv2D(3, 64, 7, strides=2, padding=(3, 3, 3, 3)),
        Dense(512, 2048)]).to(DEV)
    with torch.no_grad():
        c0 = model[0]
        c0.bn_gamma.uniform_(0.5, 1.5)
        c0.bn_var.uniform_(0.5, 2)
        c0.refresh_bn()
    plan = WeightPrepPlan(model, [dt])
    plan.run()
    torch.cuda.synchronize()
    for m in model:
        r, s, c, k = m._rsck()
        w = m.kernel.detach().float().reshape(r, s, c, k)
        if getattr(m, "bn_scale", None) is not None:
            w = w * m.bn_scale.detach().float()
        wf, wb = m._copies[dt]
        ohwi = w.permute(3, 0, 1, 2).contiguous().to(dt).float()
        assert torch.equal(wf.float().reshape(k, r, s, c), ohwi)
        ld = m.flip_ld()
        flip = w.flip(0, 1).permute(2, 0, 1, 3).reshape(c, r * s * k).to(dt).float()
        got = wb.float()[: (c - 1) * ld + r * s * k].as_strided((c, r * s * k), (ld, 1))
        assert torch.equal(got, flip)


@pytest.mark.parametrize("batch", [2, 16])
def test_grouped_conv_bf16_matches_per_level(batch):
    """bf16 grouped conv (one launch per pass over the FPN levels: the pipe /
    split-K forward, the pipelined weight gradient with its K-tiles laid end to
    end over the levels) against the same layer run level by level."""
    import fpnmt
    from fpnmt.layers import Conv2D
    fpnmt.set_precision("bf16")
    torch.manual_seed(batch)
    layer = Conv2D(256, 256, 3, padding="same", activation="relu").to(DEV)
    with torch.no_grad():
        layer.bias.normal_(0, 0.1)
    sizes = (28, 14, 7, 4, 2)
    xs = [torch.randn(batch, s, s, 256, device=DEV).to(torch.bfloat16) for s in sizes]
    gs = [torch.randn(batch, s, s, 256, device=DEV).to(torch.bfloat16) for s in sizes]
    res = {}
    for mode in ("grouped", "single"):
        layer.kernel.grad = None
        layer.bias.grad = None
        xi = [x.clone().requires_grad_(True) for x in xs]
        ys = layer(xi) if mode == "grouped" else [layer(x) for x in xi]
        torch.autograd.backward(ys, gs)
        torch.cuda.synchronize()
        res[mode] = ([y.detach().float() for y in ys], [x.grad.float() for x in xi],
                     layer.kernel.grad.detach().clone(), layer.bias.grad.detach().clone())
    (yg, dxg, dwg, dbg), (ys_, dxs, dws, dbs) = res["grouped"], res["single"]
    for a, b in zip(yg, ys_):  # bf16 outputs: a rounding step apart at most
        assert float((a - b).abs().max()) <= 2 ** -7 * max(1.0, float(b.abs().max()))
    for a, b in zip(dxg, dxs):
        assert float((a - b).abs().max()) <= 2 ** -7 * max(1.0, float(b.abs().max()))
    # fp32 weight gradients of the same bf16 products, summed in another order
    assert float((dwg - dws).abs().max()) <= 1e-3 * float(dws.abs().max())
    assert float((dbg - dbs).abs().max()) <= 1e-3 * float(dbs.abs().max())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["relu", "relu6"])
@pytest.mark.parametrize("case", [(2, 9, 9, 64, 32, 3), (16, 28, 28, 128, 256, 3), (16, 28, 28, 256, 512, 1),
                                  (32, 7, 7, 512, 512, 3), (2, 5, 5, 24, 40, 1)])
def test_conv_bwd_data_act_fused(dt, act, case):
    """fpnmt_conv2d_bwd_data_act == fpnmt_conv2d_bwd_data followed by the
    producing layer's 0/1 activation derivative, bit for bit (register-staged,
    LDS-DMA pipelined and split-K-through-workspace dgrad shapes)."""
    from fpnmt import _lib as L
    from fpnmt.layers import Conv2D
    n, h, w, c, k, r = case
    torch.manual_seed(n + h + c + k)
    layer = Conv2D(c, k, r, padding="same").to(DEV)
    wflip = layer.compute_weights(dt)[1]
    dz = torch.randn(n, h, w, k, device=DEV).to(dt)
    y_in = (torch.randn(n, h, w, c, device=DEV) * 4).to(dt)
    if act == "relu":
        y_in = y_in.clamp_min(0)
    else:
        y_in = y_in.clamp(0, 6)
    d = layer.desc(n, h, w, c, dt)
    plain = torch.empty(n, h, w, c, dtype=dt, device=DEV)
    fused = torch.full_like(plain, float("nan"))
    L.call("fpnmt_conv2d_bwd_data", d, dz.data_ptr(), wflip.data_ptr(), plain.data_ptr(), 0, L.stream_ptr())
    L.call("fpnmt_conv2d_bwd_data_act", d, dz.data_ptr(), wflip.data_ptr(), fused.data_ptr(), y_in.data_ptr(),
           L.ACT_CODES[act], L.stream_ptr())
    torch.cuda.synchronize()
    yf = y_in.float()
    mask = (yf > 0) if act == "relu" else ((yf > 0) & (yf < 6))
    ref = (plain.float() * mask.float()).to(dt)
    assert torch.equal(fused, ref)
    assert int(mask.sum()) not in (0, mask.numel())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_bwd_data_grouped_act_fused(dt):
    """Grouped (pyramid-level) bwd-data with the per-level act' mask."""
    from fpnmt import ops
    from fpnmt import _lib as L
    from fpnmt.layers import Conv2D
    torch.manual_seed(5)
    layer = Conv2D(256, 256, 3, padding="same").to(DEV)
    shapes = [(4, 28, 28), (4, 14, 14), (4, 7, 7), (4, 4, 4), (4, 2, 2)]
    xs = [(torch.randn(*s, 256, device=DEV) * 2).clamp_min(0).to(dt) for s in shapes]
    dzs = [torch.randn(*s, 256, device=DEV).to(dt) for s in shapes]
    s = L.stream_ptr()
    plain = ops._grouped_bwd_data(layer, xs, dzs, s)
    fused = ops._grouped_bwd_data(layer, xs, dzs, s, act_in=L.ACT_RELU)
    torch.cuda.synchronize()
    for p, f, x in zip(plain, fused, xs):
        assert torch.equal(f, (p.float() * (x.float() > 0).float()).to(dt))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", [256, 64, 1024])
def test_conv_single_filter_grouped(dt, c):
    """k = 1 convs (the regression head 256 -> 1) run as streaming kernels
    (conv_n1.hip) over all pyramid levels: fwd, bwd-data (plain and with the
    producer's ReLU mask) and the two-pass deterministic bwd-filter, against
    fp64 torch on the same rounded operands; two runs bitwise equal."""
    from fpnmt import ops
    from fpnmt import _lib as L
    from fpnmt.layers import Conv2D
    torch.manual_seed(c)
    layer = Conv2D(c, 1, 3, padding="same").to(DEV)
    with torch.no_grad():
        layer.bias.fill_(0.25)
    shapes = [(4, 28, 28), (4, 14, 14), (4, 7, 7), (4, 3, 3), (4, 1, 1)]
    xs = [torch.randn(*s, c, device=DEV).clamp_min(0).to(dt) for s in shapes]
    dzs = [torch.randn(*s, 1, device=DEV).to(dt) for s in shapes]
    s = L.stream_ptr()
    ys = ops._grouped_fwd(layer, xs)
    ys2 = ops._grouped_fwd(layer, xs)
    plain = ops._grouped_bwd_data(layer, xs, dzs, s)
    masked = ops._grouped_bwd_data(layer, xs, dzs, s, act_in=L.ACT_RELU)
    grads = []
    for _ in range(2):
        layer.kernel.grad = torch.zeros_like(layer.kernel)
        ops._grouped_bwd_filter(layer, xs, dzs, s)
        grads.append(layer.kernel.grad.clone())
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(ys, ys2))
    assert torch.equal(grads[0], grads[1])
    w = layer.kernel.detach().to(dt).double().cpu()  # HWIO (3, 3, c, 1)
    wgrad = torch.zeros(3, 3, c, 1, dtype=torch.float64)
    for x, y, dz, dxp, dxm in zip(xs, ys, dzs, plain, masked):
        xd = x.double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
        wd = w.permute(3, 2, 0, 1).contiguous().requires_grad_(True)
        yr = F.conv2d(xd, wd, padding=1) + 0.25
        _close(y, yr.permute(0, 2, 3, 1).float().to(DEV), dt, scale=math.sqrt(9 * c))
        yr.backward(dz.double().cpu().permute(0, 3, 1, 2))
        dx_ref = xd.grad.permute(0, 2, 3, 1).float().to(DEV)
        _close(dxp, dx_ref, dt, scale=3.0)
        assert torch.equal(dxm, (dxp.float() * (x.float() > 0).float()).to(dt))
        wgrad += wd.grad.permute(2, 3, 1, 0)
    _close(grads[0], wgrad.float().to(DEV), dt, scale=max(1.0, float(wgrad.abs().max())))


def test_gemm_log_env(tmp_path):
    """FPNMT_GEMM_LOG (the library's only environment variable) logs one line
    per GEMM launch and changes nothing else: a child process with it set runs
    a Dense forward and writes the launch's shape."""
    import os
    import subprocess
    import sys
    log = tmp_path / "gemm.log"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import torch, fpnmt; from fpnmt.layers import Dense; "
            "d = Dense(64, 96).cuda(); y = d(torch.randn(40, 64, device='cuda')); torch.cuda.synchronize(); "
            "print(float(y.abs().sum()))" % os.path.join(root, "fpn-mt-image-captioning_amd"))
    env = dict(os.environ, FPNMT_GEMM_LOG=str(log))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = log.read_text().splitlines()
    assert any("M=40 N=96 K=64" in ln for ln in lines), lines


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bias_grad_deferred_equals_immediate(dt):
    """fpnmt_bias_grad (db += column sums of dy) queued inside a deferred
    region and run at the flush — one-chunk (direct add) and multi-chunk
    (partials + ordered colsum) grids, aligned and unaligned rows, two sums
    into one db — equals the immediate launches bit for bit and the fp64 sum
    to fp32 rounding; dy is released by the caller before the flush."""
    from fpnmt import _lib as L
    from fpnmt import ops
    shapes = [(992, 512), (32, 2048), (6272, 1024), (31, 3), (200704, 64)]
    g = torch.Generator().manual_seed(5)
    dys = [torch.randn(r, c, generator=g).to(dt).to(DEV) for r, c in shapes]
    out = {}
    for defer in (False, True):
        dbs = [torch.full((c,), 0.5, device=DEV) for _, c in shapes]
        with L.deferred_reductions(defer):
            s = L.stream_ptr()
            for dy, db, (r, c) in zip(dys, dbs, shapes):
                tmp = dy.clone()  # the only reference is dropped right after the call
                ops.bias_grad(L.dtype_code(dt), r, c, tmp, db.data_ptr(), s)
                del tmp
            # a second sum into the first db (ordered after the queued one)
            ops.bias_grad(L.dtype_code(dt), shapes[0][0], shapes[0][1], dys[0], dbs[0].data_ptr(), s)
        torch.cuda.synchronize()
        out[defer] = dbs
    for a, b, dy in zip(out[False], out[True], dys):
        assert torch.equal(a, b)
    ref = 0.5 + 2 * dys[0].double().sum(0)
    assert torch.allclose(out[True][0].double(), ref, rtol=1e-5, atol=1e-3)
    for db, dy in zip(out[True][1:], dys[1:]):
        assert torch.allclose(db.double(), 0.5 + dy.double().sum(0), rtol=1e-5, atol=1e-3)


def test_conv_wide_tile_path_bf16():
    """The wide 3x3 convs' 128x256 tile (csrc/gemm_pipe.h, 8 waves, 3-stage
    ring with the next K-tile's DMA spread between the k-steps and MFMA
    priority; pipe_cfg picks it at N >= 256, K >= 2048 and >= 192 tiles of
    128x256: here the C2 P3 head conv, 32x28x28x256 -> 256, M = 25088, 196
    tiles), and its backward: bwd-data on the same tile (K = 2304) and the
    weight gradient. fp32 torch CPU reference on the same bf16-rounded operands;
    the bar is the output's own bf16 rounding plus a small absolute term
    (bf16 products summed in fp32 in a different order)."""
    from fpnmt.layers import Conv2D
    torch.manual_seed(11)
    # no activation: a ReLU mask flipped by rounding at a ~0 pre-activation
    # would make the backward comparison depend on ties, not on the kernels
    layer = Conv2D(256, 256, 3, padding="same", activation=None, use_bias=True).to(DEV)
    with torch.no_grad():
        layer.bias.normal_(0, 0.1)
    x = (torch.rand(32, 28, 28, 256, device=DEV) * 2 - 1).to(torch.bfloat16).requires_grad_(True)
    y = layer(x)
    # the reference on the host (torch CPU fp32; no GPU library kernels)
    xr = x.detach().float().cpu().permute(0, 3, 1, 2).requires_grad_(True)
    kern = layer.kernel.detach().cpu().clone().requires_grad_(True)
    wq = kern.to(torch.bfloat16).float()
    yr = F.conv2d(xr, wq.permute(3, 2, 0, 1), layer.bias.detach().float().cpu(), padding=1)

    def check(a, b, rel=2.0 ** -7, absf=2e-3):
        a, b = a.detach().float().cpu(), b.detach().float().cpu()
        err = (a - b).abs()
        bound = rel * b.abs() + absf * float(b.abs().max())
        bad = int((err > bound).sum())
        assert bad == 0, f"{bad} elements off, worst {float(err.max()):.3e} at |ref| max {float(b.abs().max()):.3e}"

    check(y, yr.permute(0, 2, 3, 1))
    g = (torch.randn(32, 28, 28, 256, device=DEV) * 0.1).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float().cpu().permute(0, 3, 1, 2))
    torch.cuda.synchronize()
    check(x.grad, xr.grad.permute(0, 2, 3, 1))
    check(layer.kernel.grad, kern.grad, rel=2.0 ** -7, absf=5e-3)


@pytest.mark.parametrize("case", ["p3_3x3", "r5_3x3", "short_1x1", "grouped"])
def test_conv_bias_grad_folded_into_wgrad(case, monkeypatch):
    """A Conv2D's bias gradient in its weight-gradient launch
    (fpnmt_conv2d_bwd_filter_bias / _grouped_bias, config.fuse_bias_wgrad):
    the LDS-DMA wgrad kernel sums the dz fragments it reads (k-steps dealt over
    the (m-tile, wave row) pairs, partial rows summed in order). No activation,
    so dz == dy and the column pass would read dy itself. Cases: the P3 head
    conv (split-K slabs), res5's 3x3 at 7x7 (few pixels), a short 1x1 the
    LDS-DMA kernel does not take (the fallback column pass) and the grouped
    head conv over five levels. db against the fp64 column sums of dy (rtol
    1e-5: fp32 sums of bf16 values in another order); dw and dx bitwise those
    of the unfolded path (the fold adds no work to them)."""
    import fpnmt
    from fpnmt.layers import Conv2D
    torch.manual_seed(7)
    geo = {"p3_3x3": (32, 28, 256, 256, 3), "r5_3x3": (32, 7, 512, 512, 3), "short_1x1": (8, 7, 512, 256, 1),
           "grouped": (16, 28, 256, 256, 3)}[case]
    n, h, cin, cout, k = geo
    layer = Conv2D(cin, cout, k, padding="same", activation=None, use_bias=True).to(DEV)
    sizes = (h, 14, 7, 4, 2) if case == "grouped" else (h,)
    xs = [(torch.rand(n, s, s, cin, device=DEV) * 2 - 1).to(torch.bfloat16) for s in sizes]
    gs = [(torch.randn(n, s, s, cout, device=DEV) * 0.1).to(torch.bfloat16) for s in sizes]
    res = {}
    for fold in (False, True):
        monkeypatch.setattr(fpnmt.config, "fuse_bias_wgrad", fold)
        layer.kernel.grad = None
        layer.bias.grad = None
        xi = [x.clone().requires_grad_(True) for x in xs]
        ys = layer(xi) if case == "grouped" else [layer(xi[0])]
        torch.autograd.backward(ys, gs)
        torch.cuda.synchronize()
        res[fold] = (layer.bias.grad.detach().clone(), layer.kernel.grad.detach().clone(), [x.grad.clone() for x in xi])
    ref = sum(g.double().sum((0, 1, 2)) for g in gs).cpu()
    for fold in (False, True):
        db = res[fold][0].double().cpu()
        assert torch.allclose(db, ref, rtol=1e-5, atol=1e-4 * float(ref.abs().max())), (fold, float((db - ref).abs().max()))
    assert torch.equal(res[False][1], res[True][1])
    for a, b in zip(res[False][2], res[True][2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,h", [(32, 28), (33, 28), (64, 28), (64, 14), (32, 14)])
def test_conv_wide_tiles_bitwise(n, h, monkeypatch):
    """The wide conv class's two loader tiles (csrc/gemm_dispatch.h
    wide_cfg, forced by FPNMT_WIDE_CFG: 128x256 cfg 6; the same image at a
    112-row M step, rows 112-127 fed the zero chunk, cfg 10) give the same K
    order per output element, so the forward,
    (14x14 at batch 64 / 32: the 128x128 loader class, cfg 7 against its
    112-row M step cfg 11; FPNMT_WIDE_CFG=6 keeps the 128-row step there too)
    the bwd-data (same class: K = 2304) and the weight gradient are bitwise
    equal; ragged M (33 images: partial last tiles) and batch 64 (two waves of
    blocks) included. The forward is also bounded against a torch CPU fp32 conv
    on the same bf16 operands (the output's bf16 rounding + 1e-2 absolute)."""
    from fpnmt.layers import Conv2D
    torch.manual_seed(5)
    layer = Conv2D(256, 256, 3, padding="same", activation="relu", use_bias=True).to(DEV)
    x0 = (torch.rand(n, h, h, 256, device=DEV) * 2 - 1).to(torch.bfloat16)
    g = (torch.randn(n, h, h, 256, device=DEV) * 0.1).to(torch.bfloat16)
    outs = {}
    for cfg in ("6", "10"):
        monkeypatch.setenv("FPNMT_WIDE_CFG", cfg)
        layer.kernel.grad = None
        x = x0.clone().requires_grad_(True)
        y = layer(x)
        y.backward(g)
        torch.cuda.synchronize()
        outs[cfg] = (y.detach().clone(), x.grad.clone(), layer.kernel.grad.clone())
    for a, b in zip(outs["6"], outs["10"]):
        assert torch.equal(a, b)
    xr = x0.float().cpu().permute(0, 3, 1, 2)
    wq = layer.kernel.detach().cpu().to(torch.bfloat16).float()
    yr = F.relu(F.conv2d(xr, wq.permute(3, 2, 0, 1), layer.bias.detach().float().cpu(), padding=1))
    err = (outs["6"][0].float().cpu() - yr.permute(0, 2, 3, 1)).abs()
    assert float(err.max()) <= 2.0 ** -7 * float(yr.abs().max()) + 1e-2


@pytest.mark.parametrize("n,h,pad", [(2, 224, 3), (2, 200, 3), (1, 512, 3)])
def test_stem_bwd_filter_vs_fp32(n, h, pad):
    """The ResNet stem's weight gradient (7x7 stride 2 over 3 channels, k 64:
    csrc/conv_stem.hip stem_wgrad_kernel, per-block fp32 slabs + the ordered
    reduce) against torch's fp32 conv2d weight gradient on the same bf16
    operands, times the folded BN scale, added into an existing gradient;
    224^2 (wo 112), 200^2 (wo 100: padded k columns), 512^2 (wo 256, the
    C3 form); outside and inside a deferred-reduction region, bitwise the
    same and run to run (fixed rows per block, split-ordered sum)."""
    import ctypes as C
    import torch.nn.functional as F
    from fpnmt import _lib as L
    g = torch.Generator().manual_seed(11 + h)
    x = (torch.rand(n, h, h, 3, generator=g) * 2 - 1).bfloat16()
    ho = (h + 2 * pad - 7) // 2 + 1
    dz = (torch.randn(n, ho, ho, 64, generator=g) * 0.5).bfloat16()
    scale = (0.5 + torch.rand(64, generator=g))
    base = torch.randn(7, 7, 3, 64, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 3, 7, 7), dz.float().permute(0, 3, 1, 2),
                                      stride=2, padding=pad)  # (64, 3, 7, 7)
    ref = base + ref.permute(2, 3, 1, 0) * scale
    d = L.ConvDesc(n=n, h=h, w=h, c=3, k=64, r=7, s=7, stride_h=2, stride_w=2, pad_t=pad, pad_b=pad, pad_l=pad,
                   pad_r=pad, dtype=L.dtype_code(torch.bfloat16), act=0, act_alpha=0.0)
    xd, dzd, sd = x.to(DEV), dz.to(DEV), scale.to(DEV)
    outs = []
    for defer in (False, True, True):
        dw = base.clone().to(DEV)
        with L.deferred_reductions(defer):
            L.call("fpnmt_conv2d_bwd_filter", C.byref(d), L.ptr(xd), L.ptr(dzd), L.ptr(sd), L.ptr(dw),
                   L.stream_ptr())
        torch.cuda.synchronize()
        outs.append(dw.cpu())
    err = (outs[0] - ref).abs().max().item()
    print(f"stem wgrad {n}x{h}^2: max|d| {err:.3e} of max|ref| {ref.abs().max().item():.3e}")
    # the same bf16 products in fp32, other summation order
    assert err <= 2e-4 * ref.abs().max().item() + 1e-4
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
