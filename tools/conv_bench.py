"""Per-shape forward-conv timing through the library (HIP events on the
launching stream): the ResNet-50-FPN forward convs at batch 64 (the
north_star headline) and the C2 step's dominant 3x3. Used for kernel A/B work
and as the target of rocprofv3 --pmc passes.

python tools/conv_bench.py [--iters N] [--only name,name] [--lib path/to/libfpnmt.so]
(--lib: time another build of the library in the same process layout, for
same-box A/B runs; tools/ab/ holds such builds, git-ignored)"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fpn-mt-image-captioning_amd"), ROOT]
import torch  # noqa: E402

# name: (n, h, w, c, k, r, stride, residual, act)
SHAPES = {
    "r2_3x3": (64, 56, 56, 64, 64, 3, 1, False, "relu"),
    "r3_3x3": (64, 28, 28, 128, 128, 3, 1, False, "relu"),
    "r4_3x3": (64, 14, 14, 256, 256, 3, 1, False, "relu"),
    "r5_3x3": (64, 7, 7, 512, 512, 3, 1, False, "relu"),
    "fpn_p3": (64, 28, 28, 256, 256, 3, 1, False, "relu"),
    "c2_p3_b32": (32, 28, 28, 256, 256, 3, 1, False, "relu"),
    "r2_a0": (64, 56, 56, 64, 64, 1, 1, False, "relu"),
    "r2_a": (64, 56, 56, 256, 64, 1, 1, False, "relu"),
    "r2_c": (64, 56, 56, 64, 256, 1, 1, True, "relu"),
    "r2_sc": (64, 56, 56, 64, 256, 1, 1, False, None),
    "r3_a0": (64, 56, 56, 256, 128, 1, 2, False, "relu"),
    "r3_sc": (64, 56, 56, 256, 512, 1, 2, False, None),
    "r3_a": (64, 28, 28, 512, 128, 1, 1, False, "relu"),
    "r3_c": (64, 28, 28, 128, 512, 1, 1, True, "relu"),
    "r4_a0": (64, 28, 28, 512, 256, 1, 2, False, "relu"),
    "r4_sc": (64, 28, 28, 512, 1024, 1, 2, False, None),
    "r4_a": (64, 14, 14, 1024, 256, 1, 1, False, "relu"),
    "r4_c": (64, 14, 14, 256, 1024, 1, 1, True, "relu"),
    "r5_a0": (64, 14, 14, 1024, 512, 1, 2, False, "relu"),
    "r5_sc": (64, 14, 14, 1024, 2048, 1, 2, False, None),
    "r5_a": (64, 7, 7, 2048, 512, 1, 1, False, "relu"),
    "r5_c": (64, 7, 7, 512, 2048, 1, 1, True, "relu"),
    "lat3": (64, 28, 28, 512, 256, 1, 1, False, None),
    "lat4": (64, 14, 14, 1024, 256, 1, 1, False, None),
    "lat5": (64, 7, 7, 2048, 256, 1, 1, False, None),
}


def run(name, iters, check):
    import fpnmt
    from fpnmt.layers import Conv2D, Init
    n, h, w, c, k, r, st, res, act = SHAPES[name]
    conv = Conv2D(c, k, r, strides=st, padding="same", activation=act, kernel_initializer="he_normal",
                  init=Init(torch.Generator().manual_seed(1))).cuda()
    x = (torch.rand(n, h, w, c, device="cuda") * 2 - 1).to(torch.bfloat16)
    ho, wo = -(-h // st), -(-w // st)
    rr = (torch.rand(n, ho, wo, k, device="cuda") * 2 - 1).to(torch.bfloat16) if res else None
    with torch.no_grad():
        y = conv(x, rr)
        if check:
            xf = x.float().permute(0, 3, 1, 2)
            wf = conv.kernel.detach().float().permute(3, 2, 0, 1)
            pad = (r - 1) // 2 if st == 1 else 0
            if st == 2 and r == 1:
                ref = torch.nn.functional.conv2d(xf, wf, stride=2)
            else:
                ref = torch.nn.functional.conv2d(xf, wf, padding=pad, stride=st)
            ref = ref.permute(0, 2, 3, 1) + conv.bias.detach().float()
            if rr is not None:
                ref = ref + rr.float()
            if act == "relu":
                ref = torch.relu(ref)
            err = float((y.float() - ref).abs().max() / ref.abs().max())
        else:
            err = float("nan")
        for _ in range(3):
            conv(x, rr)
        torch.cuda.synchronize()
        st_ = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st_)
        for _ in range(iters):
            conv(x, rr)
        e1.record(st_)
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    m = n * ho * wo
    flop = 2.0 * m * k * r * r * c
    byts = (x.numel() + m * k * (2 if res else 1)) * 2 + k * r * r * c * 2
    print(f"{name:10s} M={m:7d} N={k:5d} K={r * r * c:5d}  {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TF/s "
          f"({flop / ms / 1e9 / 25:5.1f}%)  {byts / ms / 1e6:7.0f} GB/s  relerr {err:.1e}", flush=True)
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    if a.lib:
        os.environ["FPNMT_LIBRARY"] = os.path.abspath(a.lib)
    import fpnmt
    fpnmt.set_precision("bf16")
    names = [s for s in a.only.split(",") if s] or list(SHAPES)
    tot = 0.0
    for nm in names:
        tot += run(nm, a.iters, a.check)
    print(f"total {tot * 1e3:.1f} us")


if __name__ == "__main__":
    main()
