"""Attainable bound of the R50-FPN headline forward (bench.py headline_probe:
keras-resnet ResNet-50 C2..C5 + FPN P3..P7, 224^2, batch 64, bf16): per conv
max(FLOP / 2.5 PF, HBM bytes / 8 TB/s) with the algorithmic bytes (input once,
weights once, output once, + the residual), unfused (one launch per conv, as
the library runs them) and with each ResNet bottleneck fused (only the block's
input and output, and a projection's input, touch HBM).
  python tools/attainable_r50fpn.py > profiles/r05/attainable_r50fpn.txt"""
B, PEAK, HBM = 64, 2.5e15, 8e12


def conv(rows, name, h, w, cin, cout, k, s, res=False):
    ho, wo = -(-h // s), -(-w // s)
    m, kk = B * ho * wo, k * k * cin
    byt = 2 * (B * h * w * cin + kk * cout + m * cout * (2 if res else 1))
    rows.append((name, 2.0 * m * kk * cout, byt))
    return ho, wo


def main():
    rows, blocks = [], []
    conv(rows, "stem 7x7/2 3->64", 224, 224, 3, 64, 7, 2)
    rows.append(("maxpool 3x3/2", 0.0, 2 * B * (112 * 112 + 56 * 56) * 64))
    h = w = 56
    cin = 64
    C = {}
    for si, (mid, out, n, s) in enumerate([(64, 256, 3, 1), (128, 512, 4, 2), (256, 1024, 6, 2), (512, 2048, 3, 2)]):
        for b in range(n):
            st = s if b == 0 else 1
            nm = f"res{si + 2}{'abcdef'[b]}"
            i0 = len(rows)
            ho, wo = conv(rows, f"{nm} 1x1a {cin}->{mid}" + ("/2" if st > 1 else ""), h, w, cin, mid, 1, st)
            conv(rows, f"{nm} 3x3 {mid}->{mid}", ho, wo, mid, mid, 3, 1)
            if b == 0:
                conv(rows, f"{nm} 1x1 proj {cin}->{out}" + ("/2" if st > 1 else ""), h, w, cin, out, 1, st)
            conv(rows, f"{nm} 1x1c {mid}->{out} +res", ho, wo, mid, out, 1, 1, res=True)
            io = 2 * (B * h * w * cin + B * ho * wo * out)
            blocks.append((nm, i0, len(rows), io))
            h, w, cin = ho, wo, out
        C[si + 2] = (h, w, cin)
    (h3, w3, c3), (h4, w4, c4), (h5, w5, c5) = C[3], C[4], C[5]
    conv(rows, "FPN lat5 1x1 2048->256", h5, w5, c5, 256, 1, 1)
    conv(rows, "FPN lat4 1x1 1024->256", h4, w4, c4, 256, 1, 1)
    conv(rows, "FPN lat3 1x1 512->256", h3, w3, c3, 256, 1, 1)
    rows.append(("FPN top-down upsample+add (fused)", 0.0, 2 * B * 256 * (h5 * w5 + 2 * h4 * w4 + 2 * h3 * w3)))
    conv(rows, "FPN P5 3x3 256->256", h5, w5, 256, 256, 3, 1)
    conv(rows, "FPN P4 3x3 256->256", h4, w4, 256, 256, 3, 1)
    conv(rows, "FPN P3 3x3 256->256", h3, w3, 256, 256, 3, 1)
    h6, w6 = conv(rows, "FPN P6 3x3/2 2048->256", h5, w5, c5, 256, 3, 2)
    conv(rows, "FPN P7 3x3/2 256->256", h6, w6, 256, 256, 3, 2)

    t_unf = 0.0
    print(f"{'conv':36s} {'GFLOP':>8s} {'MB':>8s} {'mfma us':>8s} {'hbm us':>8s} {'bound us':>9s}")
    for name, fl, by in rows:
        tm, th = fl / PEAK * 1e6, by / HBM * 1e6
        t_unf += max(tm, th)
        print(f"{name:36s} {fl / 1e9:8.2f} {by / 1e6:8.1f} {tm:8.1f} {th:8.1f} {max(tm, th):9.1f}")
    flop = sum(r[1] for r in rows)
    print(f"\nforward: {flop / 1e9:.1f} GFLOP ({flop / 1e9 / B:.3f} GFLOP/img); MFMA floor {flop / PEAK * 1e6:.1f} us")
    print(f"unfused attainable (sum of per-conv bounds): {t_unf:.1f} us -> mfma_frac at that time "
          f"{flop / PEAK * 1e6 / t_unf:.3f}")
    t_f = t_unf
    print("\nbottleneck blocks fused (block input + output only; weights once):")
    for nm, a, b, io in blocks:
        fl = sum(r[1] for r in rows[a:b])
        unf = sum(max(r[1] / PEAK, r[2] / HBM) for r in rows[a:b]) * 1e6
        fused = max(fl / PEAK, io / HBM) * 1e6
        t_f += fused - unf
        print(f"  {nm:6s} {fl / 1e9:6.2f} GFLOP {io / 1e6:7.1f} MB: unfused {unf:6.1f} us -> fused {fused:6.1f} us")
    print(f"fused attainable: {t_f:.1f} us -> mfma_frac {flop / PEAK * 1e6 / t_f:.3f}")


if __name__ == "__main__":
    main()
