"""Fused identity bottleneck (fpnmt_bottleneck_fwd) against the unfused three
launches, batch 64 bf16, hipGraph replay, per block shape; and the R50-FPN
headline forward with / without the fused blocks.
  python tools/probes/bottleneck_bench.py"""
import os
import sys

ROOT = os.getcwd()
sys.path[:0] = [os.path.join(ROOT, "fpn-mt-image-captioning_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402


def main():
    import fpnmt
    from bench import _graph_time, headline_probe
    from test_gpu_bottleneck import _block, _x
    fpnmt.set_precision("bf16")
    for h, c, cm in [(56, 256, 64), (28, 512, 128)]:
        blk = _block(c, cm, seed=5)
        x = _x(64, h, c, seed=6)
        res = {}
        for fused in (True, False):
            fpnmt.config.fuse_bottleneck = fused
            with torch.no_grad():
                res[fused] = _graph_time(lambda: blk(x), 20)
        fpnmt.config.fuse_bottleneck = True
        flop = 2 * 64 * h * h * (c * cm + 9 * cm * cm + cm * c)
        byt = 2 * 2 * 64 * h * h * c
        print(f"identity bottleneck {h}x{h}x{c}/{cm}, batch 64: fused {res[True] * 1e3:.1f} us "
              f"({flop / res[True] / 1e9:.0f} TFLOP/s, {byt / res[True] / 1e6:.0f} GB/s of x + y), "
              f"unfused {res[False] * 1e3:.1f} us", flush=True)
    for fused in (True, False):
        fpnmt.config.fuse_bottleneck = fused
        print(f"headline R50-FPN fwd (fuse_bottleneck={fused}):", headline_probe(), flush=True)
    fpnmt.config.fuse_bottleneck = True


if __name__ == "__main__":
    main()
