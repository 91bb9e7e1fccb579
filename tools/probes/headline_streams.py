"""Probe: the R50-FPN headline forward (batch 64, bf16) as one chain against
S concurrent chains over batch slices (forked streams captured into ONE
hipGraph, so the branches can overlap each other's latency-bound launches).
  python tools/probes/headline_streams.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.getcwd(), "fpn-mt-image-captioning_amd"), os.getcwd()]
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from models.retinanet import FeatureExtractor  # noqa: E402


def graph_time(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return min(ts)


def main():
    fpnmt.set_precision("bf16")
    fe = FeatureExtractor(backbone="resnet50", init=Init(torch.Generator().manual_seed(3))).cuda()
    B = 64
    x = (torch.rand(B, 224, 224, 3, device="cuda") * 2 - 1).to(torch.bfloat16)
    pyr = fe.retinanet_model.pyramid
    with torch.no_grad():
        ref = [t.clone() for t in pyr(x)]
        base = graph_time(lambda: pyr(x))
        print(f"one chain, batch {B}: {base:.3f} ms  ({9.354 * B / base:.1f} TFLOP/s)")
        for S in (2, 4):
            streams = [torch.cuda.Stream() for _ in range(S)]
            outs = [None] * S
            sl = B // S

            def fn():
                cur = torch.cuda.current_stream()
                for i, st in enumerate(streams):
                    st.wait_stream(cur)
                    with torch.cuda.stream(st):
                        outs[i] = pyr(x[i * sl:(i + 1) * sl])
                for st in streams:
                    cur.wait_stream(st)

            ms = graph_time(fn)
            ok = all(torch.equal(torch.cat([o[j] for o in outs]), ref[j]) for j in range(len(ref)))
            print(f"{S} concurrent chains of batch {sl}: {ms:.3f} ms  ({9.354 * B / ms:.1f} TFLOP/s), "
                  f"outputs == one chain: {ok}")
            sq = graph_time(lambda: [pyr(x[i * sl:(i + 1) * sl]) for i in range(S)])
            print(f"{S} sequential chains of batch {sl}: {sq:.3f} ms")


if __name__ == "__main__":
    main()
