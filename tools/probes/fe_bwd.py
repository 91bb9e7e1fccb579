"""Diagnostic: fp32-mode accuracy of the feature extractor's BACKWARD alone.
The upstream gradient at the five level outputs is the fp64 oracle's for the
full model (LAYERS, VOCAB); it is fed into the GPU fp32 FE, the oracle fp32
FE and the oracle fp64 FE, and intermediate / parameter gradients of the FPN
P4 path are compared against fp64.
  python tools/probes/fe_bwd.py LAYERS VOCAB"""
import math
import os
import sys

sys.path[:0] = [os.path.join(os.getcwd(), "fpn-mt-image-captioning_amd"), os.getcwd(), os.path.join(os.getcwd(), "tests")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import ref_cpu as R  # noqa: E402

WATCH = ["P3", "P4", "P5", "reg3", "reg4", "reg5", "cls4", "coatt4", "p4m"]
PARAMS = ["retinanet_model.fpn.P4.kernel", "retinanet_model.fpn.C4_reduced.kernel", "retinanet_model.fpn.P3.kernel",
          "retinanet_model.fpn.P4.bias", "retinanet_model.fpn.C4_reduced.bias", "retinanet_model.fpn.P3.bias",
          "retinanet_model.fpn.P5.kernel", "regression.kernel", "classification.kernel", "post_conv.kernel",
          "out_conv.kernel", "retinanet_model.submodels.0.convs.0.kernel"]


def oracle_fe(sd, img, keep):
    p = "encoder.feature_extractor"
    rp = p + ".retinanet_model"
    C2, C3, C4, C5 = R.resnet(sd, rp + ".backbone", img)
    c = lambda n, x: R.conv_same(x, sd[f"{rp}.fpn.{n}.kernel"], sd[f"{rp}.fpn.{n}.bias"])  # noqa: E731
    P5f = c("C5_reduced", C5)
    P5 = F.relu(c("P5", P5f))
    p4m = R.upsample_like(P5f, C4) + c("C4_reduced", C4)
    keep["p4m"] = p4m
    P4 = F.relu(c("P4", p4m))
    P3 = F.relu(c("P3", c("C3_reduced", C3) + R.upsample_like(p4m, C3)))
    P6 = R.maxpool_valid(F.relu(c("P6_conv", P5f)))
    P7 = R.maxpool_valid(F.relu(c("P7_conv", P6)))
    outs = []
    for i, f in enumerate([P3, P4, P5, P6, P7]):
        keep[f"P{i + 3}"] = f
        r, cl = f, f
        for j in range(2):
            r = F.relu(R.conv_same(r, sd[f"{rp}.submodels.0.convs.{j}.kernel"], sd[f"{rp}.submodels.0.convs.{j}.bias"]))
            cl = F.relu(R.conv_same(cl, sd[f"{rp}.submodels.1.convs.{j}.kernel"], sd[f"{rp}.submodels.1.convs.{j}.bias"]))
        reg = R.conv_same(r, sd[p + ".regression.kernel"], sd[p + ".regression.bias"])
        cls = R.conv_same(cl, sd[p + ".classification.kernel"], sd[p + ".classification.bias"])
        keep[f"reg{i + 3}"], keep[f"cls{i + 3}"] = reg, cls
        o = R.coattention(reg, cls)
        keep[f"coatt{i + 3}"] = o
        o = R.leaky(R.conv_same(o, sd[p + ".post_conv.kernel"], sd[p + ".post_conv.bias"]))
        o = R.maxpool_valid(o)
        outs.append(R.leaky(R.conv_same(o, sd[p + ".out_conv.kernel"], sd[p + ".out_conv.bias"])))
    for t in keep.values():
        if t.requires_grad:
            t.retain_grad()
    return outs


def gpu_fe(m, img, keep):
    import fpnmt
    from fpnmt import ops
    fe = m.encoder.feature_extractor
    rm = fe.retinanet_model
    fe.set_training(True)
    fpnmt.config.fuse_conv_chains = False
    C2, C3, C4, C5 = rm.backbone(img.cuda())
    fpn = rm.fpn
    p5f = fpn.C5_reduced(C5)
    P5 = fpn.P5(p5f)
    lat4, lat3 = fpn.C4_reduced(C4), fpn.C3_reduced(C3)
    p4m, p3m = ops.FpnTopDownFn.apply(p5f, lat4, lat3)
    keep["p4m"] = p4m
    P4, P3 = fpn.P4(p4m), fpn.P3(p3m)
    P6 = ops.max_pool2d_valid(fpn.P6_conv(p5f))
    P7 = ops.max_pool2d_valid(fpn.P7_conv(P6))
    outs = []
    for i, f in enumerate([P3, P4, P5, P6, P7]):
        keep[f"P{i + 3}"] = f
        reg = fe.regression(rm.submodels[0](f))
        cls = fe.classification(rm.submodels[1](f))
        keep[f"reg{i + 3}"], keep[f"cls{i + 3}"] = reg, cls
        o = fe.coattention(reg, cls)
        keep[f"coatt{i + 3}"] = o
        outs.append(fe.out_conv(ops.max_pool2d_valid(fe.post_conv(o))))
    for t in keep.values():
        if t.requires_grad:
            t.retain_grad()
    return outs


def main():
    layers, vocab = int(sys.argv[1]), int(sys.argv[2])
    image = 224
    import fpnmt
    from fpnmt.layers import Init
    from models.transformer import Transformer
    import test_gpu_model as T
    fpnmt.set_precision("fp32")
    m = Transformer(layers, 512, 8, 2048, math.ceil(image / 16) ** 2, vocab, 0.0, max_seq_len=32,
                    init=Init(torch.Generator().manual_seed(1234)))
    sd = {k: v.detach().float().clone() for k, v in m.state_dict().items()}
    m = m.cuda()
    img, tok = T._inputs(b=2, vocab=vocab, image=image)
    cfg = dict(num_layers=layers, num_heads=8, backbone="resnet50")
    # fp64 upstream gradient at the FE outputs
    sd64 = {k: v.double() for k, v in sd.items()}
    fo = R.feature_extractor(sd64, "encoder.feature_extractor", img.double(), "resnet50", True)
    lv = [f.detach().clone().requires_grad_(True) for f in fo]
    from probe_grad_boundary import oracle_tail
    loss, _ = oracle_tail(sd64, lv, tok, cfg)
    loss.backward()
    up = [x.grad.detach() for x in lv]
    print("upstream |dFE| max per level:", [f"{float(u.abs().max()):.3e}" if u.numel() else "-" for u in up])
    res = {}
    for name, dt in (("fp64", torch.float64), ("cpu32", torch.float32)):
        s = {k: v.to(dt).requires_grad_(k.startswith("encoder.feature_extractor.")) for k, v in sd.items()}
        keep = {}
        outs = oracle_fe(s, img.to(dt), keep)
        torch.autograd.backward([o for o in outs if o.numel()], [u.to(dt) for u, o in zip(up, outs) if o.numel()])
        res[name] = ({k: v.grad.double() for k, v in keep.items() if v.grad is not None},
                     {n: s["encoder.feature_extractor." + n].grad.double() for n in PARAMS})
    keep = {}
    outs = gpu_fe(m, img, keep)
    torch.autograd.backward([o for o in outs if o.numel()], [u.float().cuda() for u, o in zip(up, outs) if o.numel()])
    fe = m.encoder.feature_extractor
    pn = dict(fe.named_parameters())
    res["gpu"] = ({k: v.grad.double().cpu() for k, v in keep.items() if v.grad is not None},
                  {n: pn[n].grad.double().cpu() for n in PARAMS})
    for part, label in ((0, "activation grads"), (1, "param grads")):
        print(f"--- {label}")
        for k, r in res["fp64"][part].items():
            mx = float(r.abs().max())
            if mx == 0:
                continue
            eg = float((res["gpu"][part][k] - r).abs().max()) / mx
            ec = float((res["cpu32"][part][k] - r).abs().max()) / mx
            print(f"{k:48s} |ref| {mx:.3e}  gpu {eg:.2e}  cpu32 {ec:.2e}  ratio {eg / max(ec, 1e-30):.1f}")


if __name__ == "__main__":
    main()
