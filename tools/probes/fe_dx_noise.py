"""Run-to-run spread of the grouped / per-level FE input gradients (is the
test_fe_levels_grouped_matches_per_level dx gap order noise?)."""
import sys
sys.path[:0] = ["tests", "fpn-mt-image-captioning_amd", "."]
import torch
import test_gpu_parts as T

fe, sd = T._setup()
g = torch.Generator().manual_seed(5)
sizes = (28, 14, 7, 3, 1, 0)
feats = [torch.randn(2, s, s, 256, generator=g) for s in sizes]
def run(mode):
    fe.zero_grad(set_to_none=True)
    fd = [f.to(T.DEV).requires_grad_(True) for f in feats]
    outs = fe.levels(fd) if mode == "grouped" else [fe.level(f) for f in fd]
    ws = [torch.randn(o.shape, generator=torch.Generator().manual_seed(i)) for i, o in enumerate(outs)]
    loss = sum((o * w.to(T.DEV)).sum() for o, w in zip(outs, ws) if o.numel())
    loss.backward()
    torch.cuda.synchronize()
    return [f.grad.detach().cpu().double() if f.grad is not None else None for f in fd]
res = {m: [run(m) for _ in range(3)] for m in ("grouped", "single")}
for lv, s in enumerate(sizes):
    if not s or res["single"][0][lv] is None:
        continue
    b = res["single"][0][lv]
    print("level", s, "max|dx| %.3e" % float(b.abs().max()),
          "grouped-vs-single %s" % ["%.2e" % float((res["grouped"][i][lv] - b).abs().max()) for i in range(3)],
          "single-vs-single %s" % ["%.2e" % float((res["single"][i][lv] - b).abs().max()) for i in range(1, 3)],
          "grouped-vs-grouped %s" % ["%.2e" % float((res["grouped"][i][lv] - res["grouped"][0][lv]).abs().max()) for i in range(1, 3)])
