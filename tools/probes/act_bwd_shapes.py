"""Which act_bwd / bias_grad calls one eager C2 training step makes: wraps
fpnmt.ops.act_bwd / bias_grad and prints (rows, c, act, dropout) with a count."""
import collections
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fpn-mt-image-captioning_amd"), ROOT]
import torch  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import ops  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from fpnmt.train import TrainEngine  # noqa: E402
from models.transformer import Transformer  # noqa: E402
from utils.utils import CustomSchedule  # noqa: E402
import bench  # noqa: E402

fpnmt.set_precision("bf16")
seen = collections.Counter()
orig_act, orig_bias = ops.act_bwd, ops.bias_grad


def _caller():
    """The autograd Function backward (and its layer) that made this call."""
    fr = sys._getframe(2)
    while fr is not None:
        ctx = fr.f_locals.get("ctx")
        if ctx is not None:
            lay = getattr(ctx, "layer", None) or (getattr(ctx, "layers", None) or [None])[-1]
            return type(ctx).__name__ + ":" + str(getattr(lay, "name", None) or type(lay).__name__)
        fr = fr.f_back
    return "?"


def act_bwd(dt, rows, c, act, alpha, dy, y, dz, db, s, drop=None):
    seen[("act_bwd", rows, c, act, drop is not None, db is not None, _caller())] += 1
    return orig_act(dt, rows, c, act, alpha, dy, y, dz, db, s, drop=drop)


def bias_grad(dt, rows, c, dy, db, s):
    seen[("bias_grad", rows, c, db is not None)] += 1
    return orig_bias(dt, rows, c, dy, db, s)


ops.act_bwd, ops.bias_grad = act_bwd, bias_grad
model = Transformer(6, 512, 8, 2048, 196, 10000, 0.1, max_seq_len=32,
                    init=Init(torch.Generator().manual_seed(1))).cuda()
eng = TrainEngine(model, CustomSchedule(2048, 4000), use_graph=False)
img, tok = bench.synthetic_batch(32, 224, 10000, 32, 1000, "cuda")
eng.step(img, tok)
seen.clear()
eng.step(img, tok)
torch.cuda.synchronize()
for k, v in sorted(seen.items(), key=lambda kv: -kv[1]):
    print(v, k)
