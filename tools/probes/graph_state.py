"""After graph-replayed training steps, is the model's eager forward consistent
with its parameters? Compares an eager-trained and a graph-trained model
(same init / data), their parameters, fp32 logits, and the effect of
invalidating the compute copies."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import fpnmt  # noqa: E402
from fpnmt import layers as flayers  # noqa: E402
from fpnmt.layers import Init  # noqa: E402
from fpnmt.train import TrainEngine  # noqa: E402
from models.transformer import Transformer, create_masks  # noqa: E402
from utils.utils import CustomSchedule  # noqa: E402

layers = int(sys.argv[1]) if len(sys.argv) > 1 else 2
vocab = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
fpnmt.set_precision("bf16")
models, engs = [], []
for graph in (False, True):
    m = Transformer(layers, 512, 8, 2048, 196, vocab, 0.1, max_seq_len=32,
                    init=Init(torch.Generator().manual_seed(1234))).cuda()
    eng = TrainEngine(m, CustomSchedule(2048, 4000), use_graph=graph)
    img, tok = bench.synthetic_batch(8, 224, vocab, 32, 1000, "cuda")
    for i in range(3):
        eng.step(img, tok)
    torch.cuda.synchronize()
    models.append(m)
    engs.append(eng)
pe, pg = engs[0].arena.flat, engs[1].arena.flat
print("param |dE-G| max %.3e mean %.3e; step E %d G %d" % (float((pe - pg).abs().max()), float((pe - pg).abs().mean()),
                                                           int(engs[0].arena.step), int(engs[1].arena.step)))
for nme in ("m", "v", "vhat"):
    a, b = getattr(engs[0].arena, nme), getattr(engs[1].arena, nme)
    print(f"  {nme}: |E-G| max {float((a - b).abs().max()):.3e}, |E| max {float(a.abs().max()):.3e}")
# state dict vs arena
sd = models[1].state_dict()
k0 = next(iter(n for n, p in models[1].named_parameters()))
print("param is arena view:", models[1].get_parameter(k0).data_ptr() == engs[1].arena.flat.data_ptr())

fpnmt.set_precision("fp32")
img, tok = bench.synthetic_batch(1, 224, vocab, 32, 7, "cuda")
tar = tok[:, :-1]


def logits(m):
    with torch.no_grad():
        enc = m.encoder(img, False, None)
        lg, _ = m(enc, tar, False, create_masks(tar))
    torch.cuda.synchronize()
    return enc.float(), lg.float()


eE, lE = logits(models[0])
eG, lG = logits(models[1])
print("fp32 enc |E-G| %.3e (|enc| %.3e), logits |E-G| %.3e" % (float((eE - eG).abs().max()), float(eE.abs().max()),
                                                             float((lE - lG).abs().max())))
flayers.invalidate_weights()
eG2, lG2 = logits(models[1])
print("after invalidate: enc |E-G| %.3e, logits |E-G| %.3e" % (float((eE - eG2).abs().max()),
                                                              float((lE - lG2).abs().max())))
fpnmt.set_precision("bf16")
eGb, lGb = logits(models[1])
eEb, lEb = logits(models[0])
print("bf16 enc |E-G| %.3e logits |E-G| %.3e" % (float((eEb - eGb).abs().max()), float((lEb - lGb).abs().max())))
