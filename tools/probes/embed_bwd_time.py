"""Times fpnmt_embed_posenc_bwd at the C2 decoder shape (32 x 31 positions,
d 512, V 10000) for token mixes with and without padding."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fpn-mt-image-captioning_amd"), ROOT]
import torch
from fpnmt import _lib as L

dev = "cuda"
b, t, d, V = 32, 31, 512, 10000
for pad_from in (31, 20, 8):
    tok = torch.randint(4, V, (b, t), dtype=torch.int32)
    tok[:, pad_from:] = 0
    tok = tok.to(dev)
    dy = torch.randn(b, t, d, device=dev).to(torch.bfloat16)
    demb = torch.zeros(V, d, device=dev)
    ss = torch.zeros(1, device=dev)
    for _ in range(3):
        L.call("fpnmt_embed_posenc_bwd", L.BF16, b, t, d, tok.data_ptr(), dy.data_ptr(), demb.data_ptr(), ss.data_ptr(), L.stream_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        L.call("fpnmt_embed_posenc_bwd", L.BF16, b, t, d, tok.data_ptr(), dy.data_ptr(), demb.data_ptr(), ss.data_ptr(), L.stream_ptr())
    e1.record()
    torch.cuda.synchronize()
    print(f"pad from {pad_from}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
