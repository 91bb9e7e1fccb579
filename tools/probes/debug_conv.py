"""Isolate a conv backward mismatch: act_bwd and bwd-data separately vs fp64
CPU, over batch sizes, for one conv shape. Usage: python debug_conv.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fpn-mt-image-captioning_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import fpnmt  # noqa: E402
from fpnmt import _lib as L  # noqa: E402
from fpnmt import ops  # noqa: E402
from fpnmt.layers import Conv2D  # noqa: E402

DEV = "cuda"
for dt in (torch.float32, torch.bfloat16):
    for (n, h, c, k) in [(1, 56, 64, 64), (4, 56, 64, 64), (8, 56, 64, 64), (16, 56, 64, 64), (16, 28, 64, 64),
                         (16, 56, 64, 32), (16, 28, 128, 256)]:
        torch.manual_seed(0)
        layer = Conv2D(c, k, 3, padding="same", activation="relu", kernel_initializer="glorot_uniform").to(DEV)
        x = torch.randn(n, h, h, c, device=DEV).to(dt)
        xi = x.clone().requires_grad_(True)
        y = layer(xi)
        gy = torch.randn(y.shape, device=DEV).to(dt)
        # act_bwd alone
        dz = torch.empty_like(gy)
        db = torch.zeros(k, device=DEV)
        ops.act_bwd(L.dtype_code(dt), y.numel() // k, k, L.ACT_RELU, 0.0, gy, y, dz, db.data_ptr(), L.stream_ptr())
        dz_ref = gy.double() * (y.double() > 0)
        e_dz = float((dz.double() - dz_ref).abs().max())
        e_db = float((db.double() - dz_ref.sum((0, 1, 2))).abs().max())
        # bwd-data alone on dz_ref
        d = layer.desc(n, h, h, c, dt)
        _, wflip = layer.compute_weights(dt)
        dx = torch.empty_like(x)
        dzin = dz_ref.to(dt).contiguous()
        L.call("fpnmt_conv2d_bwd_data", d, dzin.data_ptr(), wflip.data_ptr(), dx.data_ptr(), 0, L.stream_ptr())
        torch.cuda.synchronize()
        kern = layer.kernel.detach().to(dt).double().cpu().permute(3, 2, 0, 1)  # HWIO -> OIHW
        dx_ref = torch.nn.grad.conv2d_input((n, c, h, h), kern, dzin.double().cpu().permute(0, 3, 1, 2), padding=1)
        dx_ref = dx_ref.permute(0, 2, 3, 1)
        err = (dx.double().cpu() - dx_ref).abs()
        bad = (err > 1e-3 * max(1.0, float(dx_ref.abs().max()))).nonzero()
        desc = ""
        if len(bad):
            rows = bad[:, 0] * h * h + bad[:, 1] * h + bad[:, 2]
            desc = (f" nbad={len(bad)} rows[{int(rows.min())}..{int(rows.max())}] ch[{int(bad[:, 3].min())}.."
                    f"{int(bad[:, 3].max())}] first={bad[0].tolist()}")
        print(f"{str(dt)[6:]:9s} n={n:2d} h={h} c={c} k={k}: act_bwd dz {e_dz:.2e} db {e_db:.2e} | "
              f"bwd_data max {float(err.max()):.3e} (|ref| {float(dx_ref.abs().max()):.2f}){desc}", flush=True)
