"""Co-attention for the encoder before the multi-view transformer.

Reference: models/coattention.py:9-32 (CoAttention_CNN). The spatial softmax
and the broadcast multiply run as one HIP kernel (fpnmt_spatial_softmax_fwd)
and its backward (fpnmt_spatial_softmax_bwd).
"""
from torch import nn

from fpnmt import ops


class CoAttention_CNN(nn.Module):
    def __init__(self):
        super().__init__()

    def forward(self, score, hs):
        """score (B, h, w, 1) attention logits; hs (B, h, w, C) -> (B, h, w, C).

        a = softmax(score reshaped to (B, h*w), axis=1) (coattention.py:24-27),
        context = a * hs broadcast over C (coattention.py:30)."""
        if score.shape[-1] != 1 or score.shape[:3] != hs.shape[:3]:
            raise ValueError(f"CoAttention_CNN: score {tuple(score.shape)} vs hs {tuple(hs.shape)}")
        return ops.SpatialSoftmaxFn.apply(score, hs)

    call = forward
