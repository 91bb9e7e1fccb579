"""UpsampleLike (reference: layers/_misc.py:20-42).

tf.image.resize(source, target HW, NEAREST) in TF2 uses half-pixel centres:
src = min(floor((dst + 0.5) * in / out), in - 1). The kernel is the FPN
top-down sweep with a zero lateral input (fpnmt_fpn_topdown_fwd/bwd).
"""
from torch import nn

from fpnmt import ops

__all__ = ["UpsampleLike", "resize_images"]


def resize_images(images, size, method="nearest", align_corners=False):
    """Only 'nearest' is on the hot path (the reference's UpsampleLike)."""
    if method != "nearest":
        raise NotImplementedError("resize_images: only method='nearest' is implemented")
    return ops.UpsampleFn.apply(images, int(size[0]), int(size[1]))


class UpsampleLike(nn.Module):
    """Resize ``source`` (B,h,w,C) to the spatial size of ``target``."""

    def __init__(self, name=None):
        super().__init__()
        self.lname = name

    def forward(self, inputs):
        source, target = inputs
        return resize_images(source, (target.shape[1], target.shape[2]), method="nearest")

    def compute_output_shape(self, input_shape):
        return (input_shape[0][0],) + tuple(input_shape[1][1:3]) + (input_shape[0][-1],)
