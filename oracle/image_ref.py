"""ORACLE — test infrastructure only (same rules as oracle/ref_cpu.py: only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import it).

CPU restatement of the reference's image preprocessing (dataset.py:19-26):

    img = tf.image.resize(tf.image.decode_jpeg(file, channels=3), (S, S))
    img = tf.keras.applications.mobilenet_v2.preprocess_input(img)

- tf.image.resize (TF2 `resize_images_v2`, method BILINEAR, antialias False)
  runs ResizeBilinear with half_pixel_centers=True, align_corners=False:
  per output index i, in = (i + 0.5) * (in_size / out_size) - 0.5,
  lower = max(floor(in), 0), upper = min(ceil(in), in_size - 1),
  lerp = in - floor(in); top = tl + (tr - tl) * xl, bottom = bl + (br - bl) * xl,
  out = top + (bottom - top) * yl — every step an fp32 operation (TF's
  resize_bilinear_op.cc compute_interpolation_weights / compute_lerp).
- preprocess_input for MobileNetV2 is Keras imagenet_utils mode 'tf':
  x /= 127.5; x -= 1 (fp32).

numpy float32 array arithmetic rounds every operation separately (no FMA),
which is what the HIP kernel reproduces with contraction disabled.

PARITY STATUS: pinned by closed-form known answers of the TF formula
(identity size, 2x2 -> 1x1 mean, the half-pixel 2x upscale ramp
0, 63.75, 191.25, 255 — tests/test_input_pipeline.py); TensorFlow itself
is absent here, so other values are "parity unpinned" against TF.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def axis_weights(out_size: int, in_size: int):
    """(lower, upper, lerp) per output index, TF HalfPixelScaler order."""
    scale = F32(in_size) / F32(out_size)
    i = np.arange(out_size, dtype=F32)
    x = (i + F32(0.5)) * scale - F32(0.5)
    f = np.floor(x)
    lo = np.maximum(f.astype(np.int64), 0)
    hi = np.minimum(np.ceil(x).astype(np.int64), in_size - 1)
    return lo, hi, (x - f).astype(F32)


def resize_bilinear(img_u8: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """tf.image.resize(img, (out_h, out_w)) of an (h, w, c) image -> fp32."""
    h, w = img_u8.shape[:2]
    src = img_u8.astype(F32)
    ylo, yhi, yl = axis_weights(out_h, h)
    xlo, xhi, xl = axis_weights(out_w, w)
    xl = xl[None, :, None]
    yl = yl[:, None, None]
    tl = src[ylo][:, xlo]
    tr = src[ylo][:, xhi]
    bl = src[yhi][:, xlo]
    br = src[yhi][:, xhi]
    top = tl + (tr - tl) * xl
    bottom = bl + (br - bl) * xl
    return (top + (bottom - top) * yl).astype(F32)


def preprocess_input(x: np.ndarray) -> np.ndarray:
    """mobilenet_v2.preprocess_input (imagenet_utils mode 'tf')."""
    x = x.astype(F32) / F32(127.5)
    return (x - F32(1.0)).astype(F32)


def load_image_pixels(img_u8: np.ndarray, size: int) -> np.ndarray:
    """dataset.py:19-26 after the decode: resize to (size, size), preprocess."""
    return preprocess_input(resize_bilinear(img_u8, size, size))
