"""Input pipeline: JPEG files -> the model's NHWC input batch on the GPU
(reference dataset.py:19-26 load_image and the tf.data map /
shuffle / batch / prefetch chain of dataset.py:89-92).

Split MI355X-first:
  - host: file read + JPEG decode (libjpeg through Pillow, which releases the
    GIL while decoding, so a thread pool decodes a batch in parallel; the
    reference's decode_jpeg is libjpeg too: ISLOW DCT, fancy upsampling),
    packed into ONE pinned staging buffer with an item table per batch;
  - device: one H2D copy of the packed bytes on a side stream, then ONE
    `fpnmt_image_resize_normalize` launch (bilinear resize with TF2
    half-pixel centres + mobilenet_v2.preprocess_input, bit-identical to TF's
    fp32 formula) writes the (B, S, S, 3) fp32 / bf16 input directly;
  - the next batch is decoded on the host while the current one trains
    (prefetch queue), the copy + resize of a batch is ordered before its
    consumer by a stream event (no host synchronisation).
No CPU fallback: without the HIP library this module does not import.
"""
from __future__ import annotations

import ctypes as C
import io
import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import _lib
from ._lib import call, dtype_code

PREPROCESS_DIV = 127.5  # mobilenet_v2.preprocess_input: x / 127.5 - 1 (dataset.py:24)
PREPROCESS_SUB = 1.0
ITEM_ALIGN = 16         # byte alignment of each image inside the packed buffer


class ImageItem(C.Structure):
    """fpnmt_image_item (include/fpnmt.h)."""
    _fields_ = [("offset", C.c_longlong), ("h", C.c_int), ("w", C.c_int)]


ITEM_DTYPE = np.dtype([("offset", "<i8"), ("h", "<i4"), ("w", "<i4")])


def decode_image(data: bytes) -> np.ndarray:
    """tf.image.decode_jpeg(data, channels=3) (dataset.py:22): (h, w, 3) uint8.
    Grayscale images are expanded to RGB by replication, as TF does."""
    from PIL import Image

    with Image.open(io.BytesIO(data)) as im:
        if im.mode != "RGB":
            im = im.convert("RGB")
        arr = np.asarray(im, dtype=np.uint8)
    if arr.ndim != 3 or arr.shape[2] != 3 or arr.shape[0] == 0 or arr.shape[1] == 0:
        raise ValueError(f"decoded image has shape {arr.shape}, expected (h, w, 3) with h, w > 0")
    return arr


def read_image(path) -> np.ndarray:
    """tf.io.read_file + decode_jpeg(channels=3) (dataset.py:21-22)."""
    with open(path, "rb") as f:
        return decode_image(f.read())


def pack_images(images, pin=False):
    """Pack (h, w, 3) uint8 arrays into one byte buffer + an item table.
    Returns (pixels uint8 tensor, items uint8 tensor holding n
    fpnmt_image_item records, max_w)."""
    n = len(images)
    offs = np.zeros(n, dtype=np.int64)
    total = 0
    max_w = 1
    for i, im in enumerate(images):
        if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != 3:
            raise ValueError(f"image {i}: expected (h, w, 3) uint8, got {im.dtype} {im.shape}")
        if im.shape[0] <= 0 or im.shape[1] <= 0:
            raise ValueError(f"image {i}: empty image {im.shape}")
        offs[i] = total
        total += -(-im.nbytes // ITEM_ALIGN) * ITEM_ALIGN
        max_w = max(max_w, im.shape[1])
    pixels = torch.empty(max(total, ITEM_ALIGN), dtype=torch.uint8, pin_memory=pin)
    flat = pixels.numpy()
    for i, im in enumerate(images):
        flat[offs[i]:offs[i] + im.nbytes] = np.ascontiguousarray(im).reshape(-1)
    items = torch.empty(max(n, 1) * C.sizeof(ImageItem), dtype=torch.uint8, pin_memory=pin)
    rec = items.numpy().view(ITEM_DTYPE)
    rec["offset"][:n] = offs
    for i, im in enumerate(images):
        rec["h"][i], rec["w"][i] = im.shape[0], im.shape[1]
    return pixels, items, max_w


def resize_normalize_packed(pixels_dev, items_dev, n, max_w, out_h, out_w, dtype=torch.float32, out=None,
                            div=PREPROCESS_DIV, sub=PREPROCESS_SUB):
    """One fpnmt_image_resize_normalize launch on the current stream over
    already-resident packed bytes -> (n, out_h, out_w, 3)."""
    dev = pixels_dev.device
    if out is None:
        out = torch.empty((n, out_h, out_w, 3), dtype=dtype, device=dev)
    if out.shape != (n, out_h, out_w, 3) or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous ({n}, {out_h}, {out_w}, 3) tensor, got {tuple(out.shape)}")
    call("fpnmt_image_resize_normalize", items_dev.data_ptr(), n, pixels_dev.data_ptr(), pixels_dev.numel(),
         max_w, out_h, out_w, float(div), float(sub), dtype_code(out.dtype), out.data_ptr(), _lib.stream_ptr())
    return out


def resize_normalize(images, size, dtype=torch.float32, device="cuda"):
    """dataset.py:23-24 for a list of decoded (h, w, 3) uint8 images:
    (n, size, size, 3) on the GPU. `size` is an int or (out_h, out_w)."""
    out_h, out_w = (size, size) if isinstance(size, int) else size
    pixels, items, max_w = pack_images(images, pin=torch.cuda.is_available())
    pd = pixels.to(device, non_blocking=True)
    idev = items.to(device, non_blocking=True)
    out = resize_normalize_packed(pd, idev, len(images), max_w, out_h, out_w, dtype)
    return out


def load_image(img_path, caption, size, dtype=torch.float32, device="cuda"):
    """dataset.py:19-26: (image (size, size, 3) on the GPU, caption)."""
    return resize_normalize([read_image(img_path)], size, dtype, device)[0], caption


class ImageBatchLoader:
    """Batches of (images (B, S, S, 3) on the GPU, captions (B, T) int32 on the
    GPU) from image paths + padded token rows — the tf.data chain of
    dataset.py:89-92 (map(load_image) / shuffle / batch / prefetch).

    shuffle: a seeded permutation per epoch (tf.data's BUFFER_SIZE window
    shuffle is a different random order, not a numeric difference);
    drop_remainder=False keeps the short last batch like Dataset.batch.
    Decoding runs on `threads` host threads, `prefetch` batches ahead."""

    def __init__(self, paths, captions, batch_size, image_size, dtype=torch.float32, shuffle=True, seed=0,
                 threads=8, prefetch=2, device="cuda", drop_remainder=False, decoder=read_image):
        if len(paths) != len(captions):
            raise ValueError(f"{len(paths)} paths but {len(captions)} captions")
        self.paths = list(paths)
        self.captions = np.asarray(captions, dtype=np.int32)
        self.batch_size = int(batch_size)
        self.size = (image_size, image_size) if isinstance(image_size, int) else tuple(image_size)
        self.dtype = dtype
        self.shuffle = shuffle
        self.seed = seed
        self.threads = threads
        self.prefetch = max(1, prefetch)
        self.device = torch.device(device)
        self.drop_remainder = drop_remainder
        self.decoder = decoder
        self.epoch = 0

    def __len__(self):
        n = len(self.paths)
        return n // self.batch_size if self.drop_remainder else -(-n // self.batch_size)

    def _order(self):
        idx = np.arange(len(self.paths))
        if self.shuffle:
            np.random.default_rng((self.seed, self.epoch)).shuffle(idx)
        return idx

    def _batches(self, order):
        bs = self.batch_size
        for s in range(0, len(order), bs):
            b = order[s:s + bs]
            if len(b) < bs and self.drop_remainder:
                return
            yield b

    def __iter__(self):
        order = self._order()
        self.epoch += 1
        q: queue.Queue = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()
        pin = self.device.type == "cuda"

        def produce():
            try:
                with ThreadPoolExecutor(self.threads) as pool:
                    for b in self._batches(order):
                        if stop.is_set():
                            return
                        imgs = list(pool.map(self.decoder, [self.paths[i] for i in b]))
                        pixels, items, max_w = pack_images(imgs, pin=pin)
                        q.put((b, pixels, items, max_w))
            except BaseException as e:  # surfaced to the consumer
                q.put(e)
                return
            q.put(None)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        side = torch.cuda.Stream(self.device) if pin else None
        try:
            while True:
                got = q.get()
                if got is None:
                    break
                if isinstance(got, BaseException):
                    raise got
                b, pixels, items, max_w = got
                with torch.cuda.stream(side):
                    pd = pixels.to(self.device, non_blocking=True)
                    idev = items.to(self.device, non_blocking=True)
                    caps = torch.from_numpy(self.captions[b]).to(self.device, non_blocking=True)
                    imgs = resize_normalize_packed(pd, idev, len(b), max_w, self.size[0], self.size[1], self.dtype)
                    ev = torch.cuda.Event()
                    ev.record(side)
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for t in (pd, idev, caps, imgs):
                    t.record_stream(cur)
                yield imgs, caps
        finally:
            stop.set()
            while th.is_alive():  # drain so the producer can exit
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)


def default_decode_threads():
    return max(1, min(16, os.cpu_count() or 1))
