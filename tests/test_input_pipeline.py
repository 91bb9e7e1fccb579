"""Input pipeline (reference dataset.py:19-94): the CPU
restatement of tf.image.resize + mobilenet_v2.preprocess_input pinned by
closed-form answers of TF's formula, the Keras text utilities, and (GPU) the
fpnmt_image_resize_normalize kernel bit-exact against the restatement on
ragged batches, through the C-ABI and through the batch loader over JPEG
files (decoded once on the host, compared on the same decoded pixels)."""
import io
import json
import os

import numpy as np
import pytest
import torch

from oracle import image_ref as R


# ------------------------------------------------------------ oracle KATs
def test_resize_identity_is_exact():
    img = np.random.default_rng(0).integers(0, 256, (7, 9, 3), dtype=np.uint8)
    out = R.resize_bilinear(img, 7, 9)
    assert out.dtype == np.float32 and np.array_equal(out, img.astype(np.float32))


def test_resize_2x2_to_1x1_is_the_mean():
    # in = (0 + .5) * 2 - .5 = .5 on both axes: lower 0, upper 1, lerp .5
    img = np.array([[[0, 10, 200], [4, 30, 100]], [[8, 50, 0], [12, 70, 255]]], dtype=np.uint8)
    out = R.resize_bilinear(img, 1, 1)
    assert np.array_equal(out[0, 0], np.array([6.0, 40.0, 138.75], dtype=np.float32))


def test_resize_half_pixel_upscale_ramp():
    # TF2 half-pixel 1x2 -> 1x4: in = -.25 (clamped), .25, .75, 1.25 (upper clamped)
    img = np.array([[[0, 0, 0], [255, 255, 255]]], dtype=np.uint8)
    out = R.resize_bilinear(img, 1, 4)[0, :, 0]
    assert out.tolist() == [0.0, 63.75, 191.25, 255.0]


def test_preprocess_tf_mode():
    x = np.array([0, 255, 127.5, 51], dtype=np.float32)
    y = R.preprocess_input(x)
    assert y[0] == -1.0 and y[1] == 1.0 and y[2] == 0.0
    assert y[3] == np.float32(np.float32(51) / np.float32(127.5)) - np.float32(1)


# ------------------------------------------------------------ host packing
def test_pack_images_layout():
    from fpnmt import input_pipeline as IP
    imgs = [np.full((2, 3, 3), 7, np.uint8), np.arange(5 * 1 * 3, dtype=np.uint8).reshape(5, 1, 3)]
    pixels, items, max_w = IP.pack_images(imgs)
    rec = items.numpy().view(IP.ITEM_DTYPE)
    assert max_w == 3
    assert rec["offset"].tolist() == [0, 32] and rec["h"].tolist() == [2, 5] and rec["w"].tolist() == [3, 1]
    flat = pixels.numpy()
    assert (flat[:18] == 7).all() and flat[32:47].tolist() == list(range(15))
    import ctypes
    assert ctypes.sizeof(IP.ImageItem) == IP.ITEM_DTYPE.itemsize == 16
    with pytest.raises(ValueError):
        IP.pack_images([np.zeros((0, 4, 3), np.uint8)])
    with pytest.raises(ValueError):
        IP.pack_images([np.zeros((4, 4), np.uint8)])


def test_decode_grayscale_expands_to_rgb():
    from PIL import Image
    from fpnmt import input_pipeline as IP
    g = (np.arange(12, dtype=np.uint8) * 20).reshape(3, 4)
    buf = io.BytesIO()
    Image.fromarray(g, mode="L").save(buf, format="PNG")
    rgb = IP.decode_image(buf.getvalue())
    assert rgb.shape == (3, 4, 3) and (rgb == g[..., None]).all()


# ------------------------------------------------------------ Keras text utils
def test_tokenizer_fit_and_sequences():
    from utils.text import Tokenizer, pad_sequences
    caps = ["<start> A dog. <end>", "<start> a cat, a dog <end>"]
    tok = Tokenizer(num_words=6, oov_token="unk", filters='!"#$%&()*+-/:;=?@[\\]^_`{|}~ ')
    tok.fit_on_texts(caps)
    # counts: <start> 2, a 3, dog. 1, <end> 2, cat, 1, dog 1 -> sorted desc, ties in first-seen order
    assert tok.word_index == {"unk": 1, "a": 2, "<start>": 3, "<end>": 4, "dog.": 5, "cat,": 6, "dog": 7}
    seqs = tok.texts_to_sequences(["<start> a dog . <end>", "a zebra cat"])
    # 'dog' = 7 >= num_words -> oov; '.' unseen -> oov; 'zebra' unseen -> oov
    assert seqs == [[3, 2, 1, 1, 4], [2, 1, 1]]
    assert tok.sequences_to_texts([[3, 2, 5]]) == ["<start> a dog."]
    x = pad_sequences([[1, 2, 3], [4]], padding="post")
    assert x.dtype == np.int32 and x.tolist() == [[1, 2, 3], [4, 0, 0]]
    assert pad_sequences([[1, 2, 3], [4]]).tolist() == [[1, 2, 3], [0, 0, 4]]
    assert pad_sequences([[1, 2, 3]], maxlen=2, truncating="post").tolist() == [[1, 2]]


def test_tokenizer_json_roundtrip_reference_format(tmp_path):
    from utils.text import Tokenizer, load_tokenizer_from_path, store_tokenizer_to_path
    tok = Tokenizer(num_words=100, oov_token="unk")
    tok.fit_on_texts(["the cat sat", "the dog sat down"])
    tok.word_index[""] = 0
    tok.index_word[0] = ""
    p = tmp_path / "tok.json"
    store_tokenizer_to_path(tok, p)
    raw = json.load(open(p))
    assert isinstance(raw, str)  # dataset.py:144-146: json.dumps of the to_json() string
    assert json.loads(raw)["class_name"] == "Tokenizer"
    t2 = load_tokenizer_from_path(p)
    assert t2.word_index == tok.word_index and t2.index_word == tok.index_word
    assert t2.texts_to_sequences(["the dog"]) == tok.texts_to_sequences(["the dog"])
    assert t2.num_words == 100 and t2.oov_token == "unk"


def _write_coco(root, images, captions):
    """A tiny COCO-format caption set: images [(id, file, array)], captions [(image_id, text)]."""
    from PIL import Image
    os.makedirs(root / "annotations", exist_ok=True)
    os.makedirs(root / "images" / "val", exist_ok=True)
    for _, fn, arr in images:
        Image.fromarray(arr).save(root / "images" / "val" / fn, quality=90)
    ds = {"images": [{"id": i, "file_name": fn} for i, fn, _ in images],
          "annotations": [{"id": k + 1, "image_id": i, "caption": c} for k, (i, c) in enumerate(captions)]}
    with open(root / "annotations" / "captions_val.json", "w") as f:
        json.dump(ds, f)


def test_build_caption_tokens_matches_reference_recipe(tmp_path):
    import dataset
    caps = ["<start> A man riding a horse. <end>", "<start> Two dogs, playing. <end>"]
    tok, padded, max_len = dataset.build_caption_tokens(caps, tokenizer_file=tmp_path / "t.json")
    assert (tmp_path / "t.json").is_file()
    assert tok.word_index[""] == 0 and tok.index_word[0] == ""
    # '.' and ',' are split off after fitting (dataset.py:73): the vocabulary
    # holds 'horse.', so both 'horse' and '.' map to 'unk' (1)
    assert padded.shape == (2, max_len) and max_len == 8
    row0 = tok.sequences_to_texts([padded[0]])[0].split()
    assert row0 == ["<start>", "a", "man", "riding", "a", "unk", "unk", "<end>"]
    # a second call loads the stored tokenizer and reproduces the ids
    tok2, padded2, _ = dataset.build_caption_tokens(caps, tokenizer_file=tmp_path / "t.json")
    assert np.array_equal(padded, padded2)


# ------------------------------------------------------------ GPU parity
def _rng_images(shapes, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]


RAGGED = [(480, 640), (1, 1), (224, 224), (100, 37), (50, 60), (333, 500), (640, 427)]
WIDE = [(3, 12000), (7, 5)]  # 2 x 36000 B rows exceed the 64 KB LDS window: global-memory path


@pytest.mark.gpu
@pytest.mark.parametrize("shapes", [RAGGED, WIDE], ids=["lds", "global"])
@pytest.mark.parametrize("out_hw", [(224, 224), (512, 512), (64, 96)])
def test_resize_normalize_kernel_bit_exact(out_hw, shapes):
    from fpnmt import input_pipeline as IP
    imgs = _rng_images(shapes)
    out = IP.resize_normalize(imgs, out_hw, dtype=torch.float32).cpu().numpy()
    for i, im in enumerate(imgs):
        ref = R.preprocess_input(R.resize_bilinear(im, *out_hw))
        assert np.array_equal(out[i], ref), (i, im.shape, np.abs(out[i] - ref).max())


@pytest.mark.gpu
def test_resize_normalize_bf16_is_rounded_fp32():
    from fpnmt import input_pipeline as IP
    imgs = _rng_images(RAGGED[:4], seed=1)
    out = IP.resize_normalize(imgs, 224, dtype=torch.bfloat16).cpu()
    for i, im in enumerate(imgs):
        ref = torch.from_numpy(R.preprocess_input(R.resize_bilinear(im, 224, 224))).to(torch.bfloat16)
        assert torch.equal(out[i], ref)


@pytest.mark.gpu
def test_resize_normalize_errors_and_empty_batch():
    from fpnmt import _lib as L
    from fpnmt import input_pipeline as IP
    pd = torch.zeros(64, dtype=torch.uint8, device="cuda")
    it = torch.zeros(16, dtype=torch.uint8, device="cuda")
    out = torch.empty((0, 4, 4, 3), device="cuda")
    assert IP.resize_normalize_packed(pd, it, 0, 1, 4, 4, out=out).shape == (0, 4, 4, 3)
    with pytest.raises(RuntimeError, match="bad sizes"):
        L.call("fpnmt_image_resize_normalize", it.data_ptr(), 1, pd.data_ptr(), 64, 1, 0, 4, 127.5, 1.0, 0,
               out.data_ptr(), L.stream_ptr())
    with pytest.raises(RuntimeError, match="div"):
        L.call("fpnmt_image_resize_normalize", it.data_ptr(), 1, pd.data_ptr(), 64, 1, 4, 4, 0.0, 1.0, 0,
               out.data_ptr(), L.stream_ptr())


@pytest.mark.gpu
def test_batch_loader_over_jpeg_files(tmp_path):
    """JPEG files -> ImageBatchLoader -> GPU batches equal the restatement on
    the same decoded pixels; captions follow the images; the short last batch
    is kept; a second epoch reshuffles."""
    from fpnmt import input_pipeline as IP
    shapes = [(120, 160), (64, 64), (200, 90), (31, 47), (128, 256)]
    imgs = _rng_images(shapes, seed=2)
    from PIL import Image
    paths = []
    for i, im in enumerate(imgs):
        p = tmp_path / f"{i}.jpg"
        Image.fromarray(im).save(p, quality=85)
        paths.append(str(p))
    caps = np.arange(len(paths) * 4, dtype=np.int32).reshape(len(paths), 4)
    loader = IP.ImageBatchLoader(paths, caps, batch_size=2, image_size=96, shuffle=True, seed=3, threads=3)
    assert len(loader) == 3
    seen = []
    for images, c in loader:
        assert images.shape[1:] == (96, 96, 3) and images.dtype == torch.float32
        torch.cuda.synchronize()
        for j in range(images.shape[0]):
            k = int(c[j, 0].item()) // 4
            ref = R.preprocess_input(R.resize_bilinear(IP.read_image(paths[k]), 96, 96))
            assert np.array_equal(images[j].cpu().numpy(), ref)
            seen.append(k)
    assert sorted(seen) == list(range(len(paths)))
    order2 = [int(c[j, 0]) // 4 for _, c in loader for j in range(c.shape[0])]
    assert sorted(order2) == sorted(seen)


@pytest.mark.gpu
def test_get_coco_images_dataset_end_to_end(tmp_path):
    import dataset
    imgs = _rng_images([(60, 80), (80, 60), (33, 33)], seed=4)
    _write_coco(tmp_path, [(10, "a.jpg", imgs[0]), (11, "b.jpg", imgs[1]), (12, "c.jpg", imgs[2])],
                [(10, "A dog on grass."), (11, "Two cats, sleeping."), (12, " "), (12, "A red car")])
    loader, max_len, set_len = dataset.get_coco_images_dataset(str(tmp_path), "val", tokenizer_file=tmp_path / "t.json",
                                                               batch_size=2, image_size=64, threads=2)
    assert set_len == 2 and max_len == 7  # the ' ' caption is filtered (dataset.py:50)
    n = 0
    for images, caps in loader:
        assert images.shape[1:] == (64, 64, 3) and caps.dtype == torch.int32 and caps.shape[1] == max_len
        assert float(images.min()) >= -1.0 and float(images.max()) <= 1.0
        n += images.shape[0]
    assert n == 3
    img, cap = dataset.load_image(str(tmp_path / "images" / "val" / "a.jpg"), "x", size=64)
    assert img.shape == (64, 64, 3) and cap == "x"
