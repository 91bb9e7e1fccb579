"""Dataset handling with the reference's names and call contracts
(dataset.py:15-343): COCO caption files -> tokenized, padded captions and a
batched GPU image stream; tokenizer persistence; validation generators; the
CIDEr evaluator.

What is MI355X-native: images go through fpnmt.input_pipeline (host libjpeg
decode on a thread pool into one pinned buffer per batch, then ONE HIP
launch for the TF2 bilinear resize + mobilenet_v2.preprocess_input straight
into the NHWC model input). Text (Keras Tokenizer, pad_sequences), the COCO
annotation reader and the coco-caption scorers are host code restated in
utils/text.py, utils/coco.py and utils/coco_eval.py (pycocotools,
pycocoevalcap and TensorFlow are not installed here).

Differences from the reference, deliberate:
  - get_coco_images_dataset returns an fpnmt ImageBatchLoader (iterates
    (images (B, S, S, 3) on the GPU, captions (B, T) int32 on the GPU)) in
    place of the tf.data.Dataset; shuffling is a seeded per-epoch permutation
    rather than tf.data's BUFFER_SIZE window.
  - MetricEval computes Bleu_1..4, ROUGE_L and CIDEr (METEOR / SPICE need
    Java) and returns CIDEr as the reference does.
"""
from __future__ import annotations

import json
import math
import os
import re
from pathlib import Path
from random import shuffle

import torch

from common.common_definitions import (BATCH_SIZE, BUFFER_SIZE, IMAGE_INPUT_SIZE, TOKENIZER_FILENAME,  # noqa: F401
                                       TOP_K)
from utils.coco import COCO
from utils.coco_eval import COCOEvalCap
from utils.text import (Tokenizer, load_tokenizer_from_path, pad_sequences,  # noqa: F401
                        store_tokenizer_to_path, tokenizer_from_json)

TOKENIZER_FILTERS = '!"#$%&()*+-/:;=?@[\\]^_`{|}~ '  # dataset.py:63 (keeps . , < >)


def calc_max_length(tensor):
    """dataset.py:15-16."""
    return max(len(t) for t in tensor)


def load_image(img_path, caption, size=IMAGE_INPUT_SIZE, dtype=torch.float32, device="cuda"):
    """dataset.py:19-26: read + decode_jpeg(channels=3) + resize((S, S)) +
    mobilenet_v2.preprocess_input -> ((S, S, 3) fp32 on the GPU, caption)."""
    from fpnmt.input_pipeline import load_image as _load

    return _load(img_path, caption, size, dtype, device)


def _tokenizer_from_json(json_string):
    """dataset.py:96-123."""
    return tokenizer_from_json(json_string)


def _captions_of(anns):
    anns = [a for a in anns if a["caption"] != " "]  # dataset.py:50: drop empty captions
    return anns, ["<start> " + a["caption"] + " <end>" for a in anns]


def build_caption_tokens(captions, tokenizer_file=TOKENIZER_FILENAME, num_words=TOP_K):
    """dataset.py:54-83: load (or fit + store) the tokenizer, split '.' / ','
    off the words, texts_to_sequences, pad_sequences(padding='post').
    The tokenizer is fitted on the captions BEFORE the '.'/',' split, as in
    the reference (dataset.py:64 vs :73)."""
    tokenizer_file = Path(tokenizer_file) if tokenizer_file is not None else None
    if tokenizer_file is not None and tokenizer_file.is_file():
        tokenizer = load_tokenizer_from_path(tokenizer_file)
        print("Tokenizer is loaded from", tokenizer_file)
    else:
        tokenizer = Tokenizer(num_words=num_words, oov_token="unk", filters=TOKENIZER_FILTERS)
        tokenizer.fit_on_texts(captions)
        tokenizer.word_index[""] = 0
        tokenizer.index_word[0] = ""
        if tokenizer_file is not None:
            tokenizer_file.parent.mkdir(parents=True, exist_ok=True)
            store_tokenizer_to_path(tokenizer, tokenizer_file)
    captions = [re.sub(r"([.,])", r" \1 ", c) for c in captions]
    tokens = tokenizer.texts_to_sequences(captions)
    max_seq_len = max(map(len, tokens))
    return tokenizer, pad_sequences(tokens, padding="post"), max_seq_len


def get_coco_images_dataset(dataDir, dataType, n_test=None, tokenizer_file=TOKENIZER_FILENAME,
                            batch_size=BATCH_SIZE, image_size=IMAGE_INPUT_SIZE, dtype=torch.float32, seed=0,
                            threads=8, device="cuda"):
    """dataset.py:29-94 -> (loader, max_seq_len, set_len)."""
    from fpnmt.input_pipeline import ImageBatchLoader

    coco = COCO("{}/annotations/captions_{}.json".format(dataDir, dataType))
    ann_ids = coco.getAnnIds()[:n_test] if n_test is not None else coco.getAnnIds()
    anns, captions = _captions_of(coco.loadAnns(ann_ids))
    img_ids = [a["image_id"] for a in anns]
    _, captions_token, max_seq_len = build_caption_tokens(captions, tokenizer_file)
    set_len = math.ceil(len(captions_token) / batch_size)
    imgs = coco.loadImgs(img_ids)
    img_paths = [os.path.join(dataDir, "images", dataType, img["file_name"]) for img in imgs]
    loader = ImageBatchLoader(img_paths, captions_token, batch_size, image_size, dtype=dtype, shuffle=True,
                              seed=seed, threads=threads, device=device)
    return loader, max_seq_len, set_len


def get_coco_images_captions_generator(dataDir, dataType, tokenizer_file=TOKENIZER_FILENAME,
                                       image_size=IMAGE_INPUT_SIZE):
    """dataset.py:149-190: yields (image on the GPU, tokenized reference captions)."""
    coco = COCO("{}/annotations/captions_{}.json".format(dataDir, dataType))
    tokenizer_file = Path(tokenizer_file)
    if not tokenizer_file.is_file():
        raise Exception("tokenizer is not yet created in", tokenizer_file)
    tokenizer = load_tokenizer_from_path(tokenizer_file)
    print("Tokenizer is loaded from", tokenizer_file)
    for img_id in coco.getImgIds():
        anns, captions = _captions_of(coco.loadAnns(coco.getAnnIds(imgIds=img_id)))
        captions_token = tokenizer.texts_to_sequences(captions)
        img = coco.loadImgs(img_id)[0]
        image, _ = load_image(os.path.join(dataDir, "images", dataType, img["file_name"]), None, image_size)
        yield image, captions_token


class COCO_Images_ImageID:
    """dataset.py:192-245: iterates (image on the GPU, imgId) over a shuffled
    list of the annotated image ids (one entry per non-empty caption, as the
    reference builds it), the first n_val of them."""

    def __init__(self, dataDir, dataType, n_val=None, image_size=IMAGE_INPUT_SIZE):
        self.dataDir, self.dataType, self.image_size = dataDir, dataType, image_size
        self.coco = COCO("{}/annotations/captions_{}.json".format(dataDir, dataType))
        anns = [a for a in self.coco.loadAnns(self.coco.getAnnIds()) if a["caption"] != " "]
        self.imgIds = [a["image_id"] for a in anns]
        shuffle(self.imgIds)
        self.max_len = len(self.imgIds) if n_val is None else n_val
        self.imgIds = self.imgIds if n_val is None else self.imgIds[:n_val]
        self.iterIndex = 0

    def __iter__(self):
        self.iterIndex = 0
        return self

    def __next__(self):
        if self.iterIndex >= self.max_len:
            raise StopIteration
        img_id = self.imgIds[self.iterIndex]
        img = self.coco.loadImgs(img_id)[0]
        image, _ = load_image(os.path.join(self.dataDir, "images", self.dataType, img["file_name"]), None,
                              self.image_size)
        self.iterIndex += 1
        return image, img_id


def store_additional_info(dict, filename):
    """dataset.py:248-250."""
    with open(filename, "w") as outfile:
        json.dump(dict, outfile)


def load_additional_info(filename):
    """dataset.py:252-258: {} when the file is missing or unreadable."""
    try:
        with open(filename) as infile:
            return json.load(infile)
    except (OSError, ValueError):
        return {}


class MetricEval:
    """dataset.py:260-325: CIDEr of a results file against the ground truth."""

    def __init__(self, dataDir, dataType):
        self.dataDir, self.dataType = dataDir, dataType
        self.coco = COCO("{}/annotations/captions_{}.json".format(dataDir, dataType))
        self.last_eval = {}

    def __call__(self, resFile):
        coco_res = self.coco.loadRes(resFile)
        ev = COCOEvalCap(self.coco, coco_res)
        ev.params["image_id"] = coco_res.getImgIds()  # dataset.py:291
        ev.evaluate()
        self.last_eval = dict(ev.eval)
        return ev.eval["CIDEr"]

    def print_result(self, imgId, resFile):
        """dataset.py:300-325 without the matplotlib display."""
        coco_res = self.coco.loadRes(resFile)
        print("ground truth captions")
        self.coco.showAnns(self.coco.loadAnns(self.coco.getAnnIds(imgIds=imgId)))
        print("\n")
        print("generated caption")
        self.coco.showAnns(coco_res.loadAnns(coco_res.getAnnIds(imgIds=imgId)))
