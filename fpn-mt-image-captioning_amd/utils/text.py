"""Caption text <-> token ids: the Keras text utilities the reference's data
side uses (dataset.py:61-83,96-146; utils/pipeline.py:14-15,165,185),
restated because TensorFlow / Keras are not part of this build:

  Tokenizer(num_words, filters, lower, split, char_level, oov_token):
    fit_on_texts, texts_to_sequences, sequences_to_texts, to_json, and
    tokenizer_from_json (keras_preprocessing.text, the TF 2.x Keras version)
  pad_sequences(..., padding='post')   (keras_preprocessing.sequence)

The JSON written by `store_tokenizer_to_path` / read by
`load_tokenizer_from_path` is the reference's format (the Tokenizer's
to_json() string, itself json.dumps'ed into the file), so a tokenizer file
the reference wrote loads here and vice versa.
"""
from __future__ import annotations

import json
from collections import OrderedDict, defaultdict

import numpy as np

DEFAULT_FILTERS = '!"#$%&()*+,-./:;<=>?@[\\]^_`{|}~\t\n'


def text_to_word_sequence(text, filters=DEFAULT_FILTERS, lower=True, split=" "):
    """keras_preprocessing.text.text_to_word_sequence."""
    if lower:
        text = text.lower()
    text = text.translate(str.maketrans({c: split for c in filters}))
    return [w for w in text.split(split) if w]


class Tokenizer:
    """keras_preprocessing.text.Tokenizer (word level)."""

    def __init__(self, num_words=None, filters=DEFAULT_FILTERS, lower=True, split=" ", char_level=False,
                 oov_token=None, document_count=0, **kwargs):
        if kwargs:
            raise TypeError(f"unrecognized keyword arguments: {sorted(kwargs)}")
        self.word_counts = OrderedDict()
        self.word_docs = defaultdict(int)
        self.filters = filters
        self.split = split
        self.lower = lower
        self.num_words = num_words
        self.document_count = document_count
        self.char_level = char_level
        self.oov_token = oov_token
        self.index_docs = defaultdict(int)
        self.word_index = {}
        self.index_word = {}

    def _seq(self, text):
        if self.char_level or isinstance(text, list):
            if self.lower:
                text = [t.lower() for t in text] if isinstance(text, list) else text.lower()
            return text
        return text_to_word_sequence(text, self.filters, self.lower, self.split)

    def fit_on_texts(self, texts):
        for text in texts:
            self.document_count += 1
            seq = self._seq(text)
            for w in seq:
                self.word_counts[w] = self.word_counts.get(w, 0) + 1
            for w in set(seq):
                self.word_docs[w] += 1
        wcounts = list(self.word_counts.items())
        wcounts.sort(key=lambda x: x[1], reverse=True)  # stable: ties keep first-seen order
        sorted_voc = [] if self.oov_token is None else [self.oov_token]
        sorted_voc.extend(wc[0] for wc in wcounts)
        self.word_index = dict(zip(sorted_voc, range(1, len(sorted_voc) + 1)))
        self.index_word = {c: w for w, c in self.word_index.items()}
        for w, c in list(self.word_docs.items()):
            self.index_docs[self.word_index[w]] = c

    def texts_to_sequences(self, texts):
        return list(self.texts_to_sequences_generator(texts))

    def texts_to_sequences_generator(self, texts):
        num_words = self.num_words
        oov_index = self.word_index.get(self.oov_token)
        for text in texts:
            vect = []
            for w in self._seq(text):
                i = self.word_index.get(w)
                if i is not None:
                    if num_words and i >= num_words:
                        if oov_index is not None:
                            vect.append(oov_index)
                    else:
                        vect.append(i)
                elif self.oov_token is not None:
                    vect.append(oov_index)
            yield vect

    def sequences_to_texts(self, sequences):
        num_words = self.num_words
        oov_index = self.word_index.get(self.oov_token)
        out = []
        for seq in sequences:
            vect = []
            for num in seq:
                num = int(num)
                word = self.index_word.get(num)
                if word is not None:
                    if num_words and num >= num_words:
                        if oov_index is not None:
                            vect.append(self.index_word[oov_index])
                    else:
                        vect.append(word)
                elif self.oov_token is not None:
                    vect.append(self.index_word[oov_index])
            out.append(" ".join(vect))
        return out

    def get_config(self):
        return {
            "num_words": self.num_words, "filters": self.filters, "lower": self.lower, "split": self.split,
            "char_level": self.char_level, "oov_token": self.oov_token, "document_count": self.document_count,
            "word_counts": json.dumps(self.word_counts), "word_docs": json.dumps(self.word_docs),
            "index_docs": json.dumps(self.index_docs), "index_word": json.dumps(self.index_word),
            "word_index": json.dumps(self.word_index),
        }

    def to_json(self, **kwargs):
        return json.dumps({"class_name": self.__class__.__name__, "config": self.get_config()}, **kwargs)


def tokenizer_from_json(json_string):
    """dataset.py:96-123 (_tokenizer_from_json) / keras tokenizer_from_json."""
    cfg = json.loads(json_string).get("config")
    cfg = dict(cfg)
    word_counts = json.loads(cfg.pop("word_counts"))
    word_docs = json.loads(cfg.pop("word_docs"))
    index_docs = {int(k): v for k, v in json.loads(cfg.pop("index_docs")).items()}
    index_word = {int(k): v for k, v in json.loads(cfg.pop("index_word")).items()}
    word_index = json.loads(cfg.pop("word_index"))
    tok = Tokenizer(**cfg)
    tok.word_counts = OrderedDict(word_counts)
    tok.word_docs = defaultdict(int, word_docs)
    tok.index_docs = defaultdict(int, index_docs)
    tok.word_index = word_index
    tok.index_word = index_word
    return tok


def load_tokenizer_from_path(path):
    """dataset.py:125-135: the file holds json.dumps(tokenizer.to_json())."""
    with open(path) as f:
        data = json.load(f)
    return tokenizer_from_json(data if isinstance(data, str) else json.dumps(data))


def store_tokenizer_to_path(tokenizer, path):
    """dataset.py:137-146."""
    with open(path, "w", encoding="utf-8") as f:
        f.write(json.dumps(tokenizer.to_json(), ensure_ascii=False))


def pad_sequences(sequences, maxlen=None, dtype="int32", padding="pre", truncating="pre", value=0.0):
    """keras_preprocessing.sequence.pad_sequences."""
    lengths = [len(s) for s in sequences]
    if maxlen is None:
        maxlen = max(lengths) if lengths else 0
    x = np.full((len(sequences), maxlen), value, dtype=dtype)
    for i, s in enumerate(sequences):
        if not len(s):
            continue
        trunc = s[-maxlen:] if truncating == "pre" else s[:maxlen]
        if truncating not in ("pre", "post"):
            raise ValueError(f'Truncating type "{truncating}" not understood')
        trunc = np.asarray(trunc, dtype=dtype)
        if padding == "post":
            x[i, :len(trunc)] = trunc
        elif padding == "pre":
            x[i, maxlen - len(trunc):] = trunc
        else:
            raise ValueError(f'Padding type "{padding}" not understood')
    return x
