"""Pipeline: model + optimizer construction, masked CE loss, the training step
and caption prediction (reference: utils/pipeline.py:8-154).

Same members as the reference Pipeline: transformer, learning_rate,
optimizer, train_loss (Keras Mean), ckpt / ckpt_manager / smart_ckpt_saver
(restoring the latest checkpoint at construction), loss, train_step, predict.

Differences that are deliberate and documented:
  - the tokenizer / COCO evaluator (pipeline.py:14-15, dataset.py) are out of
    the hot-path scope: pass target_vocab_size / start / end token ids, or a
    Keras tokenizer JSON with word_index;
  - train_step runs as a replayed hipGraph (fpnmt.train.TrainEngine);
  - predict reproduces the reference's beam procedure, which starts all beams
    identical and therefore equals greedy arg-max decoding with ties to the
    lowest token id (pipeline.py:101-144); it decodes BEAM_SEARCH_N identical
    rows like the reference, on the HIP decode path (fpnmt.decode).
"""
import json
import math

import torch

from common.common_definitions import (BEAM_SEARCH_N, CLIPNORM_MODE, DATADIR, DATATYPE_VAL, DROPOUT_RATE, END_TOKEN,
                                       IMAGE_INPUT_SIZE, START_TOKEN, WARM_UP_STEPS, d_model, dff, num_heads,
                                       num_layers, TOP_K)
import fpnmt
from fpnmt import ops
from fpnmt.checkpoint import Checkpoint, CheckpointManager
from fpnmt.train import TrainEngine
from models.transformer import Transformer, create_look_ahead_mask
from utils.utils import CustomSchedule, Mean, SmartCheckpointSaver


def clipnorm_for(mode=CLIPNORM_MODE, clipnorm=1.0):
    """utils/pipeline.py:30 Adam(..., clipnorm=1.): 'per_tensor' applies it
    as TF >= 2.4's apply_gradients does (clip_by_norm per gradient); 'none'
    reproduces TF 2.0-2.3 custom loops, which ignored clipnorm."""
    if mode == "per_tensor":
        return clipnorm
    if mode == "none":
        return 0.0
    raise ValueError(f"CLIPNORM_MODE must be 'per_tensor' or 'none', got {mode!r}")


def load_word_index(tokenizer_filename):
    """word_index of a Keras tokenizer JSON (dataset.py:125-135 format)."""
    with open(tokenizer_filename) as f:
        cfg = json.load(f)
    cfg = cfg.get("config", cfg)
    wi = cfg["word_index"]
    return json.loads(wi) if isinstance(wi, str) else wi


class Pipeline:
    def __init__(self, tokenizer_filename=None, checkpoint_path=None, max_seq_len=32, target_vocab_size=None,
                 image_size=IMAGE_INPUT_SIZE, n_layers=num_layers, backbone=None, rate=DROPOUT_RATE,
                 device="cuda", init=None, use_graph=True, clipnorm_mode=CLIPNORM_MODE, max_to_keep=100,
                 data_dir=DATADIR, data_type_val=DATATYPE_VAL):
        self.max_seq_len = max_seq_len
        self._metric_eval_src = (data_dir, data_type_val)
        self._metric_eval = None
        self.start_token, self.end_token = START_TOKEN, END_TOKEN
        self.tokenizer = None
        if tokenizer_filename is not None:
            from utils.text import load_tokenizer_from_path
            self.tokenizer = load_tokenizer_from_path(tokenizer_filename)  # pipeline.py:14-15
            wi = self.tokenizer.word_index
            self.start_token, self.end_token = wi["<start>"], wi["<end>"]
            if target_vocab_size is None:
                target_vocab_size = len(wi)
        self.target_vocab_size = target_vocab_size or TOP_K
        input_vocab_size = math.ceil(image_size / 16) ** 2  # pipeline.py:20
        self.transformer = Transformer(n_layers, d_model, num_heads, dff, input_vocab_size, self.target_vocab_size,
                                       rate, max_seq_len=self.max_seq_len, backbone=backbone, init=init).to(device)
        self.learning_rate = CustomSchedule(dff, WARM_UP_STEPS)  # pipeline.py:29 (d_model arg = dff)
        self.engine = TrainEngine(self.transformer, self.learning_rate, beta1=0.9, beta2=0.98, eps=1e-9,
                                  clipnorm=clipnorm_for(clipnorm_mode), use_graph=use_graph)
        self.optimizer = self.engine
        self.train_loss = Mean(name="train_loss")  # pipeline.py:35
        self.checkpoint_path = checkpoint_path
        # pipeline.py:38-48: checkpoint + manager, restore the latest if any
        self.ckpt = Checkpoint(transformer=self.transformer, optimizer=self.engine)
        self.ckpt_manager = None
        self.smart_ckpt_saver = None
        if checkpoint_path is not None:
            self.ckpt_manager = CheckpointManager(self.ckpt, checkpoint_path, max_to_keep=max_to_keep)
            self.smart_ckpt_saver = SmartCheckpointSaver(self.ckpt_manager)
            if self.ckpt_manager.latest_checkpoint:
                self.ckpt.restore(self.ckpt_manager.latest_checkpoint)
                print("Latest checkpoint restored!!")

    @property
    def metric_eval(self):
        """pipeline.py:15 MetricEval(DATADIR, DATATYPE_VAL): CIDEr of a results
        file against the ground-truth captions (train.py:76). Built on first
        use: the reference constructs it eagerly, which requires the COCO
        annotation file even for runs that never evaluate."""
        if self._metric_eval is None:
            from dataset import MetricEval
            self._metric_eval = MetricEval(*self._metric_eval_src)
        return self._metric_eval

    def loss(self, real, pred):
        """Masked sparse CE from logits, mean over ALL positions (pipeline.py:50-57)."""
        return ops.MaskedXentFn.apply(pred, real)

    def train_step(self, img, caption_token):
        """pipeline.py:64-80: one optimizer step, then train_loss(loss)
        (device-side running mean: no host synchronisation per step)."""
        loss = self.engine.step(img, caption_token)
        self.train_loss(loss)
        return loss

    # ------------------------------------------------------------ predict
    @torch.no_grad()
    def predict(self, img, max_seq_len, plot_layer=False):
        """Reference beam procedure (pipeline.py:82-154) for one image (h, w, 3):
        BEAM_SEARCH_N beams through the HIP decode path (fpnmt.decode.
        BeamDecoder: K/V cache, on-device softmax / top-k / beam bookkeeping,
        one hipGraph per step, no host round trip per token). Returns
        (token ids without <start> / <end> (int32, on the image's device),
        attention weights). The attention-weight dict of the reference's last
        decoder call (pipeline.py:109, kept for plot_attention_weights) is
        recomputed only when plot_layer is set: one transformer call on the
        identical beams' final prefix; None otherwise."""
        ids = self.predict_batch(img[None], max_seq_len, beam_n=BEAM_SEARCH_N)[0]
        out = torch.tensor(ids, dtype=torch.int32, device=img.device)
        attention_weights = None
        if plot_layer:
            tr = self.transformer
            enc = tr.encoder(img[None], False, None).repeat(BEAM_SEARCH_N, 1, 1)
            # the last call's input: <start> + every token but the final one
            ended = len(ids) < max_seq_len
            prefix = [self.start_token] + (ids if ended else ids[:-1])
            seq = torch.tensor([prefix] * BEAM_SEARCH_N, dtype=torch.int32, device=enc.device)
            _, attention_weights = tr(enc, seq, False, create_look_ahead_mask(seq.shape[1], device=enc.device))
        return out, attention_weights

    @torch.no_grad()
    def predict_batch(self, images, max_seq_len=None, beam_n=BEAM_SEARCH_N, use_graph=True):
        """predict() for a batch of images (n, h, w, 3) at once: the same
        beam procedure per image (pipeline.py:82-154), with a K/V cache and a
        hipGraph per decode step (fpnmt.decode.BeamDecoder). Returns one
        token-id list per image."""
        from fpnmt.decode import BeamDecoder
        T = max_seq_len or self.max_seq_len
        key = (images.shape[0], beam_n, T, use_graph)
        dec = getattr(self, "_decoders", {}).get(key)
        if dec is None:
            dec = BeamDecoder(self.transformer, images.shape[0], beam_n, T, self.start_token, self.end_token,
                              use_graph=use_graph)
            self.__dict__.setdefault("_decoders", {})[key] = dec
        return dec.decode(images)


    def evaluate(self, generator, max_seq_len):
        """pipeline.py:156-175: caption every (img, imgId) of the generator ->
        [{'image_id', 'caption'}] (the MetricEval results format)."""
        results = []
        for img, img_id in generator:
            result = self.predict(img, max_seq_len)[0]
            results.append({"image_id": img_id, "caption": self._to_text(result)})
        return results

    def evaluate_img(self, img, max_seq_len):
        """pipeline.py:177-193."""
        result = self.predict(img, max_seq_len)[0]
        return [{"image_id": 0, "caption": self._to_text(result)}]

    def _to_text(self, ids):
        if self.tokenizer is None:
            raise ValueError("Pipeline(tokenizer_filename=...) is needed to turn token ids into text")
        return self.tokenizer.sequences_to_texts([[int(t) for t in ids]])[0]
