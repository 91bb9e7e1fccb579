"""Multi-view transformer over the FPN levels + caption decoder
(reference: models/transformer.py:22-374), same names and call signatures.

Tensors are torch tensors on the GPU; attention runs on the fpnmt attention
kernels (QK^T and PV on MFMA, masked row softmax with the reference's
additive -1e9 mask), Dense / LayerNorm / Embedding / Dropout on fpnmt kernels.
"""
import math

import numpy as np
import torch
from torch import nn

from common.common_definitions import (ACTIVATION, BASELINE_INDEX, KERNEL_INITIALIZER, LEAKY_ALPHA, NUM_OF_PYRAMIDS,
                                       RETINANET_WEIGHT_PATH, BACKBONE, d_model as D_MODEL)
import fpnmt
from fpnmt import ops
from fpnmt.layers import Dense, DenseGroup, Embedding, LayerNormalization
from . import retinanet


# ------------------------------------------------------------------ posenc
def get_angles(pos, i, d_model):
    """transformer.py:22-24 (float64 numpy, as the reference)."""
    angle_rates = 1 / np.power(10000, (2 * (i // 2)) / np.float32(d_model))
    return pos * angle_rates


def raw_positional_encoding(position, d_model):
    """transformer.py:27-39: sin on even columns, cos on odd, cast to fp32."""
    angle_rads = get_angles(np.arange(position)[:, np.newaxis], np.arange(d_model)[np.newaxis, :], d_model)
    angle_rads[:, 0::2] = np.sin(angle_rads[:, 0::2])
    angle_rads[:, 1::2] = np.cos(angle_rads[:, 1::2])
    return torch.from_numpy(angle_rads.astype(np.float32))


def positional_encoding(position, d_model):
    return raw_positional_encoding(position, d_model)[None, ...]


# ------------------------------------------------------------------- masks
def create_padding_mask(seq):
    """(B, T) int -> (B, 1, 1, T) float, 1 where token == 0 (transformer.py:46-51)."""
    return (seq == 0).to(torch.float32)[:, None, None, :]


def create_look_ahead_mask(size, device=None):
    """1 - lower-triangular ones (transformer.py:54-56)."""
    return 1.0 - torch.tril(torch.ones((size, size), device=device))


def create_masks(tar):
    """max(padding mask, look-ahead mask) -> (B, 1, T, T) (transformer.py:59-67)."""
    look_ahead_mask = create_look_ahead_mask(tar.shape[1], device=tar.device)
    dec_target_padding_mask = create_padding_mask(tar)
    return torch.maximum(dec_target_padding_mask, look_ahead_mask)


# --------------------------------------------------------------- attention
def scaled_dot_product_attention(q, k, v, mask):
    """transformer.py:70-104 on (..., L, depth) tensors. Returns (output,
    attention_weights); weights are always materialised, as in the reference."""
    lead = q.shape[:-2]
    Lq, dk = q.shape[-2], q.shape[-1]
    Lk = k.shape[-2]
    bsz = int(np.prod(lead)) if len(lead) else 1
    q3 = q.reshape(bsz, Lq, dk)
    k3 = k.reshape(bsz, Lk, dk)
    v3 = v.reshape(bsz, Lk, v.shape[-1])
    m = None
    if mask is not None:
        m = torch.broadcast_to(mask.to(torch.float32), (*lead, Lq, Lk)).reshape(bsz, 1, Lq, Lk)
    out, w = ops.AttentionFn.apply(q3, k3, v3, m, 1, 1.0 / math.sqrt(dk))
    return out.reshape(*lead, Lq, v.shape[-1]), w.reshape(*lead, Lq, Lk)


class MultiHeadAttention(nn.Module):
    """transformer.py:107-155; call order (v, k, q, mask). Heads are column
    slices of the (B, L, d_model) projections — the split/merge transposes of
    the reference are address arithmetic inside the attention kernels."""

    def __init__(self, d_model, num_heads, init=None):
        super().__init__()
        self.num_heads = num_heads
        self.d_model = d_model
        assert d_model % self.num_heads == 0
        self.depth = d_model // self.num_heads
        self.wq = Dense(d_model, d_model, kernel_initializer=KERNEL_INITIALIZER, init=init)
        self.wk = Dense(d_model, d_model, kernel_initializer=KERNEL_INITIALIZER, init=init)
        self.wv = Dense(d_model, d_model, kernel_initializer=KERNEL_INITIALIZER, init=init)
        self.dense = Dense(d_model, d_model, kernel_initializer=KERNEL_INITIALIZER, init=init)

    def split_heads(self, x, batch_size):
        return x.reshape(batch_size, -1, self.num_heads, self.depth).permute(0, 2, 1, 3)

    def forward(self, v, k, q, mask, dropout=0.0, residual=None):
        return self.attend(self.wq(q), self.wk(k), self.wv(v), mask, dropout, residual)

    def attend(self, q, k, v, mask, dropout=0.0, residual=None):
        """Attention + output Dense on already-projected q, k, v (the fused
        projection path hands in column slices of one grouped GEMM).
        dropout / residual: the caller's `residual + Dropout(mha)` folded into
        the output Dense's GEMM epilogue."""
        scaled_attention, attention_weights = ops.AttentionFn.apply(
            q, k, v, mask, self.num_heads, 1.0 / math.sqrt(float(self.depth)))
        output = self.dense(scaled_attention, dropout=dropout, residual=residual)
        return output, attention_weights

    call = forward


class EncoderLayer(nn.Module):
    """Multi-view encoder layer (transformer.py:158-200): the baseline view
    attends to each of the other NUM_OF_PYRAMIDS-1 views with its own MHA;
    out = baseline + sum_i dropout(mha_i) (non-aliasing), LN1, FFN (leaky 0.2),
    dropout, LN2(out1 + ffn)."""

    def __init__(self, d_model, num_heads, dff, rate=0.1, init=None):
        super().__init__()
        self.mhas = nn.ModuleList([MultiHeadAttention(d_model, num_heads, init=init)
                                   for _ in range(NUM_OF_PYRAMIDS - 1)])
        self.ffn1 = Dense(d_model, dff, activation=ACTIVATION, act_alpha=LEAKY_ALPHA,
                          kernel_initializer=KERNEL_INITIALIZER, init=init)
        self.ffn2 = Dense(dff, d_model, kernel_initializer=KERNEL_INITIALIZER, init=init)
        # ffn1 only feeds ffn2: its LeakyReLU backward runs in ffn2's bwd-data epilogue
        self.ffn1.act_into_next = True
        self.layernorm1 = LayerNormalization(d_model, epsilon=1e-6)
        self.layernorm2 = LayerNormalization(d_model, epsilon=1e-6)
        self.rate = rate
        # the baseline feeds every view's query projection: one grouped GEMM
        self.q_group = DenseGroup([m.wq for m in self.mhas])
        # the views' output Dense layers: one launch for all of them
        # (ops.MultiViewAttnProjFn), kernels / biases contiguous in the arena
        self.o_group = DenseGroup([m.dense for m in self.mhas])

    def forward(self, x, training, mask, kv=None):
        """kv: per view (k, v) projections precomputed by the Encoder's grouped
        K/V GEMM (the views do not change across layers), or None."""
        baseline = x[NUM_OF_PYRAMIDS - 1]
        out = baseline
        fused = kv is not None and fpnmt.config.fuse_projections
        drop = self.rate if training else 0.0
        if fused:
            # every view's attention + output Dense + dropout + the residual
            # sum: one autograd node, one output launch
            qs = self.q_group(baseline)
            qkv = [t for i in range(NUM_OF_PYRAMIDS - 1) for t in (qs[i], kv[i][0], kv[i][1])]
            m0 = self.mhas[0]
            out = ops.MultiViewAttnProjFn.apply(baseline, self.o_group, drop, m0.num_heads,
                                                1.0 / math.sqrt(float(m0.depth)), mask, *qkv)
        else:
            for i in range(NUM_OF_PYRAMIDS - 1):
                # out = out + dropout(mha_i): one GEMM epilogue
                out, _ = self.mhas[i](x[i], x[i], baseline, mask, dropout=drop, residual=out)
        out1 = self.layernorm1(out)
        ffn_output = self.ffn2(self.ffn1(out1), dropout=drop)
        return self.layernorm2(ffn_output, residual=out1)

    call = forward


class DecoderLayer(nn.Module):
    """transformer.py:203-243."""

    def __init__(self, d_model, num_heads, dff, rate=0.1, init=None):
        super().__init__()
        self.mha1 = MultiHeadAttention(d_model, num_heads, init=init)
        self.mha2 = MultiHeadAttention(d_model, num_heads, init=init)
        self.ffn1 = Dense(d_model, dff, activation=ACTIVATION, act_alpha=LEAKY_ALPHA,
                          kernel_initializer=KERNEL_INITIALIZER, init=init)
        self.ffn2 = Dense(dff, d_model, kernel_initializer=KERNEL_INITIALIZER, init=init)
        # ffn1 only feeds ffn2: its LeakyReLU backward runs in ffn2's bwd-data epilogue
        self.ffn1.act_into_next = True
        self.layernorm1 = LayerNormalization(d_model, epsilon=1e-6)
        self.layernorm2 = LayerNormalization(d_model, epsilon=1e-6)
        self.layernorm3 = LayerNormalization(d_model, epsilon=1e-6)
        self.rate = rate
        self.qkv_group = DenseGroup([self.mha1.wq, self.mha1.wk, self.mha1.wv])

    def forward(self, x, enc_output, training, look_ahead_mask, padding_mask, kv2=None):
        """kv2: this layer's cross-attention (k, v) from the Decoder's grouped
        K/V GEMM over enc_output, or None."""
        fused = fpnmt.config.fuse_projections
        drop = self.rate if training else 0.0
        if fused:
            q, k, v = self.qkv_group(x)
            attn1, attn_weights_block1 = self.mha1.attend(q, k, v, look_ahead_mask, dropout=drop)
        else:
            attn1, attn_weights_block1 = self.mha1(x, x, x, look_ahead_mask, dropout=drop)
        out1 = self.layernorm1(attn1, residual=x)
        if fused and kv2 is not None:
            attn2, attn_weights_block2 = self.mha2.attend(self.mha2.wq(out1), kv2[0], kv2[1], padding_mask,
                                                          dropout=drop)
        else:
            attn2, attn_weights_block2 = self.mha2(enc_output, enc_output, out1, padding_mask, dropout=drop)
        out2 = self.layernorm2(attn2, residual=out1)
        ffn_output = self.ffn2(self.ffn1(out2), dropout=drop)
        out3 = self.layernorm3(ffn_output, residual=out2)
        return out3, attn_weights_block1, attn_weights_block2

    call = forward


class Encoder(nn.Module):
    """transformer.py:246-303: FeatureExtractor -> views reordered
    [P3, P4, P5, P7, P6] (baseline last) -> per view flatten, shared LN,
    + posenc[:L], dropout -> N layers updating only the baseline."""

    def __init__(self, num_layers, d_model, num_heads, dff, input_vocab_size, rate=0.1, backbone=None, init=None):
        super().__init__()
        self.d_model = d_model
        self.num_layers = num_layers
        self.x_order = [i for i in range(NUM_OF_PYRAMIDS) if i != BASELINE_INDEX] + [BASELINE_INDEX]
        self.register_buffer("pos_encoding", positional_encoding(input_vocab_size, self.d_model)[0].contiguous())
        self.enc_layers = nn.ModuleList([EncoderLayer(d_model, num_heads, dff, rate, init=init)
                                         for _ in range(num_layers)])
        self.feature_extractor = retinanet.FeatureExtractor(RETINANET_WEIGHT_PATH, backbone=backbone or BACKBONE,
                                                            init=init)
        self.layernorm1 = LayerNormalization(d_model, epsilon=1e-6)
        self.rate = rate
        # every layer's K/V projections of view i read the same x[i]: one GEMM per view
        self.kv_groups = [DenseGroup([w for l in self.enc_layers for w in (l.mhas[i].wk, l.mhas[i].wv)])
                          for i in range(NUM_OF_PYRAMIDS - 1)] if num_layers > 0 else []

    def forward(self, x, training, mask):
        return self.from_features(self.feature_extractor(x, training=training), training, mask)

    def from_features(self, x, training, mask):
        """The encoder after its FeatureExtractor (transformer.py:279-303) on
        the five level outputs — the data-parallel engine runs the transformer
        backward first and all-reduces its gradients while the feature
        extractor's backward runs."""
        # single-graph training step: the transformer's optimizer part starts
        # here in the backward, beside the feature extractor's backward
        x = ops.transformer_grads_barrier(list(x))
        x = [x[i] for i in self.x_order]
        for i_x in range(NUM_OF_PYRAMIDS):
            b, h, w, c = x[i_x].shape
            if h * w > self.pos_encoding.shape[0]:
                raise ValueError(f"view of length {h * w} exceeds the positional table "
                                 f"({self.pos_encoding.shape[0]}); raise input_vocab_size")
            x[i_x] = x[i_x].reshape(b, h * w, c)
        if fpnmt.config.fuse_view_norms:
            # every view's LN, += pe[:seq_len], dropout: one launch per pass
            x = list(ops.LayerNormViewsFn.apply(self.layernorm1, self.pos_encoding,
                                                self.rate if training else 0.0, *x))
        else:
            for i_x in range(NUM_OF_PYRAMIDS):
                _x = self.layernorm1(x[i_x], pe=self.pos_encoding)  # LN, then += pe[:seq_len]
                x[i_x] = ops.dropout(_x, self.rate, training)
        kvs = [g(x[i]) for i, g in enumerate(self.kv_groups)] if fpnmt.config.fuse_projections else None
        for i in range(self.num_layers):
            kv = [(kvs[j][2 * i], kvs[j][2 * i + 1]) for j in range(NUM_OF_PYRAMIDS - 1)] if kvs else None
            x[NUM_OF_PYRAMIDS - 1] = self.enc_layers[i](x, training, mask, kv=kv)
        return x[NUM_OF_PYRAMIDS - 1]

    call = forward


class Decoder(nn.Module):
    """transformer.py:306-341: Embedding (no sqrt(d) scale) + posenc, dropout,
    N layers; attention dict keyed decoder_layer{i}_block{1,2}."""

    def __init__(self, num_layers, d_model, num_heads, dff, target_vocab_size, rate=0.1, max_position=0,
                 max_seq_len=12, init=None):
        super().__init__()
        self.d_model = d_model
        self.num_layers = num_layers
        self.embedding = Embedding(target_vocab_size, d_model, init=init)
        self.register_buffer("pos_encoding", raw_positional_encoding(max_seq_len + max_position, d_model).contiguous())
        self.dec_layers = nn.ModuleList([DecoderLayer(d_model, num_heads, dff, rate, init=init)
                                         for _ in range(num_layers)])
        self.rate = rate
        # enc_output feeds every layer's cross-attention K/V: one GEMM
        self.cross_kv_group = DenseGroup([w for l in self.dec_layers for w in (l.mha2.wk, l.mha2.wv)]) \
            if num_layers > 0 else None

    def forward(self, x, enc_output, training, look_ahead_mask, padding_mask):
        seq_len = x.shape[1]
        if seq_len > self.pos_encoding.shape[0]:
            raise ValueError(f"target length {seq_len} exceeds max_seq_len {self.pos_encoding.shape[0]}")
        attention_weights = {}
        if fpnmt.config.fuse_view_norms:  # the embedding's Dropout in its launch
            x = self.embedding(x, self.pos_encoding, enc_output.dtype, dropout=self.rate if training else 0.0)
        else:
            x = self.embedding(x, self.pos_encoding, enc_output.dtype)
            x = ops.dropout(x, self.rate, training)
        kv = self.cross_kv_group(enc_output) if (fpnmt.config.fuse_projections and self.cross_kv_group) else None
        for i in range(self.num_layers):
            kv2 = (kv[2 * i], kv[2 * i + 1]) if kv is not None else None
            x, block1, block2 = self.dec_layers[i](x, enc_output, training, look_ahead_mask, padding_mask, kv2=kv2)
            attention_weights["decoder_layer{}_block1".format(i + 1)] = block1
            attention_weights["decoder_layer{}_block2".format(i + 1)] = block2
        return x, attention_weights

    call = forward


class Transformer(nn.Module):
    """transformer.py:344-374. training=True runs the encoder on the image;
    otherwise ``inp`` IS the encoder output (the reference's inference split)."""

    def __init__(self, num_layers, d_model, num_heads, dff, input_vocab_size, target_vocab_size, rate=0.1,
                 max_position=0, max_seq_len=12, backbone=None, init=None):
        super().__init__()
        self.encoder = Encoder(num_layers, d_model, num_heads, dff, input_vocab_size, rate, backbone=backbone,
                               init=init)
        self.decoder = Decoder(num_layers, d_model, num_heads, dff, target_vocab_size, rate, max_position,
                               max_seq_len, init=init)
        self.final_layer = Dense(d_model, target_vocab_size, out_f32=True, init=init)

    def forward(self, inp, tar, training, look_ahead_mask):
        if training:
            enc_output = self.encoder(inp, training, None)
        else:
            enc_output = inp
        dec_output, attention_weights = self.decoder(tar, enc_output, training, look_ahead_mask, None)
        final_output = self.final_layer(dec_output)
        return final_output, attention_weights

    call = forward

    @property
    def trainable_variables(self):
        return [p for p in self.parameters() if p.requires_grad]

    def save_weights(self, filepath):
        """tf.keras.Model.save_weights (train.py:96): every parameter and buffer
        (fp32 masters in the Keras layouts, BN statistics) keyed by its
        state_dict name, as one safetensors file (Keras writes h5 / TF
        checkpoints; h5py and TensorFlow are not installed here)."""
        from safetensors.torch import save_file
        import os
        # floating-point tensors as fp32 (the masters' dtype), integer buffers
        # in their own dtype (an int64 above 2^24 would not survive fp32)
        sd = {k: (v.detach().float() if v.is_floating_point() else v.detach()).contiguous().cpu()
              for k, v in self.state_dict().items()}
        d = os.path.dirname(os.path.abspath(filepath))
        os.makedirs(d, exist_ok=True)
        save_file(sd, filepath, metadata={"format": "fpnmt-weights-v1"})

    def load_weights(self, filepath):
        """Inverse of save_weights: copies every saved tensor into the model's
        parameters / buffers in place (the compute copies are refreshed at the
        next prepare)."""
        from safetensors.torch import load_file
        from fpnmt import layers as flayers
        sd = load_file(filepath)
        own = self.state_dict()
        missing = [k for k in own if k not in sd]
        if missing:
            raise ValueError(f"load_weights: {filepath} lacks {missing[:4]}")
        unexpected = [k for k in sd if k not in own]
        if unexpected:
            raise ValueError(f"load_weights: {filepath} holds tensors this model does not have: {unexpected[:4]}")
        bad = [k for k, v in own.items() if tuple(sd[k].shape) != tuple(v.shape)]
        if bad:
            raise ValueError(f"load_weights: shape mismatch for {bad[:4]}: "
                             f"{[(tuple(sd[k].shape), tuple(own[k].shape)) for k in bad[:4]]}")
        with torch.no_grad():
            for k, v in own.items():
                v.copy_(sd[k].to(v.dtype))
        flayers.invalidate_weights()
