"""ORACLE — test infrastructure only. CPU (torch fp32, eager, autograd) restatement
of the reference's FPN + multi-view-transformer captioning path
(samkoesnadi/fpn-MT-image-captioning). Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product path
(fpn-mt-image-captioning_amd/) never does.

PARITY STATUS: partially pinned. The reference is TensorFlow 2 / Keras and
TensorFlow is not installed here (an ordinary ModuleNotFoundError, not a
denial), its ResNet backbone depends on keras-resnet (absent, never vendored)
and its tests hold no golden vectors. This restatement is
pinned by the closed-form known answers the reference's own code yields
(co-attention sample coattention.py:44-51, positional encoding
transformer.py:22-39, CustomSchedule utils/utils.py:45-50, look-ahead mask
transformer.py:54-56, the beam==greedy property of pipeline.py:101-144);
full-model values are otherwise "parity unpinned" against TF.

Weights are passed as a flat name -> tensor dict using the product model's
state_dict() names (Keras layouts: conv HWIO, dense (in, out)), so both sides
run on identical weights. Dropout is not modelled (parity runs use rate 0).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

LEAKY = 0.2            # tf.nn.leaky_relu default alpha (common_definitions.py:14)
LN_EPS = 1e-6          # transformer.py:170-171,216-218,264
NUM_OF_PYRAMIDS = 5    # common_definitions.py:66
BASELINE_INDEX = 3     # common_definitions.py:70
RESNET_BLOCKS = {"resnet50": [3, 4, 6, 3], "resnet101": [3, 4, 23, 3], "resnet152": [3, 8, 36, 3]}


# ----------------------------------------------------------------- basics
def conv2d(x, kernel, bias=None, stride=1, pads=(0, 0, 0, 0)):
    """NHWC conv, HWIO kernel, explicit (top, bottom, left, right) zero pads."""
    xt = x.permute(0, 3, 1, 2)
    pt, pb, pl, pr = pads
    if pt or pb or pl or pr:
        xt = F.pad(xt, (pl, pr, pt, pb))
    if xt.shape[2] < kernel.shape[0] or xt.shape[3] < kernel.shape[1]:
        ho = max((xt.shape[2] - kernel.shape[0]) // stride + 1, 0)
        wo = max((xt.shape[3] - kernel.shape[1]) // stride + 1, 0)
        return x.new_zeros((x.shape[0], ho, wo, kernel.shape[3]))
    y = F.conv2d(xt, kernel.permute(3, 2, 0, 1).contiguous(), bias, stride=stride)
    return y.permute(0, 2, 3, 1)


def same_pads(h, w, kh, kw, sh=1, sw=1):
    """TF 'same': total = max((ceil(n/s)-1)*s + k - n, 0), before = total // 2."""
    ho, wo = -(-h // sh), -(-w // sw)
    th = max((ho - 1) * sh + kh - h, 0)
    tw = max((wo - 1) * sw + kw - w, 0)
    return th // 2, th - th // 2, tw // 2, tw - tw // 2


def conv_same(x, kernel, bias=None):
    return conv2d(x, kernel, bias, 1, same_pads(x.shape[1], x.shape[2], kernel.shape[0], kernel.shape[1]))


def leaky(x):
    return F.leaky_relu(x, LEAKY)


def maxpool_valid(x, k=2, s=2):
    """Keras MaxPooling2D(): 2x2 / 2, VALID; 1x1 -> 0x0 is legal (retinanet.py:135,139,293)."""
    n, h, w, c = x.shape
    ho, wo = max((h - k) // s + 1, 0), max((w - k) // s + 1, 0)
    if ho == 0 or wo == 0:
        return x.new_zeros((n, ho, wo, c))
    return F.max_pool2d(x.permute(0, 3, 1, 2), k, s).permute(0, 2, 3, 1)


def maxpool_same(x, k=3, s=2):
    """keras-resnet pool1: MaxPooling2D(3, 2, 'same') (pads with -inf)."""
    pt, pb, pl, pr = same_pads(x.shape[1], x.shape[2], k, k, s, s)
    xt = F.pad(x.permute(0, 3, 1, 2), (pl, pr, pt, pb), value=float("-inf"))
    return F.max_pool2d(xt, k, s).permute(0, 2, 3, 1)


def nearest_index(out, inp):
    """TF2 tf.image.resize NEAREST (half_pixel_centers): min(floor((d+.5)*in/out), in-1)."""
    d = torch.arange(out, dtype=torch.float32)
    s = torch.floor((d + 0.5) * (float(inp) / float(out))).to(torch.int64)
    return torch.clamp(s, max=inp - 1)


def upsample_like(source, target):
    """layers/_misc.py:39-42 (UpsampleLike -> resize_images(..., 'nearest'))."""
    hi = nearest_index(target.shape[1], source.shape[1])
    wi = nearest_index(target.shape[2], source.shape[2])
    return source[:, hi][:, :, wi]


def layer_norm(x, gamma, beta):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) * torch.rsqrt(var + LN_EPS) * gamma + beta


def dense(sd, p, x, act=None):
    y = x @ sd[p + ".kernel"] + sd[p + ".bias"]
    return leaky(y) if act == "leaky" else y


# ------------------------------------------------------------ ResNet (A1)
def frozen_bn_conv(sd, p, x, stride=1, pads=(0, 0, 0, 0)):
    """keras-resnet Conv2D(use_bias=False) + BatchNormalization(eps 1e-5, freeze=True)."""
    y = conv2d(x, sd[p + ".kernel"], None, stride, pads)
    sc = sd[p + ".bn_gamma"] / torch.sqrt(sd[p + ".bn_var"] + 1e-5)
    return y * sc + (sd[p + ".bn_beta"] - sd[p + ".bn_mean"] * sc)


def resnet(sd, p, x, depth="resnet50"):
    """keras_resnet.models.ResNet{50,101}(include_top=False, freeze_bn=True) -> [C2..C5]
    (models/resnet.py:99,101,112)."""
    x = F.relu(frozen_bn_conv(sd, p + ".conv1", x, 2, (3, 3, 3, 3)))
    x = maxpool_same(x, 3, 2)
    outs = []
    for si, n in enumerate(RESNET_BLOCKS[depth]):
        for bi in range(n):
            stride = 1 if (bi != 0 or si == 0) else 2
            b = f"{p}.stages.{si}.{bi}"
            y = F.relu(frozen_bn_conv(sd, b + ".conv2a", x, stride))
            y = F.relu(frozen_bn_conv(sd, b + ".conv2b", y, 1, (1, 1, 1, 1)))
            y = frozen_bn_conv(sd, b + ".conv2c", y)
            sc = frozen_bn_conv(sd, b + ".shortcut", x, stride) if bi == 0 else x
            x = F.relu(y + sc)
        outs.append(x)
    return outs


# ------------------------------------------- MobileNetV2
# keras_applications.mobilenet_v2.MobileNetV2(alpha=1.0, include_top=False,
# weights=None) as built by models/mobilenet.py:61 on Input((None, None, 3))
# (third-party, unpinned; restated from its published definition), tapped at
# block_5_add / block_12_add / out_relu (models/mobilenet.py:64).
MBV2_BLOCKS = [  # (expansion, filters, stride) for block_id 0..16
    (1, 16, 1), (6, 24, 2), (6, 24, 1), (6, 32, 2), (6, 32, 1), (6, 32, 1), (6, 64, 2), (6, 64, 1), (6, 64, 1),
    (6, 64, 1), (6, 96, 1), (6, 96, 1), (6, 96, 1), (6, 160, 2), (6, 160, 1), (6, 160, 1), (6, 320, 1)]
BN_EPS_MBV2 = 1e-3
BN_MOMENTUM_MBV2 = 0.999
# correct_pad() of a stride-2 3x3 on an input of unknown (None) size:
# adjust = (1, 1) -> ((0, 1), (0, 1)), i.e. top 0, bottom 1, left 0, right 1
STRIDE2_PADS = (0, 1, 0, 1)


def relu6(x):
    return torch.clamp(x, 0.0, 6.0)


def batch_norm(sd, p, x, training, stats=None):
    """tf.keras BatchNormalization(epsilon=1e-3, momentum=0.999) over NHWC
    channels. training: batch mean / biased variance normalise; the moving
    averages move by (1 - momentum) toward the batch mean and the
    Bessel-corrected batch variance (fused batch norm's variance output),
    recorded in ``stats`` when given. Otherwise the moving statistics."""
    g, b = sd[p + ".gamma"], sd[p + ".beta"]
    if training:
        red = tuple(range(x.dim() - 1))
        mean = x.mean(red)
        var = x.var(red, unbiased=False)
        if stats is not None:
            n = x.numel() // x.shape[-1]
            unb = var * (n / max(n - 1, 1))
            m0, v0 = sd[p + ".moving_mean"], sd[p + ".moving_variance"]
            stats[p + ".moving_mean"] = m0 * BN_MOMENTUM_MBV2 + mean.detach() * (1 - BN_MOMENTUM_MBV2)
            stats[p + ".moving_variance"] = v0 * BN_MOMENTUM_MBV2 + unb.detach() * (1 - BN_MOMENTUM_MBV2)
    else:
        mean, var = sd[p + ".moving_mean"], sd[p + ".moving_variance"]
    return (x - mean) * torch.rsqrt(var + BN_EPS_MBV2) * g + b


def depthwise_conv(x, kernel, stride=1, pads=(1, 1, 1, 1)):
    """DepthwiseConv2D(3, stride, use_bias=False): kernel (kh, kw, C, 1)."""
    c = x.shape[-1]
    xt = F.pad(x.permute(0, 3, 1, 2), (pads[2], pads[3], pads[0], pads[1]))
    w = kernel.permute(2, 3, 0, 1).contiguous()  # (C, 1, kh, kw)
    return F.conv2d(xt, w, None, stride=stride, groups=c).permute(0, 2, 3, 1)


def mobilenet_v2(sd, p, x, training=False, stats=None):
    """-> [block_5_add (H/8, 32), block_12_add (H/16, 96), out_relu (H/32, 1280)]."""
    x = conv2d(x, sd[p + ".conv1.kernel"], None, 2, STRIDE2_PADS)
    x = relu6(batch_norm(sd, p + ".bn_conv1", x, training, stats))
    taps = []
    for bi, (t, f, st) in enumerate(MBV2_BLOCKS):
        q = f"{p}.blocks.{bi}"
        inp = x
        if bi:
            x = relu6(batch_norm(sd, q + ".expand_bn", conv2d(x, sd[q + ".expand.kernel"]), training, stats))
        pads = STRIDE2_PADS if st == 2 else (1, 1, 1, 1)
        x = depthwise_conv(x, sd[q + ".depthwise.kernel"], st, pads)
        x = relu6(batch_norm(sd, q + ".depthwise_bn", x, training, stats))
        x = batch_norm(sd, q + ".project_bn", conv2d(x, sd[q + ".project.kernel"]), training, stats)
        if inp.shape[-1] == f and st == 1:
            x = inp + x
        if bi in (5, 12):
            taps.append(x)
    x = relu6(batch_norm(sd, p + ".conv_1_bn", conv2d(x, sd[p + ".conv_1.kernel"]), training, stats))
    return taps + [x]


# --------------------------------------------------------------- FPN (A2)
def pyramid_features(sd, p, C3, C4, C5):
    """retinanet.py:105-141."""
    c = lambda n, x: conv_same(x, sd[f"{p}.{n}.kernel"], sd[f"{p}.{n}.bias"])
    P5f = c("C5_reduced", C5)
    P5_up = upsample_like(P5f, C4)
    P5 = F.relu(c("P5", P5f))
    P4 = c("C4_reduced", C4)
    P4 = P5_up + P4
    P4_up = upsample_like(P4, C3)
    P4 = F.relu(c("P4", P4))
    P3 = c("C3_reduced", C3)
    P3 = P4_up + P3
    P3 = F.relu(c("P3", P3))
    P6 = maxpool_valid(F.relu(c("P6_conv", P5f)))
    P7 = maxpool_valid(F.relu(c("P7_conv", P6)))
    return [P3, P4, P5, P6, P7]


def coattention(score, hs):
    """coattention.py:13-32: softmax of score over h*w, times hs."""
    b, h, w, _ = score.shape
    a = torch.softmax(score.reshape(b, h * w), dim=1).reshape(b, h, w, 1)
    return a * hs


def feature_extractor(sd, p, img, depth="resnet50", training=False, stats=None):
    """retinanet.py:266-307 over a ResNet (frozen BN) or MobileNetV2 (BN in
    training mode when ``training``) backbone: 5 x (B, h/2, w/2, 512)."""
    rp = p + ".retinanet_model"
    if depth.startswith("mobilenet"):
        C3, C4, C5 = mobilenet_v2(sd, rp + ".backbone", img, training, stats)
    else:
        C2, C3, C4, C5 = resnet(sd, rp + ".backbone", img, depth)
    feats = pyramid_features(sd, rp + ".fpn", C3, C4, C5)
    outs = []
    for f in feats:
        r, cl = f, f
        for i in range(2):
            r = F.relu(conv_same(r, sd[f"{rp}.submodels.0.convs.{i}.kernel"], sd[f"{rp}.submodels.0.convs.{i}.bias"]))
            cl = F.relu(conv_same(cl, sd[f"{rp}.submodels.1.convs.{i}.kernel"], sd[f"{rp}.submodels.1.convs.{i}.bias"]))
        reg = conv_same(r, sd[p + ".regression.kernel"], sd[p + ".regression.bias"])
        cls = conv_same(cl, sd[p + ".classification.kernel"], sd[p + ".classification.bias"])
        o = coattention(reg, cls)
        o = leaky(conv_same(o, sd[p + ".post_conv.kernel"], sd[p + ".post_conv.bias"]))
        o = maxpool_valid(o)
        o = leaky(conv_same(o, sd[p + ".out_conv.kernel"], sd[p + ".out_conv.bias"]))
        outs.append(o)
    return outs


# ------------------------------------------------------- transformer (A7-A14)
def get_angles(pos, i, d_model):
    return pos * (1 / np.power(10000, (2 * (i // 2)) / np.float32(d_model)))


def raw_positional_encoding(position, d_model):
    """transformer.py:27-39 (float64 then fp32)."""
    a = get_angles(np.arange(position)[:, None], np.arange(d_model)[None, :], d_model)
    a[:, 0::2] = np.sin(a[:, 0::2])
    a[:, 1::2] = np.cos(a[:, 1::2])
    return torch.from_numpy(a.astype(np.float32))


def create_padding_mask(seq):
    return (seq == 0).to(torch.float32)[:, None, None, :]


def create_look_ahead_mask(size):
    return 1 - torch.tril(torch.ones(size, size))


def create_masks(tar):
    return torch.maximum(create_padding_mask(tar), create_look_ahead_mask(tar.shape[1]))


def scaled_dot_product_attention(q, k, v, mask):
    """transformer.py:70-104."""
    logits = q @ k.transpose(-1, -2) / math.sqrt(k.shape[-1])
    if mask is not None:
        logits = logits + mask * -1e9
    w = torch.softmax(logits, dim=-1)
    return w @ v, w


def mha(sd, p, v, k, q, mask, num_heads):
    """transformer.py:107-155, call order (v, k, q, mask)."""
    b = q.shape[0]
    d = sd[p + ".wq.kernel"].shape[1]
    depth = d // num_heads
    split = lambda x: x.reshape(b, -1, num_heads, depth).permute(0, 2, 1, 3)
    q, k, v = split(dense(sd, p + ".wq", q)), split(dense(sd, p + ".wk", k)), split(dense(sd, p + ".wv", v))
    o, w = scaled_dot_product_attention(q, k, v, mask)
    o = o.permute(0, 2, 1, 3).reshape(b, -1, d)
    return dense(sd, p + ".dense", o), w


def encoder_layer(sd, p, x, mask, num_heads):
    """transformer.py:176-200 (out = baseline + sum of 4 view MHAs, non-aliasing)."""
    baseline = x[NUM_OF_PYRAMIDS - 1]
    out = baseline
    for i in range(NUM_OF_PYRAMIDS - 1):
        m, _ = mha(sd, f"{p}.mhas.{i}", x[i], x[i], baseline, mask, num_heads)
        out = out + m
    out1 = layer_norm(out, sd[p + ".layernorm1.gamma"], sd[p + ".layernorm1.beta"])
    f = dense(sd, p + ".ffn2", dense(sd, p + ".ffn1", out1, "leaky"))
    return layer_norm(out1 + f, sd[p + ".layernorm2.gamma"], sd[p + ".layernorm2.beta"])


def encoder(sd, img, cfg, training=False, stats=None):
    """transformer.py:266-303 (training: BatchNormalization in training mode,
    as Keras propagates the call's training flag to the backbone)."""
    p = "encoder"
    x = feature_extractor(sd, p + ".feature_extractor", img, cfg["backbone"], training, stats)
    order = [i for i in range(NUM_OF_PYRAMIDS) if i != BASELINE_INDEX] + [BASELINE_INDEX]
    x = [x[i] for i in order]
    pe = sd[p + ".pos_encoding"]
    for i in range(NUM_OF_PYRAMIDS):
        b, h, w, c = x[i].shape
        t = x[i].reshape(b, h * w, c)
        t = layer_norm(t, sd[p + ".layernorm1.gamma"], sd[p + ".layernorm1.beta"])
        x[i] = t + pe[: h * w]
    for li in range(cfg["num_layers"]):
        x[NUM_OF_PYRAMIDS - 1] = encoder_layer(sd, f"{p}.enc_layers.{li}", x, None, cfg["num_heads"])
    return x[NUM_OF_PYRAMIDS - 1]


def decoder_layer(sd, p, x, enc, look_ahead_mask, num_heads):
    """transformer.py:224-243."""
    a1, w1 = mha(sd, p + ".mha1", x, x, x, look_ahead_mask, num_heads)
    out1 = layer_norm(a1 + x, sd[p + ".layernorm1.gamma"], sd[p + ".layernorm1.beta"])
    a2, w2 = mha(sd, p + ".mha2", enc, enc, out1, None, num_heads)
    out2 = layer_norm(a2 + out1, sd[p + ".layernorm2.gamma"], sd[p + ".layernorm2.beta"])
    f = dense(sd, p + ".ffn2", dense(sd, p + ".ffn1", out2, "leaky"))
    return layer_norm(f + out2, sd[p + ".layernorm3.gamma"], sd[p + ".layernorm3.beta"]), w1, w2


def decoder(sd, tar, enc, look_ahead_mask, cfg, emb_hook=None):
    """transformer.py:321-341 (Embedding without sqrt(d) scaling)."""
    emb = sd["decoder.embedding.embeddings"][tar.long()]
    if emb_hook is not None:
        emb = emb_hook(emb)
    x = emb + sd["decoder.pos_encoding"][: tar.shape[1]]
    weights = {}
    for li in range(cfg["num_layers"]):
        x, w1, w2 = decoder_layer(sd, f"decoder.dec_layers.{li}", x, enc, look_ahead_mask, cfg["num_heads"])
        weights[f"decoder_layer{li + 1}_block1"] = w1
        weights[f"decoder_layer{li + 1}_block2"] = w2
    return x, weights


def transformer(sd, inp, tar, training, look_ahead_mask, cfg, emb_hook=None):
    """transformer.py:359-374."""
    enc = encoder(sd, inp, cfg, training=True, stats=cfg.get("bn_stats")) if training else inp
    dec, w = decoder(sd, tar, enc, look_ahead_mask, cfg, emb_hook)
    return dec @ sd["final_layer.kernel"] + sd["final_layer.bias"], w


# ------------------------------------------------------------ train (A15)
def masked_loss(real, pred):
    """utils/pipeline.py:50-57: CE from logits * (real != 0), mean over all B*T."""
    ce = F.cross_entropy(pred.reshape(-1, pred.shape[-1]), real.reshape(-1).long(), reduction="none")
    return (ce * (real.reshape(-1) != 0).to(ce.dtype)).mean()


def custom_schedule(step, d_model=2048, warmup=4000, mult=1):
    """utils/utils.py:45-50 in fp32; lr(0) = 0."""
    f = np.float32
    step = f(step)
    rs = f(1) / np.sqrt(step) if step > 0 else f(np.inf)
    arg1 = rs / np.maximum((step - f(warmup)) * f(mult) / f(warmup * 2), f(1))
    arg2 = step * f(warmup ** -1.5)
    return float(f(1) / np.sqrt(f(d_model)) * np.minimum(arg1, arg2))


def loss_and_grads(sd, img, tok, cfg, trainable):
    """Forward + backward of one train step (pipeline.py:64-77). Returns
    (loss, logits, grads{name}, emb_sumsq) where emb_sumsq is the TF
    IndexedSlices norm^2 of the embedding gradient (per-position rows)."""
    params = {k: (v.detach().clone().requires_grad_(k in trainable)) for k, v in sd.items()}
    tar_inp, tar_real = tok[:, :-1], tok[:, 1:]
    mask = create_masks(tar_inp)
    holder = {}

    def hook(e):
        e.retain_grad()
        holder["e"] = e
        return e

    logits, _ = transformer(params, img, tar_inp, True, mask, cfg, emb_hook=hook)
    loss = masked_loss(tar_real, logits)
    loss.backward()
    grads = {k: (params[k].grad if params[k].grad is not None else torch.zeros_like(params[k])) for k in trainable}
    emb_sumsq = float((holder["e"].grad.double() ** 2).sum()) if "e" in holder else 0.0
    return loss.detach(), logits.detach(), grads, emb_sumsq


class KerasAMSGrad:
    """tf.keras Adam(beta_1, beta_2, epsilon, amsgrad=True, clipnorm) as applied by
    pipeline.py:30,78 (TF >= 2.4: per-gradient clip_by_norm; dense variables through
    ResourceApplyAdamWithAmsgrad, the embedding through the sparse Python path)."""

    def __init__(self, names, shapes, beta1=0.9, beta2=0.98, eps=1e-9, clipnorm=1.0, sparse=(), dtype=torch.float32):
        self.b1, self.b2, self.eps, self.clip = beta1, beta2, eps, clipnorm
        self.dtype = dtype
        self.m = {n: torch.zeros(s, dtype=dtype) for n, s in zip(names, shapes)}
        self.v = {n: torch.zeros(s, dtype=dtype) for n, s in zip(names, shapes)}
        self.vhat = {n: torch.zeros(s, dtype=dtype) for n, s in zip(names, shapes)}
        self.iterations = 0
        self.sparse = set(sparse)

    def apply(self, params, grads, lr_fn, norms=None):
        f = np.float64 if self.dtype == torch.float64 else np.float32
        it = self.iterations
        lr = f(lr_fn(it))
        t = f(it + 1)
        alpha = f(lr * np.sqrt(f(1) - np.power(f(self.b2), t)) / (f(1) - np.power(f(self.b1), t)))
        for n, g in grads.items():
            g = g.to(self.dtype)
            if self.clip and self.clip > 0:
                ss = (norms or {}).get(n, float((g.double() ** 2).sum()))
                nrm = math.sqrt(ss) if ss > 0 else 0.0
                g = (g * self.clip) / max(nrm, self.clip)
            m, v, vh = self.m[n], self.v[n], self.vhat[n]
            if n in self.sparse:
                m.copy_(m * self.b1 + g * (1 - self.b1))
                v.copy_(v * self.b2 + (g * g) * (1 - self.b2))
            else:
                m.add_((g - m) * (1 - self.b1))
                v.add_((g * g - v) * (1 - self.b2))
            vh.copy_(torch.maximum(vh, v))
            params[n] = params[n] - (m * float(alpha)) / (torch.sqrt(vh) + self.eps)
        self.iterations += 1


# ---------------------------------------------------------- predict (A16)
def top_k_lowest_index(x, k):
    vals, idx = torch.sort(x, descending=True, stable=True)
    return vals[:k], idx[:k]


def predict(sd, img, max_seq_len, cfg, start_token, end_token, beam_n=4):
    """utils/pipeline.py:82-154 literally (beams start identical -> greedy)."""
    enc = encoder(sd, img[None], cfg)
    enc = enc.repeat(beam_n, 1, 1)
    V = sd["final_layer.kernel"].shape[1]
    beam_output = torch.full((beam_n, 1), start_token, dtype=torch.int64)
    beam_prob = torch.ones((beam_n, 1))
    beam_result = None
    for _ in range(max_seq_len):
        mask = create_look_ahead_mask(beam_output.shape[1])
        logits, _ = transformer(sd, enc, beam_output, False, mask, cfg)
        pr = torch.softmax(logits[:, -1, :], dim=-1)
        cand = (pr * beam_prob).reshape(-1)
        vals, idx = top_k_lowest_index(cand, beam_n)
        ib = idx // V
        jb = idx - ib * V
        beam_output = torch.cat([beam_output[ib], jb[:, None]], dim=-1)
        beam_prob = vals[:, None]
        beam_result = beam_output[int(torch.argmax(beam_prob[:, 0]))]
        if int(beam_result[-1]) == end_token:
            return beam_result[1:-1]
    if int(beam_result[-1]) == end_token:
        return beam_result[1:-1]
    return beam_result[1:]


def greedy(sd, img, max_seq_len, cfg, start_token, end_token):
    """Greedy arg-max decode (ties -> lowest id) — equal to predict() by §0."""
    enc = encoder(sd, img[None], cfg)
    out = torch.tensor([[start_token]], dtype=torch.int64)
    for _ in range(max_seq_len):
        logits, _ = transformer(sd, enc, out, False, create_look_ahead_mask(out.shape[1]), cfg)
        nxt = int(torch.argmax(logits[0, -1]))
        out = torch.cat([out, torch.tensor([[nxt]])], dim=-1)
        if nxt == end_token:
            return out[0, 1:-1]
    return out[0, 1:]
