"""Batched caption decoding: the reference's beam procedure
(utils/pipeline.py:82-154, `Pipeline.predict`) for many images at once with a
K/V cache and one hipGraph per decode step (BASELINE config C5).

Reference semantics kept:
  * every step re-runs the decoder on the beams' sequences; here only the
    newest position is computed — keys/values of earlier positions are
    cached (the causal mask makes them independent of later tokens), and the
    last row of the look-ahead mask keeps every earlier position;
  * beams start identical ([<start>], prob 1); per step softmax of the last
    position, candidates p * beam_prob flattened over beam_n x V, top_k
    (ties to the lower flat index), parents / tokens by // and %, beam_prob =
    the top-k values (a product of probabilities, not logs);
  * the result is the best beam (first argmax of beam_prob) after <start>,
    without <end> when it ends with <end> — per image, frozen at the step the
    reference would `return` (fpnmt_beam_step status flag).
Beams re-rank without moving the cache: every row keeps a table of the cache
rows holding its history's keys/values (fpnmt_decode_attention `src`).

Not reproduced on this path: the attention-weight dict of the last step (the
reference returns it for plotting only).
"""
from __future__ import annotations

import math

import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr, dtype_code
from . import compute_dtype


def _gemm(m, n, k, dt, a, lda, b, c, ldc, bias, s):
    g = L.GemmDesc()
    g.m, g.n, g.k, g.batch, g.batch_inner, g.dtype = m, n, k, 1, 1, dt
    g.a_trans, g.b_trans = 0, 0
    g.lda, g.ldb, g.ldc, g.ldr = lda, k, ldc, ldc
    g.alpha, g.act, g.act_alpha, g.accumulate, g.c_f32, g.split_k = 1.0, L.ACT_NONE, 0.0, 0, 0, 1
    call("fpnmt_gemm", g, a, b, c, None, bias, None, s)


class BeamDecoder:
    """decode(images) -> list of token-id lists, one per image."""

    def __init__(self, transformer, n_images, beam_n, max_seq_len, start_token, end_token, use_graph=True):
        self.tr = transformer
        dec = transformer.decoder
        self.n_images, self.beam_n, self.T = n_images, beam_n, max_seq_len
        self.start_token, self.end_token = start_token, end_token
        self.R = n_images * beam_n
        self.d = dec.d_model
        self.L = dec.num_layers
        self.V = transformer.final_layer.kernel.shape[1]
        self.heads = dec.dec_layers[0].mha1.num_heads if self.L else 8
        self.depth = self.d // self.heads
        if max_seq_len > dec.pos_encoding.shape[0]:
            raise ValueError(f"max_seq_len {max_seq_len} exceeds the decoder's positional table")
        self.use_graph = use_graph
        self.dt = None
        self.graphs = None
        self.qkv_bias = []

    # ---------------------------------------------------------- buffers
    def _alloc(self, dev):
        dt, R, T, d = self.dt, self.R, self.T, self.d
        self.kv = torch.empty((max(self.L, 1), R, T, 2 * d), dtype=dt, device=dev)
        self.hist = [torch.empty((R, T + 1), dtype=torch.int32, device=dev) for _ in range(2)]
        self.src = [torch.empty((R, T), dtype=torch.int32, device=dev) for _ in range(2)]
        self.tok = torch.empty(R, dtype=torch.int32, device=dev)
        self.prob = torch.empty(R, dtype=torch.float32, device=dev)
        self.result = torch.zeros((self.n_images, T), dtype=torch.int32, device=dev)
        self.result_len = torch.zeros(self.n_images, dtype=torch.int32, device=dev)
        self.status = torch.zeros(self.n_images, dtype=torch.int32, device=dev)

    def _reset(self):
        R = self.R
        self.tok.fill_(self.start_token)
        self.prob.fill_(1.0)
        self.hist[0][:, 0] = self.start_token
        self.src[0][:, 0] = torch.arange(R, dtype=torch.int32, device=self.tok.device)
        self.result_len.zero_()
        self.status.zero_()

    # ------------------------------------------------------------- encoder
    def _encode(self, images):
        """Encoder once per image (pipeline.py:93-94) and every layer's cross
        K/V from one grouped GEMM (no per-beam tiling: the attention maps beam
        rows to their image)."""
        tr, dec = self.tr, self.tr.decoder
        enc = tr.encoder(images, False, None)  # (n, Lenc, d)
        self.Lenc = enc.shape[1]
        n = enc.shape[0]
        if self.L == 0:
            self.enc_kv = torch.empty((1, 1), dtype=self.dt, device=enc.device)
            return
        grp = dec.cross_kv_group
        stack, _ = grp.stacked(self.dt)
        cols = grp.n * grp.fout  # 2 * L * d
        shape = (n * self.Lenc, cols)
        if getattr(self, "enc_kv", None) is None or tuple(self.enc_kv.shape) != shape:
            # static buffer: the captured step graphs read it by address
            self.enc_kv = torch.empty(shape, dtype=self.dt, device=enc.device)
            self.graphs = None
        e2 = enc.reshape(n * self.Lenc, self.d).contiguous()
        _gemm(n * self.Lenc, cols, self.d, dtype_code(self.dt), ptr(e2), self.d, ptr(stack), ptr(self.enc_kv), cols,
              ptr(grp.bias_cat()), stream_ptr())

    def _stage_biases(self, dev):
        """Each layer's [q|k|v] bias as one vector the step graphs read by
        address: a view when the biases are adjacent (arena order), else a
        static buffer refreshed here, once per decode call, instead of a
        concatenation per layer inside every step."""
        dec = self.tr.decoder
        if len(self.qkv_bias) != self.L:
            self.qkv_bias = [None] * self.L
        for i, lay in enumerate(dec.dec_layers):
            b = lay.qkv_group.bias_cat()
            cur = self.qkv_bias[i]
            if b._base is not None or b.numel() == 0:  # a view of the parameters
                if cur is None or cur.data_ptr() != b.data_ptr():
                    self.qkv_bias[i] = b
                    self.graphs = None
                continue
            if cur is None or cur.shape != b.shape or cur._base is not None:
                self.qkv_bias[i] = torch.empty_like(b, device=dev)
                self.graphs = None
            self.qkv_bias[i].copy_(b)

    # ---------------------------------------------------------------- step
    def _step(self, t):
        tr, dec = self.tr, self.tr.decoder
        dt, code, R, T, d = self.dt, dtype_code(self.dt), self.R, self.T, self.d
        s = stream_ptr()
        hin, hout = self.hist[t % 2], self.hist[(t + 1) % 2]
        sin, sout = self.src[t % 2], self.src[(t + 1) % 2]
        x = torch.empty((R, d), dtype=dt, device=self.tok.device)
        pe = dec.pos_encoding
        call("fpnmt_embed_posenc_fwd", code, R, 1, d, ptr(self.tok), ptr(dec.embedding.embeddings),
             pe.data_ptr() + t * d * pe.element_size(), ptr(x), s)
        scale = 1.0 / math.sqrt(float(self.depth))
        for i, lay in enumerate(dec.dec_layers):
            grp = lay.qkv_group
            stack, _ = grp.stacked(dt)
            bias = self.qkv_bias[i]
            q = torch.empty((R, d), dtype=dt, device=x.device)
            _gemm(R, d, d, code, ptr(x), d, ptr(stack), ptr(q), d, ptr(bias), s)
            kvl = self.kv[i]
            # this position's key / value straight into the cache (row r, position t)
            _gemm(R, 2 * d, d, code, ptr(x), d, stack.data_ptr() + d * d * stack.element_size(),
                  kvl.data_ptr() + t * 2 * d * kvl.element_size(), T * 2 * d,
                  bias.data_ptr() + d * bias.element_size(), s)
            a = torch.empty((R, d), dtype=dt, device=x.device)
            call("fpnmt_decode_attention", code, R, self.heads, self.depth, t + 1, scale, ptr(q), d, ptr(kvl),
                 T * 2 * d, 2 * d, 0, d, ptr(sin), T, 1, ptr(a), d, s)
            out1 = lay.layernorm1(lay.mha1.dense(a), residual=x)
            q2 = lay.mha2.wq(out1)
            a2 = torch.empty((R, d), dtype=dt, device=x.device)
            cols = 2 * self.L * d
            call("fpnmt_decode_attention", code, R, self.heads, self.depth, self.Lenc, scale, ptr(q2), d,
                 ptr(self.enc_kv), self.Lenc * cols, cols, 2 * i * d, 2 * i * d + d, None, 0, self.beam_n, ptr(a2),
                 d, s)
            out2 = lay.layernorm2(lay.mha2.dense(a2), residual=out1)
            x = lay.layernorm3(lay.ffn2(lay.ffn1(out2)), residual=out2)
        logits = tr.final_layer(x)  # (R, V) fp32
        call("fpnmt_beam_step", self.n_images, self.beam_n, self.V, ptr(logits), self.V, ptr(self.prob), ptr(hin),
             ptr(hout), T + 1, t, ptr(sin), ptr(sout), T, self.end_token, ptr(self.tok), ptr(self.result), T,
             ptr(self.result_len), ptr(self.status), s)

    # -------------------------------------------------------------- decode
    @torch.no_grad()
    def decode(self, images, check_every=8):
        """images (n_images, H, W, 3) on the GPU -> list of token-id lists."""
        if images.shape[0] != self.n_images:
            raise ValueError(f"expected {self.n_images} images, got {images.shape[0]}")
        dt = compute_dtype()
        if self.dt != dt:
            self.dt = dt
            self._alloc(images.device)
            self.enc_kv = None
            self.graphs = None
        self._encode(images)
        self._stage_biases(images.device)
        self._reset()
        if self.use_graph and self.graphs is None:
            self._capture()
        for t in range(self.T):
            if self.graphs is not None:
                self.graphs[t].replay()
            else:
                self._step(t)
            if check_every and (t + 1) % check_every == 0 and t + 1 < self.T and bool(self.status.all()):
                break
        lens = self.result_len.tolist()
        res = self.result.cpu()
        return [res[i, :lens[i]].tolist() for i in range(self.n_images)]

    def _capture(self):
        """One graph per position t (the step's shapes depend on t). The
        first step runs eagerly to build compute copies / workspaces; the
        state it advances is reset before the graphs are replayed."""
        from .train import capture_sequence
        self._step(0)
        torch.cuda.synchronize()
        graphs = capture_sequence([(lambda t=t: self._step(t)) for t in range(self.T)])
        self.graphs = graphs
        self._reset()
