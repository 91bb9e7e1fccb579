"""fpnmt — MI355X-native runtime for the FPN + multi-view-transformer
captioning hot path (libfpnmt.so + thin autograd/host plumbing).

Importing this package loads the in-tree HIP library; there is no CPU or
eager-PyTorch fallback (the CPU restatement under oracle/ is test-only).
"""
import torch

from . import _lib  # noqa: F401  (fails loudly if libfpnmt.so is missing)
from . import ops, layers  # noqa: F401

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, "f32": torch.float32,
           torch.bfloat16: torch.bfloat16, torch.float32: torch.float32}


class _Config:
    dtype = torch.bfloat16
    # same-input Dense layers (K/V of a view across encoder layers, Q of all
    # views, decoder self-attn Q/K/V, cross-attn K/V across layers) as one GEMM
    fuse_projections = True
    # single-consumer conv chains (bottleneck 2a->2b->2c, submodel convs ->
    # head) through ops.conv_chain: intermediate ReLU backward fused into the
    # bwd-data epilogues
    fuse_conv_chains = True
    # inference: the ResNet identity bottlenecks with a fused kernel (res2 / res3
    # at 224^2: ops.bottleneck_fused) run as ONE launch each
    fuse_bottleneck = True
    # weight-gradient launches on a second stream beside the dgrad chain,
    # inside ops.side_wgrad() (the TrainEngine's backward): "dense" (the
    # transformer's latency-bound Dense layers), "all" (convolutions too), or
    # False. Off: measured slower on the C2 step (tools/ab_side.sh, one box:
    # 14.54 ms off, 15.73 "dense" with a fork per launch, 15.00 with forks
    # batched 16 at a time) — the captured cross-stream dependencies and the
    # contention cost more than the overlap returns.
    side_wgrad = False
    # the backward's ordered gradient reductions (split-K weight-gradient
    # slabs, bias / LayerNorm column sums) queued and run as a few batched
    # launches at its end (fpnmt_defer_begin / _flush; the TrainEngine)
    defer_reductions = True
    # single-graph step (one GPU): the transformer's clip + AMSGrad runs on a
    # second stream as soon as the transformer's backward is complete, beside
    # the feature extractor's backward; the feature extractor's part follows
    # at the end (ops.transformer_grads_barrier, TrainEngine._early_update).
    # Off: measured slower on the C2 step (profiles/r05/early_update_r5h.txt:
    # 10.84 -> 11.33 ms with 64 persistent workgroups, 10.90 -> 11.14 with one
    # per block) — its HBM traffic slows the backward more than the 0.45 ms
    # it takes off the tail; bitwise equal either way
    # (test_early_update_bitwise_equal)
    early_update = False
    early_update_grid = 64  # workgroups of the early part (persistent, striding over its blocks)
    # a tensor read by a Dense / grouped projection AND as the residual of a
    # later LayerNorm / Dense epilogue (every transformer sublayer input):
    # the residual branch's gradient goes into the projection's bwd-data GEMM
    # epilogue (dx = dz W^T + g_res) instead of an autograd add kernel
    fuse_residual_grads = True
    # the bf16 compute copies of conv / dense kernels whose k is a power of
    # two (16..4096) are written by the AMSGrad kernel itself from the
    # updated masters (fpnmt_amsgrad_step_prep) instead of a separate
    # refresh pass that re-reads them (TrainEngine)
    fuse_optimizer_prep = True
    # keras-resnet identity bottlenecks (the block input is conv 2a's input
    # and 2c's residual): x's two gradients are summed in 2a's bwd-data
    # epilogue (fpnmt_conv2d_bwd_data_res) instead of an autograd add kernel
    fuse_identity_residual = True
    # ... and, when that input is the previous bottleneck's ReLU output, its
    # ReLU' as well (fpnmt_conv2d_bwd_data_res_act): the previous block's
    # output act_bwd pass is skipped when it receives exactly that gradient
    fuse_block_act = True
    # a Conv2D's bias gradient (the column sums of its dz) in its weight-
    # gradient launch (fpnmt_conv2d_bwd_filter_bias / _grouped_bias: the
    # LDS-DMA wgrad kernel sums the dz tiles it streams through LDS) instead
    # of a separate column pass over dz, where that pass would otherwise run
    # (dz == dy: the act' was applied by the consumers, or no activation)
    fuse_bias_wgrad = True
    # a Dense with fused dropout whose output only feeds a LayerNorm (the
    # transformer's `LN(res + dropout(dense))` sublayer ends): the dropout
    # backward is written by the LayerNorm backward (fpnmt_layernorm_bwd_drop)
    # and the Dense skips its act_bwd pass
    fuse_drop_ln = True
    # a tensor with several declared GEMM consumers (ResNet projection-block
    # inputs, C3 / C4 with their FPN laterals, the FPN levels under the two
    # head chains, P5's pre-conv): the consumers' bwd-data launches accumulate
    # into one running gradient (ops.expect_consumers) instead of autograd
    # summing them with add kernels
    fuse_grad_sums = True
    # the Encoder's five view LayerNorms (+ posenc, dropout) as one launch
    # per pass (ops.LayerNormViewsFn) instead of a LayerNorm and a dropout
    # launch per view; the Decoder's embedding dropout in the embedding's
    # launches (fpnmt_embed_posenc_*_drop)
    fuse_view_norms = True
    # the FFN's ffn1 activation backward (LeakyReLU) applied in ffn2's
    # bwd-data epilogue (fpnmt_gemm_act_in) for Dense layers whose output
    # only feeds the next Dense (layers.Dense.act_into_next, set by the
    # Encoder / Decoder layers); ffn1 then skips its act_bwd pass
    fuse_ffn_act = True
    # a conv's input that is a conv chain's / conv's ReLU output (the ResNet
    # stage outputs C2..C5, the stem under its max pool): every consumer's
    # bwd-data (fpnmt_conv2d_bwd_data_mask, also accumulating and strided) or
    # the max pool's backward (fpnmt_maxpool2d_bwd_act) multiplies its
    # contribution by that ReLU', and the producer skips its act_bwd pass when
    # the summed gradient it receives carries the mask
    fuse_input_act = True
    # the gradient arena's zero fill at a step's start on this many
    # workgroups on a side stream beside the forward pass (joined before the
    # backward) instead of a full-chip fill ahead of it; 0 = inline. Off:
    # measured slower on the C2 step (profiles/r05/zero_overlap_ab_r5r.txt,
    # one box, alternating: 10.29 / 10.30 / 10.31 ms inline, 10.58 / 10.61
    # with 64 workgroups, 10.60 with 256) — the fill still saturates HBM
    # under the forward's first kernels and the graph's cross-stream fork /
    # join costs more than the ~80 us it hides; bitwise equal either way
    # (test_zero_grad_overlap_bitwise_equal)
    zero_grad_overlap_grid = 0


config = _Config()


def set_precision(p):
    """'bf16' (MFMA bf16, fp32 accumulate; the perf path) or 'fp32' (exact
    fp32 MFMA; the parity path)."""
    config.dtype = _DTYPES[p]


def compute_dtype():
    return config.dtype
