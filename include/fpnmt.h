/*
 * fpnmt.h — C-ABI of the MI355X-native FPN + multi-view-transformer captioning
 * hot path (libfpnmt.so, gfx950 only).
 *
 * Every entry point replaces a TensorFlow/Keras op that the reference calls on
 * its training / decoding path (samkoesnadi/fpn-MT-image-captioning; all
 * file:line below point into that repository):
 *
 *   fpnmt_conv2d_*         Conv2D            models/retinanet.py:55-62,94-100,118-138,287-294,
 *                                            keras-resnet convs behind models/resnet.py:99,101
 *   fpnmt_gemm             Dense / MatMul    models/transformer.py:88,102,117-121,153,165-168,211-214,357
 *   fpnmt_attention_*      scaled_dot_product_attention  models/transformer.py:70-104
 *   fpnmt_fpn_topdown_*    UpsampleLike + Add           models/retinanet.py:119,123-125,129-130; layers/_misc.py:39-42
 *   fpnmt_maxpool2d_*      MaxPooling2D()               models/retinanet.py:135,139,293 (+ keras-resnet pool1)
 *   fpnmt_spatial_softmax_* CoAttention_CNN.call        models/coattention.py:13-32
 *   fpnmt_layernorm_*      LayerNormalization(1e-6)     models/transformer.py:170-171,216-218,264
 *   fpnmt_embed_posenc_*   Embedding + positional enc.  models/transformer.py:314,326-329
 *   fpnmt_xent_fwd_bwd     masked sparse CE             utils/pipeline.py:50-57
 *   fpnmt_amsgrad_step     Adam(amsgrad, clipnorm=1)    utils/pipeline.py:29-30,78; utils/utils.py:45-50
 *   fpnmt_dropout          Dropout(rate)                models/transformer.py:173-174,219-222,262,319
 *   fpnmt_decode_attention scaled_dot_product_attention, last query row   utils/pipeline.py:105-113
 *   fpnmt_beam_step        softmax + top_k + gather + argmax of predict   utils/pipeline.py:115-147
 *
 * Conventions (all functions):
 *   - Return 0 on success or a negative FPNMT_E* code; never throw across the ABI.
 *     fpnmt_last_error() returns a thread-local message for the last failure.
 *   - Memory is caller-owned device memory; pointers are never retained.
 *   - Work is enqueued on the given stream only: no allocation, no device
 *     synchronisation, no host blocking — every call is hipGraph-capturable.
 *   - Activations are NHWC; conv weights HWIO (Keras layout) for the fp32 master
 *     copy, OHWI ("fwd") and flipped IHWO ("bwd") for the compute copies made by
 *     fpnmt_weight_prep. Dense kernels are (in, out) like Keras.
 *   - dtype selects the element type of activations / compute weights:
 *     FPNMT_F32 (exact f32 MFMA path, parity mode) or FPNMT_BF16 (bf16 MFMA,
 *     fp32 accumulate). Master weights, gradients and optimizer state are fp32.
 */
#ifndef FPNMT_H
#define FPNMT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fpnmt_stream_t; /* hipStream_t */

enum { FPNMT_F32 = 0, FPNMT_BF16 = 1 };
enum { FPNMT_ACT_NONE = 0, FPNMT_ACT_RELU = 1, FPNMT_ACT_LEAKY = 2, FPNMT_ACT_RELU6 = 3 };
enum {
  FPNMT_OK = 0,
  FPNMT_E_ARG = -1,         /* bad descriptor / null pointer / inconsistent sizes */
  FPNMT_E_UNSUPPORTED = -2, /* shape or alignment not handled by any kernel */
  FPNMT_E_HIP = -3          /* HIP launch error */
};

/* ---- library ---------------------------------------------------------- */
const char* fpnmt_last_error(void);
int fpnmt_version(void);
/* Build provenance: the first 16 hex digits of the sha256 over the csrc/
 * sources, headers, Makefile and this header the library was built from
 * (csrc/Makefile BUILD_ID). fpnmt/_lib.py refuses a library whose id does not
 * match the tree it sits in (a stale prebuilt .so). */
const char* fpnmt_build_id(void);
/* Zero `bytes` of device memory as a kernel node (a captured hipMemsetAsync
 * was measured not to re-zero on graph replay; tools/probes/conv_noise.py):
 * the gradient arena's per-step zeroing. */
int fpnmt_fill_zero(void* p, long long bytes, fpnmt_stream_t stream);
/* fpnmt_fill_zero on at most max_blocks workgroups (a 16-B aligned buffer;
 * else it is fpnmt_fill_zero): the gradient arena's zeroing as a trickle on a
 * side stream beside the forward pass (TrainEngine, zero_grad_overlap_grid),
 * instead of a full-chip fill on the critical path (keras' fresh tape
 * gradients per tape.gradient, utils/pipeline.py:77).                      */
int fpnmt_fill_zero_grid(void* p, long long bytes, int max_blocks, fpnmt_stream_t stream);

/* Process-wide GEMM workspace (device memory, ZERO-initialised by the caller,
 * >= 72 KiB, 256-B aligned; NULL detaches). Under-filled small-M GEMMs split
 * K across blocks and combine the partial tiles here in a fixed order (the
 * result is deterministic); the per-tile arrival counters are re-zeroed by
 * the kernels, so the buffer stays valid across launches and graph replays.
 * GEMMs using it must not run concurrently on different streams.          */
int fpnmt_set_workspace(void* ws, long long bytes);

/* Deferred ordered reductions. Between fpnmt_defer_begin and
 * fpnmt_defer_flush, the ordered second passes of the fp32 gradient
 * reductions — split-K weight-gradient slabs -> dw (bwd-filter / transposed
 * GEMMs with accumulate = 2), per-chunk column partials -> bias / LayerNorm
 * gamma / beta gradients (fpnmt_act_bwd, fpnmt_layernorm_bwd) — keep their
 * inputs in `arena` (device memory, 256-B aligned, caller-owned, untouched
 * until the flush) and are queued instead of launched; fpnmt_defer_flush
 * enqueues them on `stream` as a few batched launches. Results are bitwise
 * those of immediate mode (each reduction keeps its order; a reduction into
 * a destination that already has a queued one, or an immediate accumulation
 * into it, runs the queue first) — except the Dense weight-gradient GEMMs
 * entered through fpnmt_gemm_wgrad (below), which the flush runs as whole-K
 * tiles: equal to immediate mode up to fp32 summation order. Gradients are
 * complete only after the flush. A full arena falls back to immediate
 * reductions. Single stream. A plain fpnmt_gemm is never queued.
 * fpnmt_defer_peak_bytes: the most arena bytes in use so far.              */
int fpnmt_defer_begin(void* arena, long long bytes);
int fpnmt_defer_flush(fpnmt_stream_t stream);
long long fpnmt_defer_peak_bytes(void);

/* ---- general batched GEMM on MFMA (Dense layers, attention products) ---
 * C[z] = epilogue(alpha * op(A[z]) @ op(B[z]))  for z in [0, batch)
 * z is split as (zo, zi) = (z / batch_inner, z % batch_inner); operand X of
 * batch z starts at X + zo*X_so + zi*X_si (elements).
 * a_trans = 0: A is M x K, element (m,k) at A[m*lda + k]
 * a_trans = 1: A is stored K x M, element (m,k) at A[k*lda + m]
 * b_trans = 0: B is stored N x K (k contiguous), element (k,n) at B[n*ldb + k]
 * b_trans = 1: B is stored K x N (n contiguous), element (k,n) at B[k*ldb + n]
 * Epilogue: v = acc*alpha; v *= col_scale[n]; v += bias[n]; v += R[m*ldr+n];
 *           v = act(v); C = v (or C += v when accumulate; atomic when
 *           accumulate == 2, which also allows split-K over blocks).
 * c_f32 = 1 writes C as fp32 regardless of dtype.                        */
typedef struct fpnmt_gemm_desc {
  int m, n, k;
  int batch, batch_inner;
  int dtype;
  int a_trans, b_trans;
  long long lda, ldb, ldc, ldr;
  long long a_so, a_si, b_so, b_si, c_so, c_si, r_so, r_si;
  float alpha;
  int act;
  float act_alpha;
  int accumulate; /* 0 store, 1 read-modify-write, 2 fp32 atomic add */
  int c_f32;
  int split_k;    /* >=1; >1 requires accumulate == 2 */
  /* fused dropout (batch == 1, accumulate != 2): when drop_p > 0 the output is
   * R + dropout(act(alpha*AB*col_scale + bias)) — residual AFTER the dropout —
   * with keep(row, col) = uniform01(key, row*n + col) >= drop_p, scaled by
   * 1/(1-drop_p), key = drop_seed + (*drop_seed_dev) * 0x9E3779B97F4A7C15
   * (the fpnmt_dropout mask of the dense (m, n) output).                   */
  float drop_p;
  unsigned long long drop_seed;
  const long long* drop_seed_dev;
} fpnmt_gemm_desc;

int fpnmt_gemm(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C,
               const float* col_scale, const float* bias, const void* R,
               fpnmt_stream_t stream);
/* Dense weight gradient C (+)= alpha * A^T B (a_trans = b_trans = 1, fp32 C,
 * accumulate 1 or 2, no epilogue ops; same descriptor as fpnmt_gemm).
 * Replaces Keras' kernel gradient of Dense (transformer.py:117-121, 165-168,
 * 211-214, 357 under tape.gradient, utils/pipeline.py:77). Outside a deferred
 * region it is fpnmt_gemm. Between fpnmt_defer_begin and fpnmt_defer_flush
 * it MAY be queued and run at the flush: A and B must then stay valid and
 * unmodified until fpnmt_defer_flush returns, and C is complete only after
 * it (the result equals immediate mode up to fp32 summation order).        */
int fpnmt_gemm_wgrad(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, fpnmt_stream_t stream);
/* C = (A B) * act_in'(y_in): the backward-data GEMM of a Dense layer whose
 * input y_in is the activated output of the previous Dense (the FFN's
 * ffn2 <- LeakyReLU(ffn1), transformer.py:165-168 / 211-214) with that
 * activation's derivative applied in the epilogue; y_in rows of
 * stride d->ldr. act_in: relu (0/1), relu6 (0/1), leaky_relu (1 / act_alpha,
 * read from the sign of y_in). Plain single GEMMs only (no act, dropout,
 * accumulate, batch).                                                      */
int fpnmt_gemm_act_in(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, const void* y_in,
                      int act_in, float act_alpha, fpnmt_stream_t stream);

/* ---- fused ResNet identity bottleneck (inference) ----------------------
 * keras-resnet bottleneck_2d, blocks 1.. of a stage (reference
 * models/resnet.py:99-112, keras_resnet.blocks.bottleneck_2d with
 * freeze_bn=True) in ONE launch:
 *   y = relu(x + bc + Wc * relu(b3 + W3 (*) pad1(relu(ba + Wa * x))))
 * x, y: NHWC bf16 (n, h, w, c), y must not alias x; wa: OHWI bf16 (cm, 1, 1,
 * c), w3: (cm, 3, 3, cm), wc: (c, 1, 1, cm) with the frozen BN scale folded
 * (fpnmt_weight_prep); ba / b3 / bc: fp32 folded BN shifts. The same values
 * as the three fpnmt_conv2d_fwd calls up to fp32 summation order (the 64 /
 * 128-channel intermediates are rounded to bf16 as the unfused path stores
 * them). Shapes with a kernel: (h, w, c, cm) = (56, 56, 256, 64) and (28, 28,
 * 512, 128) (ResNet-50/101/152 res2 / res3 at 224^2); any other shape returns
 * FPNMT_E_UNSUPPORTED without launching (the caller runs the three convs).
 * Needs the workspace (fpnmt_set_workspace) for its zero page.            */
int fpnmt_bottleneck_fwd(int n, int h, int w, int c, int cm, const void* x, const void* wa, const float* ba,
                         const void* w3, const float* b3, const void* wc, const float* bc, void* y,
                         fpnmt_stream_t stream);

/* ---- implicit-GEMM convolution ----------------------------------------
 * Output size: ho = (h + pad_t + pad_b - r)/stride_h + 1 (same for w).
 * fwd:   y = act((conv(x, w_ohwi)) * scale[k] + bias[k] + residual)
 *        (scale/bias/residual optional; scale carries a frozen BatchNorm)
 * bwd_data: dx (+)= conv_transpose(dz, w) with w_flip = flipped IHWO copy;
 *        supports stride 1 (any r,s, symmetric pads) and 1x1 stride s, pad 0.
 * bwd_filter: dw_hwio (fp32) += col_scale[k] * sum_pixels im2col(x)^T dz
 *        (atomic accumulate, split-K over pixels).                          */
typedef struct fpnmt_conv_desc {
  int n, h, w, c;
  int k, r, s;
  int stride_h, stride_w;
  int pad_t, pad_b, pad_l, pad_r;
  int dtype;
  int act;
  float act_alpha;
} fpnmt_conv_desc;

int fpnmt_conv2d_fwd(const fpnmt_conv_desc* d, const void* x, const void* w_ohwi,
                     const float* scale, const float* bias, const void* residual,
                     void* y, fpnmt_stream_t stream);
int fpnmt_conv2d_bwd_data(const fpnmt_conv_desc* d, const void* dz, const void* w_flip,
                          void* dx, int accumulate, fpnmt_stream_t stream);
int fpnmt_conv2d_bwd_filter(const fpnmt_conv_desc* d, const void* x, const void* dz,
                            const float* col_scale, float* dw_hwio, fpnmt_stream_t stream);
/* bwd_filter and the layer's bias gradient in one call: also db (fp32 [k]) +=
 * sum over pixels of dz (the Keras Conv2D bias gradient, reference
 * models/retinanet.py Conv2D(use_bias=True) layers under utils/pipeline.py:
 * 64-80's tape.gradient). The column sums ride in the LDS-DMA weight-gradient
 * kernel, which streams dz through LDS anyway (per-(split, m-tile, wave row)
 * partial rows summed in a fixed order); other weight-gradient paths run
 * fpnmt_bias_grad's column pass after it. Deterministic either way.         */
int fpnmt_conv2d_bwd_filter_bias(const fpnmt_conv_desc* d, const void* x, const void* dz,
                                 const float* col_scale, float* dw_hwio, float* db,
                                 fpnmt_stream_t stream);
/* bwd_data with the PRODUCING layer's activation backward fused into the
 * epilogue: dx = conv_transpose(dz, w) * act_in'(y_in), y_in = the (n,h,w,c)
 * activation output that was this conv's input x, act_in = FPNMT_ACT_RELU or
 * FPNMT_ACT_RELU6 (0/1 derivatives). Equals fpnmt_conv2d_bwd_data followed by
 * fpnmt_act_bwd(act_in, y_in) bit for bit (a conv chain's backward: the
 * Keras layer pair Conv2D(activation='relu') -> Conv2D). Stride 1 only.    */
int fpnmt_conv2d_bwd_data_act(const fpnmt_conv_desc* d, const void* dz, const void* w_flip,
                              void* dx, const void* y_in, int act_in, fpnmt_stream_t stream);
/* bwd_data into an input gradient that the PRODUCING layer's activation
 * backward is folded into, one consumer at a time (round 6): dx (+)=
 * conv_transpose(dz, w) * act'(y), y = that activation's (n,h,w,c) output
 * (this conv's input x), act = FPNMT_ACT_RELU / RELU6. With accumulate = 1
 * the old dx must already carry the mask (zero where act'(y) = 0: every
 * earlier consumer used this entry); the result is then act'(y) * (old + new),
 * the value fpnmt_conv2d_bwd_data (accumulating) + fpnmt_act_bwd would give
 * (a zero may differ in sign). Stride 1, or 1x1 stride s pad 0 (the rows
 * scattered into the zero-filled / accumulated dx). Replaces the keras-resnet
 * stage output's ReLU backward of tape.gradient (utils/pipeline.py:77) that
 * runs after the stage's consumers (next stage's projection block, FPN
 * lateral conv) have summed their gradients.                              */
int fpnmt_conv2d_bwd_data_mask(const fpnmt_conv_desc* d, const void* dz, const void* w_flip,
                               void* dx, int accumulate, const void* y, int act,
                               fpnmt_stream_t stream);
/* bwd_data with a second gradient of the same input added in the epilogue:
 * dx = conv_transpose(dz, w) + res, res an (n,h,w,c) tensor of the dtype —
 * keras-resnet's identity bottleneck (models/resnet.py: the block input x is
 * conv 2a's input AND the residual of 2c's add), so x's two gradients need no
 * separate add. One rounding of the fp32 sum (bf16); equal to bwd_data then
 * an fp32 add bit for bit in fp32. Stride 1 only.                        */
int fpnmt_conv2d_bwd_data_res(const fpnmt_conv_desc* d, const void* dz, const void* w_flip,
                              void* dx, const void* res, fpnmt_stream_t stream);
/* bwd_data_res followed by the activation backward of the layer that
 * produced the input: dx = (conv_transpose(dz, w) + res) * act_in'(y_in),
 * y_in = the input x itself (the previous bottleneck's ReLU output: its
 * `Activation('relu')` after the Add), act_in = FPNMT_ACT_RELU / RELU6. The
 * mask is applied in the GEMM epilogue where the launch takes the pipe
 * kernel (bf16), else by an in-place pass after it; either way equal to
 * bwd_data_res then fpnmt_act_bwd(act_in, y_in) bit for bit. Stride 1 only. */
int fpnmt_conv2d_bwd_data_res_act(const fpnmt_conv_desc* d, const void* dz, const void* w_flip,
                                  void* dx, const void* res, const void* y_in, int act_in,
                                  fpnmt_stream_t stream);

/* ---- grouped convolution: one shared-weight conv over several inputs ----
 * The retinanet submodels / heads / co-attention convs run ONE weight set
 * over the five pyramid levels (models/retinanet.py:297-301, the
 * `[self.level(f) for f in features]` loop): these launch every level in one
 * grouped implicit GEMM (groups split the output rows for fwd / bwd-data and
 * the pixel reduction for bwd-filter). d gives c, k, r, s, strides, pads,
 * dtype, act; d->n/h/w are ignored (per level below). Levels with no output
 * pixels are skipped (bwd-data zero-fills their dx unless accumulating).
 * bwd-data: stride 1 only.                                                 */
typedef struct fpnmt_conv_level {
  int n, h, w;            /* this level's input shape (n, h, w, c) */
  const void* x;          /* fwd / bwd-filter: input;  bwd-data: dz */
  const void* dz;         /* bwd-filter: output gradient (n, ho, wo, k) */
  const void* residual;   /* fwd: optional (n, ho, wo, k);
                             bwd-data _act: the level's y_in (n, h, w, c) */
  void* y;                /* fwd: output;  bwd-data: dx */
} fpnmt_conv_level;
int fpnmt_conv2d_fwd_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                             const void* w_ohwi, const float* scale, const float* bias,
                             fpnmt_stream_t stream);
int fpnmt_conv2d_bwd_data_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                  const void* w_flip, int accumulate, fpnmt_stream_t stream);
int fpnmt_conv2d_bwd_filter_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                    const float* col_scale, float* dw_hwio, fpnmt_stream_t stream);
/* the grouped form of fpnmt_conv2d_bwd_filter_bias: db += the column sums of
 * every level's dz (a shared head conv's bias gradient over P3..P7)         */
int fpnmt_conv2d_bwd_filter_grouped_bias(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                         const float* col_scale, float* dw_hwio, float* db,
                                         fpnmt_stream_t stream);
/* grouped bwd-data with the producing layer's act' fused (per level y_in in
 * lv[i].residual), as fpnmt_conv2d_bwd_data_act                            */
int fpnmt_conv2d_bwd_data_grouped_act(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                      const void* w_flip, int act_in, fpnmt_stream_t stream);
/* grouped bwd-data with each level's contribution times act'(y_i), y_i in
 * lv[i].residual (the level input's producing activation output; NULL: that
 * level unmasked), accumulating too (then, as fpnmt_conv2d_bwd_data_mask, the
 * old dx must already carry the mask): the heads' first conv over the FPN
 * levels P3..P5 (ReLU convs, retinanet.py:105-136) into their summed gradient. */
int fpnmt_conv2d_bwd_data_grouped_mask(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                       const void* w_flip, int accumulate, int act, fpnmt_stream_t stream);

/* Compute copies of an fp32 HWIO master (r,s,c,k), each scaled per output
 * channel k by scale[k] (frozen BN; NULL = 1):
 *   w_ohwi[k][r][s][c]            (forward B operand, row stride r*s*c)
 *   w_flip[c][R-1-r][S-1-s][k]    (backward-data B operand; row c starts at
 *                                  c*ld_flip, ld_flip = 0 means r*s*k — a
 *                                  larger ld interleaves grouped Dense layers)
 * Either destination may be NULL.                                          */
int fpnmt_weight_prep(const float* w_hwio, int r, int s, int c, int k, const float* scale,
                      int dtype, void* w_ohwi, void* w_flip, long long ld_flip, fpnmt_stream_t stream);
/* The same for a whole model in ONE launch: items_dev is a device array of
 * n_items descriptors; tile_start[i] = sum over j < i of r*s*ceil(c/32)*ceil(k/32)
 * and total_tiles the full sum (each 32x32 (c,k) tile is read once and
 * written to both layouts).                                                */
typedef struct fpnmt_wprep_item {
  const float* w_hwio;
  const float* scale;
  void* w_ohwi;
  void* w_flip;
  int r, s, c, k;
  long long tile_start;
  long long ld_flip;   /* as fpnmt_weight_prep; 0 = r*s*k */
} fpnmt_wprep_item;
int fpnmt_weight_prep_batched(const fpnmt_wprep_item* items_dev, int n_items, long long total_tiles,
                              int dtype, fpnmt_stream_t stream);

/* ---- elementwise / reductions ---------------------------------------- */
/* dz = dy * act'(y)   (y is the activation OUTPUT; relu/leaky sign tests);
 * optionally db[c] += sum_rows dz  (rows x c, c = channel count). With a
 * workspace ws of fpnmt_act_bwd_ws_bytes() the column sums go through
 * per-chunk partials and one atomic per column; ws == NULL falls back to
 * one atomic per column per row chunk (contended: ~10x slower for wide c). */
long long fpnmt_act_bwd_ws_bytes(int dtype, long long rows, int c);
/* drop_p > 0: dz also carries the dropout mask of a fused GEMM epilogue
 * (fpnmt_gemm_desc.drop_*; same seed / key), dz = dy * keep / (1 - drop_p)
 * * act'(y), y then being the pre-dropout activation.                     */
int fpnmt_act_bwd(int dtype, long long rows, int c, int act, float act_alpha,
                  const void* dy, const void* y, void* dz, float* db, float* ws,
                  float drop_p, unsigned long long drop_seed, const long long* drop_seed_dev,
                  fpnmt_stream_t stream);
/* out = cast(in) between f32 / bf16; n elements */
/* db += column sums of dy (rows x c): a bias gradient (Dense / Conv2D
 * use_bias with a linear output, or after a fused act' epilogue). Equals
 * fpnmt_act_bwd(act NONE, dz = dy) bit for bit. Between fpnmt_defer_begin and
 * fpnmt_defer_flush the launch is QUEUED (batched with the other queued
 * bias gradients at the flush): dy must stay allocated and unmodified until
 * the flush.                                                               */
int fpnmt_bias_grad(int dtype, long long rows, int c, const void* dy, float* db, fpnmt_stream_t stream);
int fpnmt_cast(int in_dtype, int out_dtype, long long n, const void* in, void* out,
               fpnmt_stream_t stream);
/* y = x * keep / (1-p), keep = u(key, i) >= p with key = seed + *seed_dev
 * (seed_dev: optional device int64, e.g. the optimizer step, so a replayed
 * hipGraph draws a fresh mask every step); in place allowed.              */
int fpnmt_dropout(int dtype, long long n, float p, unsigned long long seed,
                  const long long* seed_dev, const void* x, void* y, fpnmt_stream_t stream);
/* out = a + b (n elements) — residual join of two gradient branches */
int fpnmt_add(int dtype, long long n, const void* a, const void* b, void* out,
              fpnmt_stream_t stream);

/* ---- pooling ----------------------------------------------------------
 * Max pool NHWC, window (kh,kw), stride (sh,sw), pads (pt,pl) — padded taps
 * never win (TF "same" pads with -inf); output size (ho,wo) given.
 * argmax (optional, n*ho*wo*c bytes): window tap r*kw+q of the first max.  */
int fpnmt_maxpool2d_fwd(int dtype, int n, int h, int w, int c, int kh, int kw, int sh, int sw,
                        int pt, int pl, int ho, int wo, const void* x, void* y,
                        uint8_t* argmax, fpnmt_stream_t stream);
/* dx = routed dy (the first max in window order gets the gradient; every dx
 * element is written, gather form, no atomics). Routing comes from argmax
 * when non-null (x may then be null), else is recomputed from x.           */
int fpnmt_maxpool2d_bwd(int dtype, int n, int h, int w, int c, int kh, int kw, int sh, int sw,
                        int pt, int pl, int ho, int wo, const void* x, const uint8_t* argmax,
                        const void* dy, void* dx, fpnmt_stream_t stream);
/* fpnmt_maxpool2d_bwd (argmax routing) times the PRODUCER's activation
 * derivative: dx = routed dy * act'(x), x = the pool's input (that
 * activation's output), act = FPNMT_ACT_RELU / RELU6, or
 * FPNMT_ACT_LEAKY (slope alpha) when the windows do not overlap (kh <= sh,
 * kw <= sw: one rounding, as the separate pass). Equals fpnmt_maxpool2d_bwd
 * + fpnmt_act_bwd(act, x) (a zero may differ in sign): the ResNet stem's
 * ReLU under its max pool (models/resnet.py conv1 -> pool1), the feature
 * extractor's LeakyReLU coatt conv under MaxPooling2D (retinanet.py:292-293),
 * in tape.gradient (utils/pipeline.py:77).                                */
int fpnmt_maxpool2d_bwd_act(int dtype, int n, int h, int w, int c, int kh, int kw, int sh, int sw,
                            int pt, int pl, int ho, int wo, const uint8_t* argmax, const void* dy,
                            const void* x, int act, float alpha, void* dx, fpnmt_stream_t stream);

/* ---- FPN top-down pathway (one sweep) ----------------------------------
 * P4m = lat4 + up(lat5 -> h4 x w4);  P3m = lat3 + up(P4m -> h3 x w3)
 * up = TF2 nearest resize (half-pixel centres): src = min(floor((d+.5)*in/out), in-1)
 * All (n, h_i, w_i, c). bwd: d_lat5 (+)= down(d_P4 + down(d_P3)),
 * d_lat4 = d_P4m + down(d_P3m); d_lat3 = d_P3m (caller aliases, no copy). */
int fpnmt_fpn_topdown_fwd(int dtype, int n, int c, int h5, int w5, int h4, int w4, int h3,
                          int w3, const void* lat5, const void* lat4, const void* lat3,
                          void* p4m, void* p3m, fpnmt_stream_t stream);
int fpnmt_fpn_topdown_bwd(int dtype, int n, int c, int h5, int w5, int h4, int w4, int h3,
                          int w3, const void* d_p4m, const void* d_p3m, void* d_lat4,
                          void* d_lat5, int accumulate_lat5, fpnmt_stream_t stream);

/* ---- co-attention spatial softmax (models/coattention.py:13-32) --------
 * a = softmax over the hw positions of score (n, hw);  ctx = a (x) hs (n, hw, c)
 * fwd also writes a (fp32, n*hw) for the backward.                        */
int fpnmt_spatial_softmax_fwd(int dtype, int n, int hw, int c, const void* score, const void* hs,
                              void* ctx, float* a_out, fpnmt_stream_t stream);
int fpnmt_spatial_softmax_bwd(int dtype, int n, int hw, int c, const float* a, const void* hs,
                              const void* d_ctx, void* d_score, void* d_hs, double* ws,
                              fpnmt_stream_t stream); /* ws: n*hw fp64 (da, kept in fp64) */

/* ---- attention (models/transformer.py:70-104) ---------------------------
 * q: (B, Lq, H*D) rows of stride ldq, head h at column h*D; k, v likewise.
 * mask (optional, fp32): additive mask * -1e9, element (b,h,i,j) at
 *   mask[b*m_sb + h*m_sh + i*m_si + j*m_sj] (strides may be 0 = broadcast).
 * out: (B, Lq, H*D) stride ldo. weights (B,H,Lq,Lk) in dtype, row stride ldw >= lk
 * (padded to a multiple of 8; pad columns are written as 0). ws: fp32
 * scratch of fpnmt_attention_ws_bytes().                                   */
typedef struct fpnmt_attn_desc {
  int b, h, lq, lk, d;
  int dtype;
  long long ldq, ldk, ldv, ldo, ldw;
  float scale;
  long long m_sb, m_sh, m_si, m_sj;
} fpnmt_attn_desc;
size_t fpnmt_attention_ws_bytes(const fpnmt_attn_desc* d);
int fpnmt_attention_fwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v,
                        const float* mask, void* out, void* weights, void* ws,
                        fpnmt_stream_t stream);
/* Backward: given dO (ldo), the forward's weights P and the inputs, write dq,
 * dk, dv (same strides as q,k,v). ws as above.                             */
int fpnmt_attention_bwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v,
                        const void* weights, const void* d_out, void* dq, void* dk, void* dv,
                        void* ws, fpnmt_stream_t stream);
/* The n <= FPNMT_MAX_VIEWS per-view attentions of one EncoderLayer
 * (transformer.py:184-190: the baseline's query row against each view's
 * keys), each with its own descriptor / pointers (table entry i): the
 * results of n fpnmt_attention_fwd / _bwd calls up to fp32 summation order
 * (the grouped launch runs every view on the multi-wave one-query body; the
 * single-view call sends views with fewer than 128 keys to a one-wave body,
 * so short views such as P6 / P7 may differ in the last bits). Views sharing
 * b, h and scale that are all one-query bf16, D = 64, without a mask run as
 * ONE launch; otherwise the calls are made one by one (ws[i] as above).    */
#define FPNMT_MAX_VIEWS 4
int fpnmt_attention_fwd_views(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                              const void* const* v, const float* const* mask, void* const* out,
                              void* const* weights, void* const* ws, fpnmt_stream_t stream);
int fpnmt_attention_bwd_views(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                              const void* const* v, const void* const* weights, const void* const* d_out,
                              void* const* dq, void* const* dk, void* const* dv, void* const* ws,
                              fpnmt_stream_t stream);

/* ---- multi-view encoder output (reference models/transformer.py
 * EncoderLayer.call :184-190: out = baseline + sum_i Dropout(mha_i.dense(o_i)))
 * fwd: out (m, n) = R + sum_{i < nseg} dropout_i(A_i W_i + bias[i*n ..]) with
 *   A = the views' attention outputs side by side (m, nseg*k; row stride lda,
 *   view i at column i*k), W = the views' Dense kernels as ONE stacked
 *   (nseg*n, k) k-contiguous operand (rows i*n .. i*n+n-1 = view i's OHWI
 *   copy), bias nseg*n fp32 (optional), R (m, n; optional). Dropout of view i
 *   at (row, col): keep = uniform01(key, row*(nseg*n) + i*n + col) >= drop_p,
 *   scaled by 1/(1-drop_p), key as fpnmt_gemm_desc's — the fpnmt_dropout mask
 *   of the virtual (m, nseg*n) matrix of the views' pre-sum outputs.
 *   nseg == 4 (NUM_OF_PYRAMIDS - 1); k % 16 == 0.
 * bwd_dz: dz (m, nseg*n) = that mask applied to dy broadcast over the views;
 *   db[nseg*n] += dz's column sums (fixed order; optional). The views' dA and
 *   dW are then batched fpnmt_gemm launches over dz.                        */
int fpnmt_view_proj_fwd(int dtype, int m, int n, int k, int nseg, const void* A, long long lda, const void* W,
                        const float* bias, const void* R, long long ldr, void* out, long long ldo, float drop_p,
                        unsigned long long seed, const long long* seed_dev, fpnmt_stream_t stream);
int fpnmt_view_proj_bwd_dz(int dtype, int m, int n, int nseg, const void* dy, long long lddy, void* dz, float* db,
                           float drop_p, unsigned long long seed, const long long* seed_dev,
                           fpnmt_stream_t stream);

/* ---- LayerNorm (eps, last axis, affine), optional fused residual --------
 * x' = x + res (res optional); y = (x'-mu)/sqrt(var+eps)*gamma + beta + pe[row % pe_rows]
 * (pe optional: positional encoding added after the norm, Encoder path).
 * Saves mean/rstd (fp32, rows) for the backward.                           */
int fpnmt_layernorm_fwd(int dtype, long long rows, int d, float eps, const void* x,
                        const void* res, const float* gamma, const float* beta, const float* pe,
                        int pe_rows, void* y, float* mean, float* rstd, fpnmt_stream_t stream);
/* dx = LN'(dy) (x' recomputed from x [+ res]); dgamma/dbeta (fp32) += column
 * sums (per-block partials reduced in block order: deterministic). dx is also
 * the gradient of res.                                                      */
int fpnmt_layernorm_bwd(int dtype, long long rows, int d, const void* x, const void* res,
                        const float* gamma, const float* mean, const float* rstd, const void* dy,
                        void* dx, float* dgamma, float* dbeta, fpnmt_stream_t stream);
/* The Encoder's view LayerNorms (transformer.py:279-292: per view, the shared
 * LayerNormalization, + pe[:L_i], dropout) as ONE launch per pass. View i:
 * x (rows, d) -> y = dropout(LN(x) + pe[row % pe_rows]) with the mask
 * fpnmt_dropout(seed_i) would draw on the (rows, d) output (drop_p 0: none);
 * mean / rstd saved per row. Backward: dx of view i from its dy, the dropout
 * mask applied to dy first; dgamma / dbeta (+=) summed view by view, each
 * view's rows in the order of its own fpnmt_layernorm_bwd (same results).  */
#define FPNMT_MAX_LN_VIEWS 8
typedef struct fpnmt_ln_view {
  const void* x;     /* fwd / bwd: the view's input rows                    */
  void* y;           /* fwd: output;  bwd: dx                                */
  const void* dy;    /* bwd: the gradient of y                               */
  float* mean;
  float* rstd;
  long long rows;
  int pe_rows;       /* fwd with pe: the view's positions (L_i)              */
  unsigned long long seed;
} fpnmt_ln_view;
int fpnmt_layernorm_views_fwd(int dtype, int n, int d, float eps, const fpnmt_ln_view* views,
                              const float* gamma, const float* beta, const float* pe, float drop_p,
                              const long long* seed_dev, fpnmt_stream_t stream);
int fpnmt_layernorm_views_bwd(int dtype, int n, int d, const fpnmt_ln_view* views, const float* gamma,
                              float drop_p, const long long* seed_dev, float* dgamma, float* dbeta,
                              fpnmt_stream_t stream);
/* fpnmt_layernorm_bwd + the backward of the dropout fused into the Dense
 * that produced x (x = dropout(A W + b), transformer.py:232-242 / :190-194):
 * also dz = keep(row * d + col) ? dx / (1 - drop_p) : 0 with the forward
 * GEMM epilogue's mask (drop_seed + *drop_seed_dev * golden), computed from
 * the stored dx exactly as fpnmt_act_bwd would — one launch instead of two.
 * dz (rows x d) feeds that Dense's bias / weight / data gradients.          */
int fpnmt_layernorm_bwd_drop(int dtype, long long rows, int d, const void* x, const void* res,
                             const float* gamma, const float* mean, const float* rstd, const void* dy,
                             void* dx, float* dgamma, float* dbeta, float drop_p,
                             unsigned long long drop_seed, const long long* drop_seed_dev, void* dz,
                             fpnmt_stream_t stream);

/* ---- decoder embedding + positional encoding ---------------------------
 * y[b,t,:] = E[tok[b,t],:] + pe[t,:]   (no sqrt(d) scale, transformer.py:326-329)
 * bwd: dE[tok] += dy rows, each id's rows summed in position order (no
 * atomics: deterministic); sumsq += sum of squared row grads (TF
 * IndexedSlices norm for clip_by_norm, duplicates counted), in fixed order.
 * Uses the fpnmt workspace (fpnmt_set_workspace) as scratch.             */
int fpnmt_embed_posenc_fwd(int dtype, int b, int t, int d, const int32_t* tok, const float* emb,
                           const float* pe, void* y, fpnmt_stream_t stream);
int fpnmt_embed_posenc_bwd(int dtype, int b, int t, int d, const int32_t* tok, const void* dy,
                           float* d_emb, float* sumsq, fpnmt_stream_t stream);
/* The same with the decoder's Dropout after the embedding (transformer.py:
 * 331) fused: y = dropout(E[tok] + pe) with fpnmt_dropout(seed)'s mask on
 * the (b*t, d) output; the backward applies that mask to dy first.        */
int fpnmt_embed_posenc_fwd_drop(int dtype, int b, int t, int d, const int32_t* tok, const float* emb,
                                const float* pe, void* y, float drop_p, unsigned long long seed,
                                const long long* seed_dev, fpnmt_stream_t stream);
int fpnmt_embed_posenc_bwd_drop(int dtype, int b, int t, int d, const int32_t* tok, const void* dy,
                                float* d_emb, float* sumsq, float drop_p, unsigned long long seed,
                                const long long* seed_dev, fpnmt_stream_t stream);

/* ---- train-step targets (utils/pipeline.py:66-69, transformer.py:42-67)
 * From padded captions tok (b, t_full) of int64 (tok_bytes 8) or int32 (4)
 * ids, row stride ld_tok elements, in one launch: tar_inp = tok[:, :-1] and
 * tar_real = tok[:, 1:] (int32, (b, t_full-1)) and the decoder mask (b, 1,
 * t, t) fp32 = max(padding mask of tar_inp, look-ahead mask): 1 where
 * tar_inp[b, j] == 0 or j > i.                                             */
int fpnmt_decoder_targets(int b, int t_full, const void* tok, int tok_bytes, long long ld_tok, int32_t* tar_inp,
                          int32_t* tar_real, float* mask, fpnmt_stream_t stream);

/* ---- masked sparse cross-entropy (utils/pipeline.py:50-57) -------------
 * loss = mean over ALL rows of ce(row) * (label != 0); writes loss (fp32
 * scalar, overwritten) and dlogits = d loss / d logits * dloss_scale.     */
int fpnmt_xent_fwd_bwd(int dtype, long long rows, int v, const float* logits, long long ld,
                       const int32_t* labels, float* loss, void* dlogits, long long ldd,
                       float dloss_scale, fpnmt_stream_t stream);

/* ---- optimizer: Keras Adam(amsgrad) + per-tensor clip_by_norm ----------
 * Tensors are segments [off[i], off[i+1]) of flat fp32 arrays, processed in
 * blocks of block_elems that never cross a segment: block b covers
 * [blk_start[b], min(blk_start[b]+block_elems, off[blk_seg[b]+1])).
 * seg_flags[i]: bit0 = sumsq[i] is supplied by the caller (TF IndexedSlices
 * norm of the embedding, fpnmt_embed_posenc_bwd), bit1 = apply the Keras
 * sparse-path update formula (m*b1 + (1-b1)g) instead of the fused dense
 * kernel's (m += (g-m)(1-b1)).
 * fpnmt_grad_sumsq writes blk_part[b] = sum(g^2) over block b (scaled
 * gradient g*grad_scale) for segments without bit0; fpnmt_amsgrad_step sums
 * segment i's partials blk_part[seg_blk0[i] .. seg_blk0[i+1]) in block order
 * (deterministic: no atomics), or takes sumsq[i] for bit0 segments. With
 * clipnorm <= 0 no norm is read (blk_part / seg_blk0 may be null).
 * step: device int64 = Keras `iterations` (0-based), incremented on device.
 * lr = d_model^-0.5 * min(rsqrt(step)/max((step-warm)*mult/(2*warm),1), step*warm_pow)
 * with warm_pow = warm^-1.5 (CustomSchedule, utils/utils.py:45-50); when
 * sched_d_model <= 0 the constant const_lr is used.                       */
int fpnmt_grad_sumsq(int nblocks, const int32_t* blk_seg, const long long* blk_start,
                     int block_elems, const long long* off, const int32_t* seg_flags,
                     const float* g, float grad_scale, float* blk_part, fpnmt_stream_t stream);
typedef struct fpnmt_adam_desc {
  float beta1, beta2, eps, clipnorm;
  float sched_d_model, sched_warmup, sched_mult, sched_warm_pow;
  float const_lr;
  float grad_scale; /* gradients are used as g*grad_scale (1/world after a SUM all-reduce);
                       caller-supplied (bit0) sumsq entries are scaled by grad_scale^2 */
} fpnmt_adam_desc;
int fpnmt_amsgrad_step(const fpnmt_adam_desc* d, int nblocks, const int32_t* blk_seg,
                       const long long* blk_start, int block_elems, const long long* off,
                       const int32_t* seg_flags, float* param, const float* grad, float* m,
                       float* v, float* vhat, const float* sumsq, const float* blk_part,
                       const int32_t* seg_blk0, long long* step, fpnmt_stream_t stream);
/* fpnmt_amsgrad_step_prep: the same step, and for every segment whose
 * preps[seg].ohwi is non-null (a conv / dense kernel in HWIO (r,s,c,k) order,
 * k a power of two <= block_elems dividing it) the bf16 compute copies of
 * the updated weights are written from the same pass, as
 * fpnmt_weight_prep(dtype FPNMT_BF16) would write them from the new masters:
 * ohwi[k][r][s][c] and flip[c*ld_flip + ((r-1-i)*s + (s-1-j))*k + kk], both
 * scaled by scale[kk] when scale is non-null. preps may be null (plain step).
 * Replaces the separate refresh pass after apply_gradients (utils/pipeline.py:78). */
typedef struct fpnmt_seg_prep {
  void* ohwi;
  void* flip;
  const float* scale;
  int r, s, c, k;
  long long ld_flip; /* 0 = r*s*k */
  uint32_t c_magic, c_shift; /* c as a fast divisor: q / c = (hi32(q*magic) + q) >> shift */
} fpnmt_seg_prep;
int fpnmt_amsgrad_step_prep(const fpnmt_adam_desc* d, int nblocks, const int32_t* blk_seg,
                            const long long* blk_start, int block_elems, const long long* off,
                            const int32_t* seg_flags, float* param, const float* grad, float* m,
                            float* v, float* vhat, const float* sumsq, const float* blk_part,
                            const int32_t* seg_blk0, long long* step, const fpnmt_seg_prep* preps,
                            fpnmt_stream_t stream);
/* Block-range forms: the blocks [blk_first, blk_first + nblocks) of the same
 * tables (all other pointers as above: blk_seg / blk_start / blk_part /
 * seg_blk0 index the WHOLE arena's blocks), for a step whose segments are
 * updated in parts, e.g. the transformer's while the feature extractor's
 * backward still runs. The range must hold whole segments. inc_step = 0
 * leaves `step` as it is (every part of one step must read the same value;
 * the last part increments it). max_grid > 0: at most that many workgroups,
 * each striding over the range (a small footprint beside other work); 0:
 * one workgroup per block. Results do not depend on max_grid.            */
int fpnmt_grad_sumsq_part(int blk_first, int nblocks, int max_grid, const int32_t* blk_seg,
                          const long long* blk_start, int block_elems, const long long* off,
                          const int32_t* seg_flags, const float* g, float grad_scale, float* blk_part,
                          fpnmt_stream_t stream);
int fpnmt_amsgrad_step_part(const fpnmt_adam_desc* d, int blk_first, int nblocks, int inc_step, int max_grid,
                            const int32_t* blk_seg, const long long* blk_start, int block_elems,
                            const long long* off, const int32_t* seg_flags, float* param,
                            const float* grad, float* m, float* v, float* vhat, const float* sumsq,
                            const float* blk_part, const int32_t* seg_blk0, long long* step,
                            const fpnmt_seg_prep* preps, fpnmt_stream_t stream);

/* ---- batched beam decode (BASELINE C5; utils/pipeline.py:82-154) --------
 * fpnmt_decode_attention: softmax(q k^T * scale) v for ONE query position per
 * row (the last position of the reference's full-prefix recompute; its
 * look-ahead mask row keeps every position <= t). Row r, head h:
 *   q at q + r*ldq + h*depth; key / value of position j at
 *   kv + R*row_stride + j*pos_stride + {k_off | v_off} + h*depth, where
 *   R = src ? src[r*src_ld + j] : r / row_div
 * (src: the beam's cache-row table, so beams share history without copies;
 * row_div: rows per encoder output for the cross-attention). heads <= 8,
 * depth <= 64. out at out + r*ldo + h*depth. Attention weights are not
 * materialised on this path.
 * fpnmt_beam_step: per image (beam_n consecutive rows): p = softmax(logits
 * row), candidates p * beam_prob over beam_n x vocab, top beam_n in
 * tf.math.top_k order (value desc, lower flat index first); new beams take
 * parent = flat / vocab, token = flat % vocab:
 *   hist_out[r][0..t] = hist_in[parent][0..t], hist_out[r][t+1] = token,
 *   src_out[r][0..t] = src_in[parent][0..t], src_out[r][t+1] = r,
 *   tok_out[r] = token, beam_prob[r] = candidate value.
 * While status[img] == 0 the best beam (first argmax of the new
 * probabilities) is copied to result[img] (tokens after <start>, without a
 * final <end>), result_len[img] set, and status[img] = 1 once it ends.     */
int fpnmt_decode_attention(int dtype, int rows, int heads, int depth, int lk, float scale, const void* q,
                           long long ldq, const void* kv, long long row_stride, long long pos_stride,
                           long long k_off, long long v_off, const int32_t* src, int src_ld, int row_div,
                           void* out, long long ldo, fpnmt_stream_t stream);
int fpnmt_beam_step(int n_images, int beam_n, int vocab, const float* logits, long long ldl, float* beam_prob,
                    const int32_t* hist_in, int32_t* hist_out, int hist_ld, int t, const int32_t* src_in,
                    int32_t* src_out, int src_ld, int end_token, int32_t* tok_out, int32_t* result, int result_ld,
                    int32_t* result_len, int32_t* status, fpnmt_stream_t stream);

/* ---- MobileNetV2 backbone (models/mobilenet.py:43-72 ->
 * keras MobileNetV2(alpha=1.0), models/retinanet.py:274) -------------------
 * BatchNormalization(epsilon, momentum) in training mode over the channels
 * of (rows, c) NHWC activations, c % 8 == 0:
 *   fpnmt_bn_stats: batch mean / biased variance (fp32) into mean, var;
 *     when moving_mean / moving_var are given they move toward the batch
 *     statistics: m = m*momentum + mean*(1-momentum), v likewise with the
 *     Bessel-corrected variance (Keras fused batch norm).
 *   fpnmt_bn_apply: y = act((x - mean) * rsqrt(var + eps) * gamma + beta)
 *     [+ residual]; act in {NONE, RELU, RELU6}. Inference passes the moving
 *     statistics as mean / var.
 *   fpnmt_bn_bwd: g = dy * act'(y); dbeta += sum g, dgamma += sum g*xhat;
 *     dx = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) (training-mode BN).
 * DepthwiseConv2D (kh, kw <= 3, no bias), weights in the Keras (kh, kw, C, 1)
 * order = (kh, kw, C) fp32; 4 independent pads (TF / correct_pad):
 *   fwd y (n, ho, wo, c); bwd_data dx (n, h, w, c) overwritten;
 *   bwd_filter dw += sum over pixels.
 * Every reduction is per-block partials summed in a fixed order through the
 * fpnmt workspace (deterministic).                                         */
int fpnmt_bn_stats(int dtype, long long rows, int c, const void* x, float* mean, float* var,
                   float* moving_mean, float* moving_var, float momentum, fpnmt_stream_t stream);
int fpnmt_bn_apply(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                   const float* gamma, const float* beta, float eps, int act, const void* residual, void* y,
                   fpnmt_stream_t stream);
int fpnmt_bn_bwd(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                 const float* gamma, float eps, int act, const void* y, const void* dy, void* dx,
                 float* dgamma, float* dbeta, fpnmt_stream_t stream);
/* Cross-replica (sync) BatchNorm under data parallelism, the statistics of
 * the GLOBAL batch as the reference computes them on one device
 * (models/mobilenet.py:61 Keras BatchNormalization): each rank
 * reduces its rows to fp64 sums (2c + 1 doubles: [0, c) and [c, 2c) the
 * per-channel sums, [2c] the row count), the caller SUM-all-reduces them
 * over the ranks (RCCL / gloo), then
 *   fpnmt_bn_stats_sums: sum x, sum x^2 of this rank's rows;
 *   fpnmt_bn_stats_finalize: mean / biased variance (and the moving
 *     averages) from the all-reduced sums;
 *   fpnmt_bn_bwd_sums: sum g, sum g*xhat of this rank's rows
 *     (g = dy * act'(y)); the rank's own parts are added to dgamma / dbeta;
 *   fpnmt_bn_bwd_dx: dx from the all-reduced backward sums; the global row
 *     count is read on the device from sums[2c] (the all-reduced count, so
 *     ranks whose shards differ in size normalise by the same total).
 * With one rank the sequence equals fpnmt_bn_stats / fpnmt_bn_bwd. */
int fpnmt_bn_stats_sums(int dtype, long long rows, int c, const void* x, double* sums, fpnmt_stream_t stream);
int fpnmt_bn_stats_finalize(int c, const double* sums, float* mean, float* var, float* moving_mean,
                            float* moving_var, float momentum, fpnmt_stream_t stream);
int fpnmt_bn_bwd_sums(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                      float eps, int act, const void* y, const void* dy, double* sums, float* dgamma,
                      float* dbeta, fpnmt_stream_t stream);
int fpnmt_bn_bwd_dx(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                    const float* gamma, float eps, int act, const void* y, const void* dy, const double* sums,
                    void* dx, fpnmt_stream_t stream);
int fpnmt_depthwise_fwd(int dtype, int n, int h, int w, int c, int kh, int kw, int stride, int pad_t,
                        int pad_b, int pad_l, int pad_r, const void* x, const float* w_hwc, void* y,
                        fpnmt_stream_t stream);
int fpnmt_depthwise_bwd_data(int dtype, int n, int h, int w, int c, int kh, int kw, int stride, int pad_t,
                             int pad_b, int pad_l, int pad_r, const void* dy, const float* w_hwc, void* dx,
                             fpnmt_stream_t stream);
int fpnmt_depthwise_bwd_filter(int dtype, int n, int h, int w, int c, int kh, int kw, int stride, int pad_t,
                               int pad_b, int pad_l, int pad_r, const void* x, const void* dy, float* dw_hwc,
                               fpnmt_stream_t stream);

/* ---- input pipeline (dataset.py:19-26 load_image) --------
 * Replaces tf.image.resize(img, (out_h, out_w)) (bilinear, TF2 half-pixel
 * centres, no antialias) followed by mobilenet_v2.preprocess_input
 * (x / 127.5 - 1; pass div = 127.5, sub = 1) for a batch of decoded RGB
 * uint8 images of any sizes, in one launch:
 *   out[i] (out_h, out_w, 3) NHWC = resize(image i) / div - sub,
 * image i = the h*w*3 bytes at pixels + items_dev[i].offset (rows of w RGB
 * triples, as tf.image.decode_jpeg(channels=3) returns them). items_dev is a
 * device array of n items; max_w >= every item's w sizes the LDS row window
 * (a wider row is read from global memory instead). pixel_bytes = the
 * packed buffer's size (no read past it). fp32 arithmetic bit-identical to
 * TF's formula (no FMA contraction, IEEE divide); bf16 output is the RNE
 * rounding of that fp32 value. Items with h or w <= 0 produce zeros.      */
typedef struct fpnmt_image_item {
  long long offset; /* byte offset of pixel (0, 0) in the packed buffer */
  int h, w;         /* decoded rows / columns */
} fpnmt_image_item;
int fpnmt_image_resize_normalize(const fpnmt_image_item* items_dev, int n, const uint8_t* pixels,
                                 long long pixel_bytes, int max_w, int out_h, int out_w, float div, float sub,
                                 int dtype, void* out, fpnmt_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FPNMT_H */
