// Batched beam decode (BASELINE config C5; reference utils/pipeline.py:82-154):
// one query row per beam, a K/V cache that is never moved, and a per-beam
// table of cache rows.
//
//  * decode_attn_kernel: scaled-dot-product attention of ONE query position
//    per row (transformer.py:70-104 with Lq = 1; the look-ahead mask of the
//    last position is all-keep) over Lk cached positions. The key/value of
//    position j of row r live in cache row src[r][j] (the beam whose history
//    the row inherited when it was written), so re-ranking beams never copies
//    the cache: it rewrites the small int table (vLLM-style block table, one
//    entry per position). Cross-attention uses row r / row_div instead (one
//    encoder output per image, shared by its beams: the reference's tf.tile).
//  * beam_step_kernel: per image, softmax of each beam's logits, candidates
//    p * beam_prob over beam_n x V, top-k (k = beam_n) in tf.math.top_k order
//    (value desc, then lower flat index), the new histories / cache tables of
//    the image's beams, the best beam (argmax of the new probabilities, first
//    max) and the result capture / stop flag (`beam_result[-1] == end`).
#include "common.h"
#include <initializer_list>

namespace fpnmt {

constexpr int DEC_MAX_D = 64;  // head depth handled per wave (d_model / heads = 64)

template <typename T>
__global__ __launch_bounds__(512) void decode_attn_kernel(int rows, int heads, int depth, int lk, float scale,
                                                          const T* __restrict__ q, long long ldq,
                                                          const T* __restrict__ kv, long long row_stride,
                                                          long long pos_stride, long long k_off, long long v_off,
                                                          const int32_t* __restrict__ src, int src_ld, int row_div,
                                                          T* __restrict__ out, long long ldo) {
  const int r = blockIdx.x;
  const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (r >= rows || h >= heads) return;
  __shared__ float qs[8][DEC_MAX_D];
  __shared__ float ps[8][64];
  __shared__ long long rs[8][64];  // cache row of each position of the chunk (src table or own)
  const T* qrow = q + (long long)r * ldq + h * depth;
  if (lane < depth) qs[h][lane] = to_f32(qrow[lane]) * scale;
  __syncthreads();
  const int own = r / row_div;
  // 16-B key loads: bf16, depth % 8 == 0 and 16-B aligned rows / offsets
  const bool vec16 = sizeof(T) == 2 && depth % 8 == 0 && (((uintptr_t)kv | (row_stride | pos_stride | k_off) * 2) & 15) == 0;
  float m = -INFINITY, l = 0.f, o = 0.f;  // online softmax over chunks of 64 positions
  for (int j0 = 0; j0 < lk; j0 += 64) {
    const int j = j0 + lane;
    float s = -INFINITY;
    if (j < lk) {
      const long long kr = src ? (long long)src[(long long)r * src_ld + j] : own;
      rs[h][lane] = kr;
      const T* krow = kv + kr * row_stride + (long long)j * pos_stride + k_off + h * depth;
      float acc = 0.f;
      if (vec16) {
        for (int d = 0; d < depth; d += 8) {
          const bf16x8 kk = *(const bf16x8*)(krow + d);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc += qs[h][d + e] * (float)kk[e];
        }
      } else {
        for (int d = 0; d < depth; ++d) acc += qs[h][d] * to_f32(krow[d]);
      }
      s = acc;
    }
    const float cm = wave_max(s);
    const float mn = fmaxf(m, cm);
    const float p = j < lk ? expf(s - mn) : 0.f;
    const float corr = expf(m - mn);  // m = -inf on the first chunk: exp(-inf) = 0
    l = l * corr + wave_sum(p);
    o = o * corr;
    ps[h][lane] = p;
    __syncthreads();
    const int n = min(64, lk - j0);
    if (lane < depth) {
      // row indices from LDS (written with the scores) and eight value loads
      // issued before their FMAs: the loop no longer waits out a src-table
      // load plus a value load per position (round 6, profiles/r06/c5_*.txt);
      // the FMAs keep the position order
      const T* vb = kv + v_off + h * depth + lane;
      int jj = 0;
      for (; jj + 8 <= n; jj += 8) {
        float vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          vv[u] = to_f32(vb[rs[h][jj + u] * row_stride + (long long)(j0 + jj + u) * pos_stride]);
#pragma unroll
        for (int u = 0; u < 8; ++u) o += ps[h][jj + u] * vv[u];
      }
      for (; jj < n; ++jj) o += ps[h][jj] * to_f32(vb[rs[h][jj] * row_stride + (long long)(j0 + jj) * pos_stride]);
    }
    __syncthreads();
    m = mn;
  }
  if (lane < depth) out[(long long)r * ldo + h * depth + lane] = from_f32<T>(lk > 0 ? o / l : 0.f);
}

// bf16, depth 64, 16-B aligned cache rows (the decoder's shapes): one
// 64-lane block per (row, head), lane = position-group pg (lane >> 3) x
// channel-group cg (lane & 7). The lane keeps its 8 query channels in
// registers (bf16 pairs: scores by v_dot2, fp32 accumulate, scaled after the
// channel reduction); per chunk of 8 * PS positions the chunk's cache rows come
// in with one coalesced src load (staged through LDS), then every lane issues
// its PS key and PS value loads (16 B: positions pg*PS + i, channels
// cg*8..+7) before using any. Scores reduce over the 8 channel lanes by DPP
// (quad_perm, half-row mirror: no LDS round trips); softmax statistics over pg online across
// chunks; values accumulate per lane in position order and are summed over pg
// through LDS in pg order at the end (deterministic). Replaces, for these
// shapes, the lane-per-position kernel's per-position load latencies (a depth
// loop of dependent key loads, one 2-B value load per position): C5 self-
// attention at lk 32 48.4 -> 17.2 us, cross-attention 27.3 -> 8.5 us
// (tools/dec_attn_bench.hip, profiles/r06/dec_attn.txt).
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8_cg(float a) {  // over lanes (pg, 0..7), every lane gets the sum
  a += dpp_f<0xB1>(a);   // quad_perm [1,0,3,2]: xor 1
  a += dpp_f<0x4E>(a);   // quad_perm [2,3,0,1]: xor 2
  return a + dpp_f<0x141>(a);  // row_half_mirror: the other quad of the 8
}

// PS positions per lane per chunk (8 * PS per chunk); LATE_V: the value loads
// issued after the scores, into the key registers (fewer VGPRs, one more
// latency per chunk); MINW: waves per SIMD asked of the register allocator.
template <int PS, bool LATE_V, int MINW>
__global__ __launch_bounds__(64, MINW) void decode_attn_v_kernel(int rows, int heads, int lk, float scale,
                                                                 const bf16* __restrict__ q, long long ldq,
                                                                 const bf16* __restrict__ kv, long long row_stride,
                                                                 long long pos_stride, long long k_off,
                                                                 long long v_off, const int32_t* __restrict__ src,
                                                                 int src_ld, int row_div, bf16* __restrict__ out,
                                                                 long long ldo) {
  constexpr int D = 64, CH = 8 * PS;
  const int r = blockIdx.x / heads, h = blockIdx.x - r * heads;
  if (r >= rows) return;
  const int lane = threadIdx.x, pg = lane >> 3, cg = lane & 7;
  __shared__ int rsh[CH];
  __shared__ float red[8][D + 4];
  // the query's 8 channels stay bf16 pairs: scores by v_dot2 (fp32 accumulate),
  // scaled after the channel reduction
  const bf16x8 qq = *(const bf16x8*)(q + (long long)r * ldq + h * D + cg * 8);
  const int own = r / row_div;
  const bf16* kb = kv + k_off + h * D + cg * 8;
  const long long kvd = v_off - k_off;
  float m = -INFINITY, l = 0.f;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.f;
  for (int j0 = 0; j0 < lk; j0 += CH) {
    int kr[PS];
    if (src) {
      __syncthreads();  // the previous chunk's reads of rsh are done
      if (lane < CH) rsh[lane] = j0 + lane < lk ? src[(long long)r * src_ld + j0 + lane] : own;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < PS; ++i) kr[i] = rsh[pg * PS + i];
    } else {
#pragma unroll
      for (int i = 0; i < PS; ++i) kr[i] = own;
    }
    const bf16* pk[PS];
#pragma unroll
    for (int i = 0; i < PS; ++i) pk[i] = kb + (long long)kr[i] * row_stride + (long long)(j0 + pg * PS + i) * pos_stride;
    bf16x8 kk[PS], vv[PS];
#pragma unroll
    for (int i = 0; i < PS; ++i)
      if (j0 + pg * PS + i < lk) kk[i] = *(const bf16x8*)pk[i];
    if constexpr (!LATE_V) {
#pragma unroll
      for (int i = 0; i < PS; ++i)
        if (j0 + pg * PS + i < lk) vv[i] = *(const bf16x8*)(pk[i] + kvd);
    }
    float s[PS];
    float cm = -INFINITY;
#pragma unroll
    for (int i = 0; i < PS; ++i) {
      float a = 0.f;
#pragma unroll
      for (int e = 0; e < 8; e += 2)
        a = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{qq[e], qq[e + 1]}, bf16x2_t{kk[i][e], kk[i][e + 1]}, a, false);
      a = sum8_cg(a) * scale;
      s[i] = j0 + pg * PS + i < lk ? a : -INFINITY;
      cm = fmaxf(cm, s[i]);
    }
    if constexpr (LATE_V) {
#pragma unroll
      for (int i = 0; i < PS; ++i)
        if (j0 + pg * PS + i < lk) vv[i] = *(const bf16x8*)(pk[i] + kvd);
    }
    cm = fmaxf(cm, dpp_f<0x128>(cm));  // row_ror 8: xor 8
    cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
    cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
    const float mn = fmaxf(m, cm);
    const float corr = expf(m - mn);  // m = -inf on the first chunk: exp(-inf) = 0
    float ps = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= corr;
#pragma unroll
    for (int i = 0; i < PS; ++i) {
      if (j0 + pg * PS + i < lk) {
        const float p = expf(s[i] - mn);
        ps += p;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += p * (float)vv[i][e];
      }
    }
    ps += dpp_f<0x128>(ps);
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
  }
  // sum over the 8 position groups in pg order, one channel per lane
  *(f32x4*)&red[pg][cg * 8] = f32x4{o[0], o[1], o[2], o[3]};
  *(f32x4*)&red[pg][cg * 8 + 4] = f32x4{o[4], o[5], o[6], o[7]};
  __syncthreads();
  float acc = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) acc += red[g][lane];
  out[(long long)r * ldo + h * D + lane] = (bf16)(lk > 0 ? acc / l : 0.f);
}

// ---- beam step -----------------------------------------------------------
constexpr int BEAM_MAX = 16;
constexpr int BS_THREADS = 512;

// tf.math.top_k order: larger value first, equal values by lower index
__device__ __forceinline__ bool better(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi);
}

__global__ __launch_bounds__(BS_THREADS) void beam_step_kernel(
    int beam_n, int vocab, const float* __restrict__ logits, long long ldl, float* __restrict__ beam_prob,
    const int32_t* __restrict__ hist_in, int32_t* __restrict__ hist_out, int hist_ld, int t,
    const int32_t* __restrict__ src_in, int32_t* __restrict__ src_out, int src_ld, int end_token,
    int32_t* __restrict__ tok_out, int32_t* __restrict__ result, int result_ld, int32_t* __restrict__ result_len,
    int32_t* __restrict__ status) {
  const int img = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = BS_THREADS / 64;
  __shared__ float rmax[BEAM_MAX], rinv[BEAM_MAX], bprob[BEAM_MAX];
  __shared__ float lv[BS_THREADS][BEAM_MAX];
  __shared__ int li[BS_THREADS][BEAM_MAX];
  __shared__ float sel_v[BEAM_MAX];
  __shared__ int sel_i[BEAM_MAX];
  __shared__ float red_v[NW];
  __shared__ int red_i[NW], red_t[NW];
  const int row0 = img * beam_n;
  // Round 6: every pass over a beam row runs on one wave with 16-B loads,
  // four of them in flight per lane (the scalar strided loops waited out one
  // load latency per iteration: 333 us per step at 256 images x 8 beams x
  // V 10 000, profiles/r06/c5_beam_step.txt). vec: rows 16-B aligned, V % 4 == 0.
  const bool vec = (vocab & 3) == 0 && (ldl & 3) == 0 && ((uintptr_t)logits & 15) == 0;
  const int nv4 = vocab >> 2;
  // 1. per-beam softmax statistics (wave per beam row)
  for (int b = wave; b < beam_n; b += NW) {
    const float* lr = logits + (long long)(row0 + b) * ldl;
    float mx = -INFINITY;
    if (vec) {
      const f32x4* l4 = (const f32x4*)lr;
      int j = lane;
      for (; j + 192 < nv4; j += 256) {
        const f32x4 a = l4[j], c = l4[j + 64], d = l4[j + 128], e = l4[j + 192];
#pragma unroll
        for (int q = 0; q < 4; ++q) mx = fmaxf(mx, fmaxf(fmaxf(a[q], c[q]), fmaxf(d[q], e[q])));
      }
      for (; j < nv4; j += 64) {
        const f32x4 a = l4[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) mx = fmaxf(mx, a[q]);
      }
    } else {
      for (int j = lane; j < vocab; j += 64) mx = fmaxf(mx, lr[j]);
    }
    mx = wave_max(mx);
    float s = 0.f;
    if (vec) {
      const f32x4* l4 = (const f32x4*)lr;
      int j = lane;
      for (; j + 192 < nv4; j += 256) {
        const f32x4 a = l4[j], c = l4[j + 64], d = l4[j + 128], e = l4[j + 192];
#pragma unroll
        for (int q = 0; q < 4; ++q) s += expf(a[q] - mx);
#pragma unroll
        for (int q = 0; q < 4; ++q) s += expf(c[q] - mx);
#pragma unroll
        for (int q = 0; q < 4; ++q) s += expf(d[q] - mx);
#pragma unroll
        for (int q = 0; q < 4; ++q) s += expf(e[q] - mx);
      }
      for (; j < nv4; j += 64) {
        const f32x4 a = l4[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) s += expf(a[q] - mx);
      }
    } else {
      for (int j = lane; j < vocab; j += 64) s += expf(lr[j] - mx);
    }
    s = wave_sum(s);
    if (lane == 0) {
      rmax[b] = mx;
      rinv[b] = s;  // the sum; p = exp(l - max) / sum like the softmax it restates
      bprob[b] = beam_prob[row0 + b];
    }
  }
  __syncthreads();
  // 2. per-thread sorted top-k of its candidates c = p * beam_prob (flat
  //    index f = b * V + j; any partition of the candidates gives the same
  //    final top-k, ties broken by the lower f)
  const int K = beam_n;
  float tv[BEAM_MAX];
  int ti[BEAM_MAX];
#pragma unroll
  for (int k = 0; k < BEAM_MAX; ++k) {
    tv[k] = -INFINITY;
    ti[k] = 0x7fffffff;
  }
  auto offer = [&](float c, int f) {
    if (better(c, f, tv[BEAM_MAX - 1], ti[BEAM_MAX - 1])) {
      // sorted insert by compare-swap down the list (compile-time indices
      // only: a runtime-indexed register array would live in scratch)
      float cv = c;
      int ci = f;
#pragma unroll
      for (int k = 0; k < BEAM_MAX; ++k) {
        if (better(cv, ci, tv[k], ti[k])) {
          const float sv = tv[k];
          const int si = ti[k];
          tv[k] = cv;
          ti[k] = ci;
          cv = sv;
          ci = si;
        }
      }
    }
  };
  if (vec) {
    for (int b = wave; b < beam_n; b += NW) {
      const f32x4* l4 = (const f32x4*)(logits + (long long)(row0 + b) * ldl);
      const float mx = rmax[b], sm = rinv[b], bp = bprob[b];
      const int f0 = b * vocab;
      int j = lane;
      for (; j + 64 < nv4; j += 128) {
        const f32x4 a = l4[j], c = l4[j + 64];
#pragma unroll
        for (int q = 0; q < 4; ++q) offer((expf(a[q] - mx) / sm) * bp, f0 + 4 * j + q);
#pragma unroll
        for (int q = 0; q < 4; ++q) offer((expf(c[q] - mx) / sm) * bp, f0 + 4 * (j + 64) + q);
      }
      for (; j < nv4; j += 64) {
        const f32x4 a = l4[j];
#pragma unroll
        for (int q = 0; q < 4; ++q) offer((expf(a[q] - mx) / sm) * bp, f0 + 4 * j + q);
      }
    }
  } else {
    const int total = beam_n * vocab;
    for (int f = tid; f < total; f += BS_THREADS) {
      const int b = f / vocab, j = f - b * vocab;
      offer((expf(logits[(long long)(row0 + b) * ldl + j] - rmax[b]) / rinv[b]) * bprob[b], f);
    }
  }
#pragma unroll
  for (int k = 0; k < BEAM_MAX; ++k) {
    lv[tid][k] = tv[k];
    li[tid][k] = ti[k];
  }
  __syncthreads();
  // 3. k rounds of a block arg-best over the list heads
  int head = 0;
  for (int round = 0; round < K; ++round) {
    float bv = head < K ? lv[tid][head] : -INFINITY;
    int bi = head < K ? li[tid][head] : 0x7fffffff;
    int bt = tid;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      const int ot = __shfl_xor(bt, o, 64);
      if (better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
        bt = ot;
      }
    }
    if (lane == 0) {
      red_v[wave] = bv;
      red_i[wave] = bi;
      red_t[wave] = bt;
    }
    __syncthreads();
    if (tid == 0) {
      float wv = red_v[0];
      int wi = red_i[0], wt = red_t[0];
      for (int w = 1; w < NW; ++w)
        if (better(red_v[w], red_i[w], wv, wi)) {
          wv = red_v[w];
          wi = red_i[w];
          wt = red_t[w];
        }
      sel_v[round] = wv;
      sel_i[round] = wi;
      red_t[0] = wt;
    }
    __syncthreads();
    if (tid == red_t[0]) ++head;
    __syncthreads();
  }
  // 4. new beams: parent = flat / V, token = flat % V (pipeline.py:128-141);
  //    best beam = argmax of the new probabilities, first max (:143)
  int best = 0;
  for (int k = 1; k < K; ++k)
    if (sel_v[k] > sel_v[best]) best = k;
  for (int e = tid; e < K * (t + 2); e += BS_THREADS) {
    const int k = e / (t + 2), pos = e - k * (t + 2);
    const int parent = sel_i[k] / vocab, tok = sel_i[k] - parent * vocab;
    const int r = row0 + k, pr = row0 + parent;
    hist_out[(long long)r * hist_ld + pos] = pos <= t ? hist_in[(long long)pr * hist_ld + pos] : tok;
    if (pos <= t) src_out[(long long)r * src_ld + pos] = src_in[(long long)pr * src_ld + pos];
    else if (pos < src_ld) src_out[(long long)r * src_ld + pos] = r;  // next step writes its K/V at row r
  }
  if (tid < K) {
    const int parent = sel_i[tid] / vocab, tok = sel_i[tid] - parent * vocab;
    tok_out[row0 + tid] = tok;
    beam_prob[row0 + tid] = sel_v[tid];
  }
  // 5. result capture (pipeline.py:143-154): while running, the best beam's
  //    tokens after <start>; when it ends with <end>, without it, and stop
  if (status[img] == 0) {
    const int parent = sel_i[best] / vocab, tok = sel_i[best] - parent * vocab;
    const int pr = row0 + parent;
    const bool ended = tok == end_token;
    const int n = ended ? t : t + 1;  // tokens kept after <start>
    for (int pos = tid; pos < n; pos += BS_THREADS)
      result[(long long)img * result_ld + pos] =
          pos + 1 <= t ? hist_in[(long long)pr * hist_ld + pos + 1] : tok;
    __syncthreads();
    if (tid == 0) {
      result_len[img] = n;
      if (ended) status[img] = 1;
    }
  }
}

// ---- one-query attention (Lq = 1) for the training path -----------------
// The multi-view encoder attends from ONE baseline token per image at 224^2
// (transformer.py:176-200, the P6 view is 1x1): QK^T / softmax / PV as
// batched GEMMs with M = 1 are 3 latency-bound launches forward and 5+
// backward per MHA. Here one wave per (image, head) — grid (B, H), so the
// waves spread over B*H CUs — does the whole forward (scores in LDS, weights
// written in dtype like the general path, PV from the dtype-rounded weights)
// and one kernel the whole backward. Key / value rows are read as 16-B
// vectors when the layout allows (VEC).
// LDS per block: q or dO (64) + scores / dS and P (2 * Lk) floats.
constexpr int Q1_MAX_LK = 4096;

template <typename T, bool VEC>
__device__ __forceinline__ float q1_dot(const float* __restrict__ x, const T* __restrict__ row, int D) {
  float acc = 0.f;
  if constexpr (VEC) {
    for (int d = 0; d < D; d += 8) {
      const bf16x8 r = *(const bf16x8*)(row + d);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += x[d + e] * (float)r[e];
    }
  } else {
    for (int d = 0; d < D; ++d) acc += x[d] * to_f32(row[d]);
  }
  return acc;
}

template <typename T, bool VEC>
__global__ __launch_bounds__(64) void attn_q1_fwd_kernel(int H, int Lk, int D, float scale,
                                                         const T* __restrict__ q, long long ldq,
                                                         const T* __restrict__ k, long long ldk,
                                                         const T* __restrict__ v, long long ldv,
                                                         const float* __restrict__ mask, long long m_sb,
                                                         long long m_sh, long long m_sj,
                                                         T* __restrict__ out, long long ldo,
                                                         T* __restrict__ w, long long ldw) {
  extern __shared__ float q1_sm[];
  const int b = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  float* qs = q1_sm;
  float* ps = qs + 64;
  if (lane < D) qs[lane] = to_f32(q[(long long)b * ldq + h * D + lane]) * scale;
  __syncthreads();
  const T* kb = k + (long long)b * Lk * ldk + h * D;
  const float* mrow = mask ? mask + b * m_sb + h * m_sh : nullptr;
  float mx = -INFINITY;
  if constexpr (VEC) {
    if (D == 64) {
      // 4 key rows per lane per batch, 8 x 16-B loads each, all in flight
      for (int j0 = lane; j0 < Lk; j0 += 256) {
        bf16x8 r[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const T* kr = kb + (long long)min(j0 + 64 * u, Lk - 1) * ldk;
#pragma unroll
          for (int c = 0; c < 8; ++c) r[u][c] = *(const bf16x8*)(kr + 8 * c);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + 64 * u;
          float acc = 0.f;
#pragma unroll
          for (int c = 0; c < 8; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc += qs[8 * c + e] * (float)r[u][c][e];
          if (j < Lk) {
            if (mrow) acc += mrow[(long long)j * m_sj] * -1e9f;
            ps[j] = acc;
            mx = fmaxf(mx, acc);
          }
        }
      }
    }
  }
  if (!(VEC && D == 64)) {
    for (int j = lane; j < Lk; j += 64) {
      float acc = q1_dot<T, VEC>(qs, kb + (long long)j * ldk, D);
      if (mrow) acc += mrow[(long long)j * m_sj] * -1e9f;
      ps[j] = acc;
      mx = fmaxf(mx, acc);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Lk; j += 64) {
    const float e = expf(ps[j] - mx);
    ps[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  T* wr = w + ((long long)b * H + h) * ldw;
  for (int j = lane; j < (int)ldw; j += 64) {
    const T pv = from_f32<T>(j < Lk ? ps[j] / sum : 0.f);
    wr[j] = pv;
    if (j < Lk) ps[j] = to_f32(pv);  // PV uses the stored (dtype-rounded) weights
  }
  __syncthreads();
  if constexpr (VEC) {
    if (D == 64) {
      // lane = key slot ks (8) x dim group dg (8 dims, one 16-B vector): 8
      // keys per iteration, then a reduction over the key slots
      const int ks = lane >> 3, dg = lane & 7;
      const T* vb = v + (long long)b * Lk * ldv + h * D + dg * 8;
      float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      // 8 rows per lane in flight per batch (clamped rows, zero weight past Lk)
      for (int j0 = ks; j0 < Lk; j0 += 64) {
        bf16x8 r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = *(const bf16x8*)(vb + (long long)min(j0 + 8 * u, Lk - 1) * ldv);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = j0 + 8 * u;
          const float pj = j < Lk ? ps[j] : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += pj * (float)r[u][e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 8, 64);
        o[e] += __shfl_xor(o[e], 16, 64);
        o[e] += __shfl_xor(o[e], 32, 64);
      }
      if (ks == 0) {
        bf16x8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[e] = (bf16)o[e];
        *(bf16x8*)(out + (long long)b * ldo + h * D + dg * 8) = ov;
      }
      return;
    }
  }
  if (lane < D) {
    const T* vb = v + (long long)b * Lk * ldv + h * D + lane;
    float o0 = 0.f, o1 = 0.f;
    int j = 0;
    for (; j + 1 < Lk; j += 2) {
      o0 += ps[j] * to_f32(vb[(long long)j * ldv]);
      o1 += ps[j + 1] * to_f32(vb[(long long)(j + 1) * ldv]);
    }
    if (j < Lk) o0 += ps[j] * to_f32(vb[(long long)j * ldv]);
    out[(long long)b * ldo + h * D + lane] = from_f32<T>(o0 + o1);
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(64) void attn_q1_bwd_kernel(int H, int Lk, int D, float scale,
                                                         const T* __restrict__ q, long long ldq,
                                                         const T* __restrict__ k, long long ldk,
                                                         const T* __restrict__ v, long long ldv,
                                                         const T* __restrict__ w, long long ldw,
                                                         const T* __restrict__ dout, long long ldo,
                                                         T* __restrict__ dq, T* __restrict__ dk,
                                                         T* __restrict__ dv) {
  extern __shared__ float q1_sm[];
  const int b = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  float* gs = q1_sm;     // dO of this head
  float* dps = gs + 64;  // dP, then dS
  float* pw = dps + Lk;  // P
  const float qd = lane < D ? to_f32(q[(long long)b * ldq + h * D + lane]) : 0.f;
  if (lane < D) gs[lane] = to_f32(dout[(long long)b * ldo + h * D + lane]);
  __syncthreads();
  const T* wr = w + ((long long)b * H + h) * ldw;
  const T* vb = v + (long long)b * Lk * ldv + h * D;
  float acc = 0.f;
  if constexpr (VEC) {
    if (D == 64) {
      for (int j0 = lane; j0 < Lk; j0 += 256) {
        bf16x8 r[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const T* vr = vb + (long long)min(j0 + 64 * u, Lk - 1) * ldv;
#pragma unroll
          for (int c = 0; c < 8; ++c) r[u][c] = *(const bf16x8*)(vr + 8 * c);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + 64 * u;
          float dp = 0.f;
#pragma unroll
          for (int c = 0; c < 8; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) dp += gs[8 * c + e] * (float)r[u][c][e];
          if (j < Lk) {
            const float pj = to_f32(wr[j]);
            dps[j] = dp;
            pw[j] = pj;
            acc += pj * dp;
          }
        }
      }
    }
  }
  if (!(VEC && D == 64)) {
    for (int j = lane; j < Lk; j += 64) {
      const float dp = q1_dot<T, VEC>(gs, vb + (long long)j * ldv, D);
      const float pj = to_f32(wr[j]);
      dps[j] = dp;
      pw[j] = pj;
      acc += pj * dp;
    }
  }
  const float dsum = wave_sum(acc);
  for (int j = lane; j < Lk; j += 64) dps[j] = pw[j] * (dps[j] - dsum);  // dS
  __syncthreads();
  if constexpr (VEC) {
    if (D == 64) {
      // lane = key slot ks x dim group dg: rows of dK / dV as 16-B stores,
      // dq over key slots then reduced
      const int ks = lane >> 3, dg = lane & 7;
      float qv[8], gv[8], dqv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        qv[e] = __shfl(qd, dg * 8 + e, 64) * scale;
        gv[e] = gs[dg * 8 + e];
        dqv[e] = 0.f;
      }
      const long long kof = (long long)b * Lk * ldk + h * D + dg * 8;
      const long long vof = (long long)b * Lk * ldv + h * D + dg * 8;
      for (int j0 = ks; j0 < Lk; j0 += 64) {
        bf16x8 kr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) kr[u] = *(const bf16x8*)(k + kof + (long long)min(j0 + 8 * u, Lk - 1) * ldk);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = j0 + 8 * u;
          if (j >= Lk) break;
          const float ds = dps[j], pj = pw[j];
          bf16x8 dko, dvo;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            dko[e] = (bf16)(ds * qv[e]);
            dvo[e] = (bf16)(pj * gv[e]);
            dqv[e] += ds * (float)kr[u][e];
          }
          *(bf16x8*)(dk + kof + (long long)j * ldk) = dko;
          *(bf16x8*)(dv + vof + (long long)j * ldv) = dvo;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dqv[e] += __shfl_xor(dqv[e], 8, 64);
        dqv[e] += __shfl_xor(dqv[e], 16, 64);
        dqv[e] += __shfl_xor(dqv[e], 32, 64);
      }
      if (ks == 0) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)(scale * dqv[e]);
        *(bf16x8*)(dq + (long long)b * ldq + h * D + dg * 8) = o;
      }
      return;
    }
  }
  // dk_j = scale * dS_j * q, dv_j = P_j * dO: lane d of every row j (coalesced)
  if (lane < D) {
    T* dkb = dk + (long long)b * Lk * ldk + h * D + lane;
    T* dvb = dv + (long long)b * Lk * ldv + h * D + lane;
    const float gd = gs[lane];
    const T* kb = k + (long long)b * Lk * ldk + h * D + lane;
    float dq0 = 0.f, dq1 = 0.f;
    int j = 0;
    for (; j + 1 < Lk; j += 2) {
      const float ds0 = dps[j], ds1 = dps[j + 1];
      const float k0 = to_f32(kb[(long long)j * ldk]), k1 = to_f32(kb[(long long)(j + 1) * ldk]);
      dkb[(long long)j * ldk] = from_f32<T>(scale * ds0 * qd);
      dkb[(long long)(j + 1) * ldk] = from_f32<T>(scale * ds1 * qd);
      dvb[(long long)j * ldv] = from_f32<T>(pw[j] * gd);
      dvb[(long long)(j + 1) * ldv] = from_f32<T>(pw[j + 1] * gd);
      dq0 += ds0 * k0;
      dq1 += ds1 * k1;
    }
    if (j < Lk) {
      const float ds = dps[j];
      dkb[(long long)j * ldk] = from_f32<T>(scale * ds * qd);
      dvb[(long long)j * ldv] = from_f32<T>(pw[j] * gd);
      dq0 += ds * to_f32(kb[(long long)j * ldk]);
    }
    dq[(long long)b * ldq + h * D + lane] = from_f32<T>(scale * (dq0 + dq1));
  }
}

// Multi-wave form of the two kernels above for the long views (bf16, D = 64,
// Lk >= Q1_MW_MIN_LK: the P3 / P4 views of the encoder, 784 / 196 keys at
// 224^2): NW waves per (image, head) share the key rows (scores, dS) and the
// PV / dK / dV slots, with the softmax max / sums and the per-wave PV and dq
// partials combined through LDS in wave order. One wave per block left the
// 256 blocks of the batch-32 step at one wave per CU (6.8 / 10.8 us per
// launch at 0.9 / 1.1 TB/s); with 4 waves the P3 view's launches (784 keys,
// 51 MB of K + V read forward, of dK + dV written backward) run in 7.8 /
// 11.9 us = 6.5 / 4.3 TB/s of algorithmic bytes (8 waves: no faster).
// LDS: q or dO (64) + 2*NW + NW*64 partials + 2*Lk floats.
constexpr int Q1_MW = 4;
constexpr int Q1_MW_MIN_LK = 128;

template <int NW>
__device__ __forceinline__ void q1_fwd_mw_body(int b, int h, int H, int Lk, float scale,
                                               const bf16* __restrict__ q, long long ldq,
                                               const bf16* __restrict__ k, long long ldk,
                                               const bf16* __restrict__ v, long long ldv,
                                               const float* __restrict__ mask, long long m_sb, long long m_sh,
                                               long long m_sj, bf16* __restrict__ out, long long ldo,
                                               bf16* __restrict__ w, long long ldw) {
  constexpr int NT = 64 * NW, KS = NT / 8;
  extern __shared__ float q1_sm[];
  float* qs = q1_sm;
  float* red = qs + 64;
  float* opart = red + 2 * NW;
  float* ps = opart + NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 64) qs[tid] = (float)q[(long long)b * ldq + h * 64 + tid] * scale;
  __syncthreads();
  const bf16* kb = k + (long long)b * Lk * ldk + h * 64;
  const float* mrow = mask ? mask + b * m_sb + h * m_sh : nullptr;
  float mx = -INFINITY;
  for (int j0 = tid; j0 < Lk; j0 += 4 * NT) {
    bf16x8 r[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bf16* kr = kb + (long long)min(j0 + NT * u, Lk - 1) * ldk;
#pragma unroll
      for (int c = 0; c < 8; ++c) r[u][c] = *(const bf16x8*)(kr + 8 * c);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + NT * u;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += qs[8 * c + e] * (float)r[u][c][e];
      if (j < Lk) {
        if (mrow) acc += mrow[(long long)j * m_sj] * -1e9f;
        ps[j] = acc;
        mx = fmaxf(mx, acc);
      }
    }
  }
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) mx = fmaxf(mx, red[i]);
  float sum = 0.f;
  for (int j = tid; j < Lk; j += NT) {
    const float e = expf(ps[j] - mx);
    ps[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[NW + wave] = sum;
  __syncthreads();
  sum = red[NW];
#pragma unroll
  for (int i = 1; i < NW; ++i) sum += red[NW + i];
  bf16* wr = w + ((long long)b * H + h) * ldw;
  for (int j = tid; j < (int)ldw; j += NT) {
    const bf16 pv = (bf16)(j < Lk ? ps[j] / sum : 0.f);
    wr[j] = pv;
    if (j < Lk) ps[j] = (float)pv;  // PV uses the stored (dtype-rounded) weights
  }
  __syncthreads();
  // thread = key slot ks (KS) x dim group dg (8 dims, one 16-B vector)
  const int ks = tid >> 3, dg = tid & 7;
  const bf16* vb = v + (long long)b * Lk * ldv + h * 64 + dg * 8;
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = ks; j0 < Lk; j0 += 8 * KS) {
    bf16x8 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = *(const bf16x8*)(vb + (long long)min(j0 + KS * u, Lk - 1) * ldv);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + KS * u;
      const float pj = j < Lk ? ps[j] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pj * (float)r[u][e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o[e] += __shfl_xor(o[e], 8, 64);
    o[e] += __shfl_xor(o[e], 16, 64);
    o[e] += __shfl_xor(o[e], 32, 64);
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) opart[wave * 64 + lane * 8 + e] = o[e];
  }
  __syncthreads();
  if (tid < 8) {
    bf16x8 ov;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = opart[tid * 8 + e];
#pragma unroll
      for (int i = 1; i < NW; ++i) t += opart[i * 64 + tid * 8 + e];
      ov[e] = (bf16)t;
    }
    *(bf16x8*)(out + (long long)b * ldo + h * 64 + tid * 8) = ov;
  }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_q1_fwd_mw_kernel(int H, int Lk, float scale,
                                                               const bf16* __restrict__ q, long long ldq,
                                                               const bf16* __restrict__ k, long long ldk,
                                                               const bf16* __restrict__ v, long long ldv,
                                                               const float* __restrict__ mask, long long m_sb,
                                                               long long m_sh, long long m_sj,
                                                               bf16* __restrict__ out, long long ldo,
                                                               bf16* __restrict__ w, long long ldw) {
  q1_fwd_mw_body<NW>(blockIdx.x, blockIdx.y, H, Lk, scale, q, ldq, k, ldk, v, ldv, mask, m_sb, m_sh, m_sj, out, ldo,
                     w, ldw);
}

template <int NW>
__device__ __forceinline__ void q1_bwd_mw_body(int b, int h, int H, int Lk, float scale,
                                               const bf16* __restrict__ q, long long ldq,
                                               const bf16* __restrict__ k, long long ldk,
                                               const bf16* __restrict__ v, long long ldv,
                                               const bf16* __restrict__ w, long long ldw,
                                               const bf16* __restrict__ dout, long long ldo,
                                               bf16* __restrict__ dq, bf16* __restrict__ dk,
                                               bf16* __restrict__ dv) {
  constexpr int NT = 64 * NW, KS = NT / 8;
  extern __shared__ float q1_sm[];
  float* gs = q1_sm;  // dO of this head
  float* red = gs + 64;
  float* qpart = red + 2 * NW;
  float* dps = qpart + NW * 64;  // dP, then dS
  float* pw = dps + Lk;          // P
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float qd = (float)q[(long long)b * ldq + h * 64 + lane];
  if (tid < 64) gs[tid] = (float)dout[(long long)b * ldo + h * 64 + tid];
  __syncthreads();
  const bf16* wr = w + ((long long)b * H + h) * ldw;
  const bf16* vb = v + (long long)b * Lk * ldv + h * 64;
  float acc = 0.f;
  for (int j0 = tid; j0 < Lk; j0 += 4 * NT) {
    bf16x8 r[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bf16* vr = vb + (long long)min(j0 + NT * u, Lk - 1) * ldv;
#pragma unroll
      for (int c = 0; c < 8; ++c) r[u][c] = *(const bf16x8*)(vr + 8 * c);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + NT * u;
      float dp = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) dp += gs[8 * c + e] * (float)r[u][c][e];
      if (j < Lk) {
        const float pj = (float)wr[j];
        dps[j] = dp;
        pw[j] = pj;
        acc += pj * dp;
      }
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  float dsum = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) dsum += red[i];
  for (int j = tid; j < Lk; j += NT) dps[j] = pw[j] * (dps[j] - dsum);  // dS
  __syncthreads();
  const int ks = tid >> 3, dg = tid & 7;
  float qv[8], gv[8], dqv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    qv[e] = __shfl(qd, dg * 8 + e, 64) * scale;
    gv[e] = gs[dg * 8 + e];
    dqv[e] = 0.f;
  }
  const long long kof = (long long)b * Lk * ldk + h * 64 + dg * 8;
  const long long vof = (long long)b * Lk * ldv + h * 64 + dg * 8;
  for (int j0 = ks; j0 < Lk; j0 += 8 * KS) {
    bf16x8 kr[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) kr[u] = *(const bf16x8*)(k + kof + (long long)min(j0 + KS * u, Lk - 1) * ldk);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + KS * u;
      if (j >= Lk) break;
      const float ds = dps[j], pj = pw[j];
      bf16x8 dko, dvo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dko[e] = (bf16)(ds * qv[e]);
        dvo[e] = (bf16)(pj * gv[e]);
        dqv[e] += ds * (float)kr[u][e];
      }
      *(bf16x8*)(dk + kof + (long long)j * ldk) = dko;
      *(bf16x8*)(dv + vof + (long long)j * ldv) = dvo;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    dqv[e] += __shfl_xor(dqv[e], 8, 64);
    dqv[e] += __shfl_xor(dqv[e], 16, 64);
    dqv[e] += __shfl_xor(dqv[e], 32, 64);
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) qpart[wave * 64 + lane * 8 + e] = dqv[e];
  }
  __syncthreads();
  if (tid < 8) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = qpart[tid * 8 + e];
#pragma unroll
      for (int i = 1; i < NW; ++i) t += qpart[i * 64 + tid * 8 + e];
      o[e] = (bf16)(scale * t);
    }
    *(bf16x8*)(dq + (long long)b * ldq + h * 64 + tid * 8) = o;
  }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_q1_bwd_mw_kernel(int H, int Lk, float scale,
                                                               const bf16* __restrict__ q, long long ldq,
                                                               const bf16* __restrict__ k, long long ldk,
                                                               const bf16* __restrict__ v, long long ldv,
                                                               const bf16* __restrict__ w, long long ldw,
                                                               const bf16* __restrict__ dout, long long ldo,
                                                               bf16* __restrict__ dq, bf16* __restrict__ dk,
                                                               bf16* __restrict__ dv) {
  q1_bwd_mw_body<NW>(blockIdx.x, blockIdx.y, H, Lk, scale, q, ldq, k, ldk, v, ldv, w, ldw, dout, ldo, dq, dk, dv);
}

// The encoder layer's per-view attentions (one baseline query row against
// each view's keys, transformer.py:184-190) as ONE launch: blockIdx.z = view,
// each block the multi-wave body of its view. Heavy views first in the
// table (P3's 784 keys) so their blocks start first.
struct Q1View {
  const bf16 *q, *k, *v;
  bf16 *out, *w;
  const bf16* dout;
  bf16 *dq, *dk, *dv;
  long long ldq, ldk, ldv, ldo, ldw;
  int lk;
};
struct Q1Views {
  Q1View v[FPNMT_MAX_VIEWS];
};

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_q1_views_fwd_kernel(const Q1Views A, int H, float scale) {
  const Q1View& a = A.v[blockIdx.z];
  q1_fwd_mw_body<NW>(blockIdx.x, blockIdx.y, H, a.lk, scale, a.q, a.ldq, a.k, a.ldk, a.v, a.ldv, nullptr, 0, 0, 0,
                     a.out, a.ldo, a.w, a.ldw);
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_q1_views_bwd_kernel(const Q1Views A, int H, float scale) {
  const Q1View& a = A.v[blockIdx.z];
  q1_bwd_mw_body<NW>(blockIdx.x, blockIdx.y, H, a.lk, scale, a.q, a.ldq, a.k, a.ldk, a.v, a.ldv, a.w, a.ldw,
                     a.dout, a.ldo, a.dq, a.dk, a.dv);
}

static bool q1_vec(const fpnmt_attn_desc* d, const void* k, const void* v, const void* o1 = nullptr,
                   const void* o2 = nullptr, const void* o3 = nullptr) {
  return d->dtype == FPNMT_BF16 && d->d % 8 == 0 && d->ldk % 8 == 0 && d->ldv % 8 == 0 && d->ldq % 8 == 0 &&
         d->ldo % 8 == 0 && (((uintptr_t)k | (uintptr_t)v | (uintptr_t)o1 | (uintptr_t)o2 | (uintptr_t)o3) & 15) == 0;
}

int attn_q1_fwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const float* mask, void* out,
                void* weights, hipStream_t s) {
  const size_t smem = (size_t)(64 + 2 * d->lk) * sizeof(float);
  const dim3 grid(d->b, d->h);
  if (d->dtype == FPNMT_BF16 && d->d == 64 && d->lk >= Q1_MW_MIN_LK && q1_vec(d, k, v, out)) {
    const size_t sm = (size_t)(64 + 2 * Q1_MW + 64 * Q1_MW + d->lk) * sizeof(float);
    hipLaunchKernelGGL((attn_q1_fwd_mw_kernel<Q1_MW>), grid, dim3(64 * Q1_MW), sm, s, d->h, d->lk, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, mask, d->m_sb, d->m_sh,
                       d->m_sj, (bf16*)out, d->ldo, (bf16*)weights, d->ldw);
  } else if (d->dtype == FPNMT_BF16) {
    if (q1_vec(d, k, v, out))
      hipLaunchKernelGGL((attn_q1_fwd_kernel<bf16, true>), grid, dim3(64), smem, s, d->h, d->lk, d->d, d->scale,
                         (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, mask, d->m_sb,
                         d->m_sh, d->m_sj, (bf16*)out, d->ldo, (bf16*)weights, d->ldw);
    else
      hipLaunchKernelGGL((attn_q1_fwd_kernel<bf16, false>), grid, dim3(64), smem, s, d->h, d->lk, d->d, d->scale,
                         (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, mask, d->m_sb,
                         d->m_sh, d->m_sj, (bf16*)out, d->ldo, (bf16*)weights, d->ldw);
  } else {
    hipLaunchKernelGGL((attn_q1_fwd_kernel<float, false>), grid, dim3(64), smem, s, d->h, d->lk, d->d, d->scale,
                       (const float*)q, d->ldq, (const float*)k, d->ldk, (const float*)v, d->ldv, mask, d->m_sb,
                       d->m_sh, d->m_sj, (float*)out, d->ldo, (float*)weights, d->ldw);
  }
  return check_launch("attention_q1_fwd");
}

int attn_q1_bwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const void* weights,
                const void* dout, void* dq, void* dk, void* dv, hipStream_t s) {
  const size_t smem = (size_t)(64 + 2 * d->lk) * sizeof(float);
  const dim3 grid(d->b, d->h);
  if (d->dtype == FPNMT_BF16 && d->d == 64 && d->lk >= Q1_MW_MIN_LK && q1_vec(d, k, v, dq, dk, dv)) {
    const size_t sm = (size_t)(64 + 2 * Q1_MW + 64 * Q1_MW + 2 * d->lk) * sizeof(float);
    hipLaunchKernelGGL((attn_q1_bwd_mw_kernel<Q1_MW>), grid, dim3(64 * Q1_MW), sm, s, d->h, d->lk, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, (const bf16*)weights,
                       d->ldw, (const bf16*)dout, d->ldo, (bf16*)dq, (bf16*)dk, (bf16*)dv);
  } else if (d->dtype == FPNMT_BF16) {
    if (q1_vec(d, k, v, dq, dk, dv))
      hipLaunchKernelGGL((attn_q1_bwd_kernel<bf16, true>), grid, dim3(64), smem, s, d->h, d->lk, d->d, d->scale,
                         (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv,
                         (const bf16*)weights, d->ldw, (const bf16*)dout, d->ldo, (bf16*)dq, (bf16*)dk, (bf16*)dv);
    else
      hipLaunchKernelGGL((attn_q1_bwd_kernel<bf16, false>), grid, dim3(64), smem, s, d->h, d->lk, d->d, d->scale,
                         (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv,
                         (const bf16*)weights, d->ldw, (const bf16*)dout, d->ldo, (bf16*)dq, (bf16*)dk, (bf16*)dv);
  } else {
    hipLaunchKernelGGL((attn_q1_bwd_kernel<float, false>), grid, dim3(64), smem, s, d->h, d->lk, d->d, d->scale,
                       (const float*)q, d->ldq, (const float*)k, d->ldk, (const float*)v, d->ldv,
                       (const float*)weights, d->ldw, (const float*)dout, d->ldo, (float*)dq, (float*)dk, (float*)dv);
  }
  return check_launch("attention_q1_bwd");
}

bool attn_q1_ok(const fpnmt_attn_desc* d) {
  return d->lq == 1 && d->lk > 0 && d->lk <= Q1_MAX_LK && d->h <= 65535 && d->d <= 64;
}

// one view of a grouped launch: the multi-wave body's requirements. A view
// without keys (a 0x0 pyramid level) is fine there: its blocks write the
// zero output / weights / dq that the attention over no keys has.
bool attn_q1_view_ok(const fpnmt_attn_desc* d, const void* k, const void* v, const void* o1, const void* o2,
                     const void* o3) {
  return d->lq == 1 && d->lk >= 0 && d->lk <= Q1_MAX_LK && d->h <= 65535 && d->dtype == FPNMT_BF16 && d->d == 64 &&
         d->b > 0 && q1_vec(d, k, v, o1, o2, o3);
}

static void q1_views_table(int n, const fpnmt_attn_desc* d, Q1Views& A, int& order_lk) {
  // heaviest view first (lowest blockIdx.z dispatches first)
  int idx[FPNMT_MAX_VIEWS];
  for (int i = 0; i < n; ++i) idx[i] = i;
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && d[idx[j]].lk > d[idx[j - 1]].lk; --j) std::swap(idx[j], idx[j - 1]);
  order_lk = n ? d[idx[0]].lk : 0;
  for (int i = 0; i < n; ++i) A.v[i].lk = idx[i];  // view index; filled by the callers
}

int attn_q1_views_fwd(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                      const void* const* v, void* const* out, void* const* w, hipStream_t s) {
  Q1Views A{};
  int max_lk = 0;
  q1_views_table(n, d, A, max_lk);
  for (int i = 0; i < n; ++i) {
    const int j = A.v[i].lk;
    Q1View& a = A.v[i];
    a.q = (const bf16*)q[j]; a.k = (const bf16*)k[j]; a.v = (const bf16*)v[j];
    a.out = (bf16*)out[j]; a.w = (bf16*)w[j];
    a.ldq = d[j].ldq; a.ldk = d[j].ldk; a.ldv = d[j].ldv; a.ldo = d[j].ldo; a.ldw = d[j].ldw;
    a.lk = d[j].lk;
  }
  const size_t sm = (size_t)(64 + 2 * Q1_MW + 64 * Q1_MW + max_lk) * sizeof(float);
  hipLaunchKernelGGL((attn_q1_views_fwd_kernel<Q1_MW>), dim3(d[0].b, d[0].h, n), dim3(64 * Q1_MW), sm, s, A, d[0].h,
                     d[0].scale);
  return check_launch("attention_q1_views_fwd");
}

int attn_q1_views_bwd(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                      const void* const* v, const void* const* w, const void* const* dout, void* const* dq,
                      void* const* dk, void* const* dv, hipStream_t s) {
  Q1Views A{};
  int max_lk = 0;
  q1_views_table(n, d, A, max_lk);
  for (int i = 0; i < n; ++i) {
    const int j = A.v[i].lk;
    Q1View& a = A.v[i];
    a.q = (const bf16*)q[j]; a.k = (const bf16*)k[j]; a.v = (const bf16*)v[j];
    a.w = (bf16*)w[j]; a.dout = (const bf16*)dout[j];
    a.dq = (bf16*)dq[j]; a.dk = (bf16*)dk[j]; a.dv = (bf16*)dv[j];
    a.ldq = d[j].ldq; a.ldk = d[j].ldk; a.ldv = d[j].ldv; a.ldo = d[j].ldo; a.ldw = d[j].ldw;
    a.lk = d[j].lk;
  }
  const size_t sm = (size_t)(64 + 2 * Q1_MW + 64 * Q1_MW + 2 * max_lk) * sizeof(float);
  hipLaunchKernelGGL((attn_q1_views_bwd_kernel<Q1_MW>), dim3(d[0].b, d[0].h, n), dim3(64 * Q1_MW), sm, s, A, d[0].h,
                     d[0].scale);
  return check_launch("attention_q1_views_bwd");
}

}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

int fpnmt_decode_attention(int dtype, int rows, int heads, int depth, int lk, float scale, const void* q,
                           long long ldq, const void* kv, long long row_stride, long long pos_stride,
                           long long k_off, long long v_off, const int32_t* src, int src_ld, int row_div,
                           void* out, long long ldo, fpnmt_stream_t stream) {
  if (rows <= 0 || heads <= 0) return 0;
  if (heads > 8 || depth > DEC_MAX_D || depth <= 0) return fail(FPNMT_E_UNSUPPORTED, "decode_attention: heads <= 8, depth <= 64");
  if (!q || !out || (lk > 0 && !kv)) return fail(FPNMT_E_ARG, "decode_attention: null pointer");
  if (row_div <= 0) return fail(FPNMT_E_ARG, "decode_attention: row_div must be >= 1");
  if (src && src_ld < lk) return fail(FPNMT_E_ARG, "decode_attention: src_ld < lk");
  dim3 block(64 * heads);
  const bool v16 = depth == 64 && ((uintptr_t)q & 15) == 0 && (ldq & 7) == 0 && ((uintptr_t)kv & 15) == 0 &&
                   ((row_stride | pos_stride | k_off | v_off) & 7) == 0 && ((uintptr_t)out & 15) == 0 &&
                   (ldo & 7) == 0;
  // tools/dec_attn_bench.hip (profiles/r06/dec_attn.txt): 2 positions per lane
  // at 8 waves per SIMD up to lk 16, 4 per lane (96 VGPRs) above
  if (dtype == FPNMT_BF16 && v16 && lk <= 16)
    hipLaunchKernelGGL((decode_attn_v_kernel<2, false, 8>), dim3(rows * heads), dim3(64), 0, S(stream), rows, heads,
                       lk, scale, (const bf16*)q, ldq, (const bf16*)kv, row_stride, pos_stride, k_off, v_off, src,
                       src_ld, row_div, (bf16*)out, ldo);
  else if (dtype == FPNMT_BF16 && v16)
    hipLaunchKernelGGL((decode_attn_v_kernel<4, false, 1>), dim3(rows * heads), dim3(64), 0, S(stream), rows, heads,
                       lk, scale, (const bf16*)q, ldq, (const bf16*)kv, row_stride, pos_stride, k_off, v_off, src,
                       src_ld, row_div, (bf16*)out, ldo);
  else if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((decode_attn_kernel<bf16>), dim3(rows), block, 0, S(stream), rows, heads, depth, lk, scale,
                       (const bf16*)q, ldq, (const bf16*)kv, row_stride, pos_stride, k_off, v_off, src, src_ld,
                       row_div, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL((decode_attn_kernel<float>), dim3(rows), block, 0, S(stream), rows, heads, depth, lk, scale,
                       (const float*)q, ldq, (const float*)kv, row_stride, pos_stride, k_off, v_off, src, src_ld,
                       row_div, (float*)out, ldo);
  return check_launch("decode_attention");
}

int fpnmt_beam_step(int n_images, int beam_n, int vocab, const float* logits, long long ldl, float* beam_prob,
                    const int32_t* hist_in, int32_t* hist_out, int hist_ld, int t, const int32_t* src_in,
                    int32_t* src_out, int src_ld, int end_token, int32_t* tok_out, int32_t* result, int result_ld,
                    int32_t* result_len, int32_t* status, fpnmt_stream_t stream) {
  if (n_images <= 0) return 0;
  if (beam_n <= 0 || beam_n > BEAM_MAX) return fail(FPNMT_E_UNSUPPORTED, "beam_step: 1 <= beam_n <= 16");
  if (vocab <= 0 || t < 0 || t + 2 > hist_ld || t + 1 > src_ld || t + 1 > result_ld)
    return fail(FPNMT_E_ARG, "beam_step: bad vocab / position / table widths");
  if (!logits || !beam_prob || !hist_in || !hist_out || !src_in || !src_out || !tok_out || !result || !result_len ||
      !status)
    return fail(FPNMT_E_ARG, "beam_step: null pointer");
  hipLaunchKernelGGL(beam_step_kernel, dim3(n_images), dim3(BS_THREADS), 0, S(stream), beam_n, vocab, logits, ldl,
                     beam_prob, hist_in, hist_out, hist_ld, t, src_in, src_out, src_ld, end_token, tok_out, result,
                     result_ld, result_len, status);
  return check_launch("beam_step");
}

}  // extern "C"

namespace fpnmt {

// ---- fused short-sequence attention (decoder self-attention T=31, cross-
// attention over a 1-position encoder output; transformer.py:70-104) ---------
// The general path is 3 launches forward (QK^T GEMM, masked softmax, PV GEMM)
// and 5 backward, each latency-bound at these sizes (~8-10 us per launch for
// a few KFLOP per (image, head)). Here one 256-thread block per (image, head)
// stages Q, K, V (and dO, P) in LDS as fp32 and does the whole forward or
// backward. Numerics follow the general path: scores / dP in fp32, weights
// and dS rounded to dtype before they are used (as the GEMMs read them from
// their dtype buffers), softmax over S + mask * -1e9.
constexpr int SM_MAX_L = 32, SM_MAX_D = 64;

template <typename T>
__device__ __forceinline__ void sm_load(float (*dst)[SM_MAX_D + 1], const T* __restrict__ src, long long ld, int rows,
                                        int D) {
  for (int e = threadIdx.x; e < rows * D; e += 256) {
    const int r = e / D, c = e - r * D;
    dst[r][c] = to_f32(src[(long long)r * ld + c]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void attn_small_fwd_kernel(int H, int Lq, int Lk, int D, float scale,
                                                             const T* __restrict__ q, long long ldq,
                                                             const T* __restrict__ k, long long ldk,
                                                             const T* __restrict__ v, long long ldv,
                                                             const float* __restrict__ mask, long long msb,
                                                             long long msh, long long msi, long long msj,
                                                             T* __restrict__ out, long long ldo,
                                                             T* __restrict__ w, long long ldw) {
  __shared__ float Q[SM_MAX_L][SM_MAX_D + 1], K[SM_MAX_L][SM_MAX_D + 1], V[SM_MAX_L][SM_MAX_D + 1];
  __shared__ float P[SM_MAX_L][SM_MAX_L + 1];
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  sm_load(Q, q + (long long)b * Lq * ldq + h * D, ldq, Lq, D);
  sm_load(K, k + (long long)b * Lk * ldk + h * D, ldk, Lk, D);
  sm_load(V, v + (long long)b * Lk * ldv + h * D, ldv, Lk, D);
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * Lk; e += 256) {
    const int i = e / Lk, j = e - i * Lk;
    float s = 0.f;
    for (int c = 0; c < D; ++c) s += Q[i][c] * K[j][c];
    P[i][j] = s * scale;
  }
  __syncthreads();
  // one wave per row: lane j holds column j
  const float* mb = mask ? mask + (long long)b * msb + (long long)h * msh : nullptr;
  T* wb = w + ((long long)b * H + h) * Lq * ldw;
  for (int i = wave; i < Lq; i += 4) {
    float s = -INFINITY;
    if (lane < Lk) {
      s = P[i][lane];
      if (mb) s += mb[(long long)i * msi + (long long)lane * msj] * -1e9f;
    }
    const float mx = wave_max(s);
    const float ex = lane < Lk ? expf(s - mx) : 0.f;
    const float sum = wave_sum(ex);
    const T pt = from_f32<T>(lane < Lk ? ex * (1.f / sum) : 0.f);
    for (int j = lane; j < (int)ldw; j += 64) wb[(long long)i * ldw + j] = j == lane ? pt : from_f32<T>(0.f);
    if (lane < Lk) P[i][lane] = to_f32(pt);
  }
  __syncthreads();
  T* ob = out + (long long)b * Lq * ldo + h * D;
  for (int e = threadIdx.x; e < Lq * D; e += 256) {
    const int i = e / D, c = e - i * D;
    float o = 0.f;
    for (int j = 0; j < Lk; ++j) o += P[i][j] * V[j][c];
    ob[(long long)i * ldo + c] = from_f32<T>(o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void attn_small_bwd_kernel(int H, int Lq, int Lk, int D, float scale,
                                                             const T* __restrict__ q, long long ldq,
                                                             const T* __restrict__ k, long long ldk,
                                                             const T* __restrict__ v, long long ldv,
                                                             const T* __restrict__ w, long long ldw,
                                                             const T* __restrict__ dout, long long ldo,
                                                             T* __restrict__ dq, T* __restrict__ dk,
                                                             T* __restrict__ dv) {
  __shared__ float Q[SM_MAX_L][SM_MAX_D + 1], K[SM_MAX_L][SM_MAX_D + 1], V[SM_MAX_L][SM_MAX_D + 1],
      G[SM_MAX_L][SM_MAX_D + 1];
  __shared__ float P[SM_MAX_L][SM_MAX_L + 1], dS[SM_MAX_L][SM_MAX_L + 1];
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long qo = (long long)b * Lq * ldq + h * D, ko = (long long)b * Lk * ldk + h * D,
                  vo = (long long)b * Lk * ldv + h * D;
  sm_load(Q, q + qo, ldq, Lq, D);
  sm_load(K, k + ko, ldk, Lk, D);
  sm_load(V, v + vo, ldv, Lk, D);
  sm_load(G, dout + (long long)b * Lq * ldo + h * D, ldo, Lq, D);
  const T* wb = w + ((long long)b * H + h) * Lq * ldw;
  for (int e = threadIdx.x; e < Lq * Lk; e += 256) {
    const int i = e / Lk, j = e - i * Lk;
    P[i][j] = to_f32(wb[(long long)i * ldw + j]);
  }
  __syncthreads();
  // dP = dO V^T
  for (int e = threadIdx.x; e < Lq * Lk; e += 256) {
    const int i = e / Lk, j = e - i * Lk;
    float s = 0.f;
    for (int c = 0; c < D; ++c) s += G[i][c] * V[j][c];
    dS[i][j] = s;
  }
  __syncthreads();
  // dS = P (dP - sum_j P_j dP_j), rounded to dtype
  for (int i = wave; i < Lq; i += 4) {
    const float pj = lane < Lk ? P[i][lane] : 0.f, dpj = lane < Lk ? dS[i][lane] : 0.f;
    const float dot = wave_sum(pj * dpj);
    if (lane < Lk) dS[i][lane] = to_f32(from_f32<T>(pj * (dpj - dot)));
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * D; e += 256) {  // dQ = scale dS K
    const int i = e / D, c = e - i * D;
    float s = 0.f;
    for (int j = 0; j < Lk; ++j) s += dS[i][j] * K[j][c];
    dq[qo + (long long)i * ldq + c] = from_f32<T>(s * scale);
  }
  for (int e = threadIdx.x; e < Lk * D; e += 256) {  // dK = scale dS^T Q, dV = P^T dO
    const int j = e / D, c = e - j * D;
    float sk = 0.f, sv = 0.f;
    for (int i = 0; i < Lq; ++i) {
      sk += dS[i][j] * Q[i][c];
      sv += P[i][j] * G[i][c];
    }
    dk[ko + (long long)j * ldk + c] = from_f32<T>(sk * scale);
    dv[vo + (long long)j * ldv + c] = from_f32<T>(sv);
  }
}

// bf16 with D % 8 == 0, every ld % 8 == 0 and 16-B aligned bases: 16-B row
// chunks (one per thread per operand: rows <= 32, D/8 <= 8), all operand loads
// issued before the LDS stores; 1x4 score strips and 8-column output strips.
__device__ __forceinline__ void sm_put8(float* dst, const bf16x8& r) {
#pragma unroll
  for (int e = 0; e < 8; ++e) dst[e] = (float)r[e];
}
__device__ __forceinline__ bf16x8 sm_pack8(const float (&o)[8]) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = from_f32<bf16>(o[e]);
  return r;
}

// S[i][j0..j0+3] = sum_c X[i][c] Y[j][c] for Lq x ceil(Lk/4) strips
__device__ __forceinline__ void sm_strips(float (*X)[SM_MAX_D + 1], float (*Y)[SM_MAX_D + 1],
                                          float (*Sout)[SM_MAX_L + 1], int Lq, int Lk, int D, float scale) {
  const int nj4 = (Lk + 3) >> 2;
  for (int e = threadIdx.x; e < Lq * nj4; e += 256) {
    const int i = e / nj4, j0 = (e - i * nj4) * 4;
    const int j1 = min(j0 + 1, Lk - 1), j2 = min(j0 + 2, Lk - 1), j3 = min(j0 + 3, Lk - 1);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int c = 0; c < D; ++c) {
      const float x = X[i][c];
      a0 += x * Y[j0][c];
      a1 += x * Y[j1][c];
      a2 += x * Y[j2][c];
      a3 += x * Y[j3][c];
    }
    Sout[i][j0] = a0 * scale;
    if (j0 + 1 < Lk) Sout[i][j0 + 1] = a1 * scale;
    if (j0 + 2 < Lk) Sout[i][j0 + 2] = a2 * scale;
    if (j0 + 3 < Lk) Sout[i][j0 + 3] = a3 * scale;
  }
}

__global__ __launch_bounds__(256) void attn_small_fwd_vec_kernel(int H, int Lq, int Lk, int D, float scale,
                                                                 const bf16* __restrict__ q, long long ldq,
                                                                 const bf16* __restrict__ k, long long ldk,
                                                                 const bf16* __restrict__ v, long long ldv,
                                                                 const float* __restrict__ mask, long long msb,
                                                                 long long msh, long long msi, long long msj,
                                                                 bf16* __restrict__ out, long long ldo,
                                                                 bf16* __restrict__ w, long long ldw) {
  __shared__ float Q[SM_MAX_L][SM_MAX_D + 1], K[SM_MAX_L][SM_MAX_D + 1], V[SM_MAX_L][SM_MAX_D + 1];
  __shared__ float P[SM_MAX_L][SM_MAX_L + 1];
  const int b = blockIdx.x, h = blockIdx.y, t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int dch = D >> 3, r = t / dch, c0 = (t - r * dch) * 8;
  const bool hq = r < Lq, hk = r < Lk;
  bf16x8 rq, rk, rv;
  if (hq) rq = *(const bf16x8*)(q + ((long long)b * Lq + r) * ldq + h * D + c0);
  if (hk) {
    rk = *(const bf16x8*)(k + ((long long)b * Lk + r) * ldk + h * D + c0);
    rv = *(const bf16x8*)(v + ((long long)b * Lk + r) * ldv + h * D + c0);
  }
  if (hq) sm_put8(&Q[r][c0], rq);
  if (hk) {
    sm_put8(&K[r][c0], rk);
    sm_put8(&V[r][c0], rv);
  }
  __syncthreads();
  sm_strips(Q, K, P, Lq, Lk, D, scale);
  __syncthreads();
  const float* mb = mask ? mask + (long long)b * msb + (long long)h * msh : nullptr;
  bf16* wb = w + ((long long)b * H + h) * Lq * ldw;
  for (int i = wave; i < Lq; i += 4) {
    float s = -INFINITY;
    if (lane < Lk) {
      s = P[i][lane];
      if (mb) s += mb[(long long)i * msi + (long long)lane * msj] * -1e9f;
    }
    const float mx = wave_max(s);
    const float ex = lane < Lk ? expf(s - mx) : 0.f;
    const float sum = wave_sum(ex);
    const bf16 pt = from_f32<bf16>(lane < Lk ? ex * (1.f / sum) : 0.f);
    if (lane < (int)ldw) wb[(long long)i * ldw + lane] = pt;
    if (lane < Lk) P[i][lane] = to_f32(pt);
  }
  __syncthreads();
  for (int e = t; e < Lq * dch; e += 256) {
    const int i = e / dch, cc = (e - i * dch) * 8;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < Lk; ++j) {
      const float p = P[i][j];
#pragma unroll
      for (int u = 0; u < 8; ++u) o[u] += p * V[j][cc + u];
    }
    *(bf16x8*)(out + ((long long)b * Lq + i) * ldo + h * D + cc) = sm_pack8(o);
  }
}

__global__ __launch_bounds__(256) void attn_small_bwd_vec_kernel(int H, int Lq, int Lk, int D, float scale,
                                                                 const bf16* __restrict__ q, long long ldq,
                                                                 const bf16* __restrict__ k, long long ldk,
                                                                 const bf16* __restrict__ v, long long ldv,
                                                                 const bf16* __restrict__ w, long long ldw,
                                                                 const bf16* __restrict__ dout, long long ldo,
                                                                 bf16* __restrict__ dq, bf16* __restrict__ dk,
                                                                 bf16* __restrict__ dv) {
  __shared__ float Q[SM_MAX_L][SM_MAX_D + 1], K[SM_MAX_L][SM_MAX_D + 1], V[SM_MAX_L][SM_MAX_D + 1],
      G[SM_MAX_L][SM_MAX_D + 1];
  __shared__ float P[SM_MAX_L][SM_MAX_L + 1], dS[SM_MAX_L][SM_MAX_L + 1];
  const int b = blockIdx.x, h = blockIdx.y, t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int dch = D >> 3, r = t / dch, c0 = (t - r * dch) * 8;
  const bool hq = r < Lq, hk = r < Lk;
  const int wch = (int)(ldw >> 3), pr = t / wch, pc = (t - pr * wch) * 8;  // weights: ldw / 8 chunks per row
  const bool hp = pr < Lq;
  const bf16* wb = w + ((long long)b * H + h) * Lq * ldw;
  bf16x8 rq, rk, rv, rg, rp;
  if (hq) {
    rq = *(const bf16x8*)(q + ((long long)b * Lq + r) * ldq + h * D + c0);
    rg = *(const bf16x8*)(dout + ((long long)b * Lq + r) * ldo + h * D + c0);
  }
  if (hk) {
    rk = *(const bf16x8*)(k + ((long long)b * Lk + r) * ldk + h * D + c0);
    rv = *(const bf16x8*)(v + ((long long)b * Lk + r) * ldv + h * D + c0);
  }
  if (hp) rp = *(const bf16x8*)(wb + (long long)pr * ldw + pc);
  if (hq) {
    sm_put8(&Q[r][c0], rq);
    sm_put8(&G[r][c0], rg);
  }
  if (hk) {
    sm_put8(&K[r][c0], rk);
    sm_put8(&V[r][c0], rv);
  }
  if (hp)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (pc + e < Lk) P[pr][pc + e] = (float)rp[e];
  __syncthreads();
  sm_strips(G, V, dS, Lq, Lk, D, 1.f);  // dP = dO V^T
  __syncthreads();
  for (int i = wave; i < Lq; i += 4) {
    const float pj = lane < Lk ? P[i][lane] : 0.f, dpj = lane < Lk ? dS[i][lane] : 0.f;
    const float dot = wave_sum(pj * dpj);
    if (lane < Lk) dS[i][lane] = to_f32(from_f32<bf16>(pj * (dpj - dot)));
  }
  __syncthreads();
  for (int e = t; e < Lq * dch; e += 256) {  // dQ = scale dS K
    const int i = e / dch, cc = (e - i * dch) * 8;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < Lk; ++j) {
      const float x = dS[i][j];
#pragma unroll
      for (int u = 0; u < 8; ++u) o[u] += x * K[j][cc + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] *= scale;
    *(bf16x8*)(dq + ((long long)b * Lq + i) * ldq + h * D + cc) = sm_pack8(o);
  }
  for (int e = t; e < Lk * dch; e += 256) {  // dK = scale dS^T Q, dV = P^T dO
    const int j = e / dch, cc = (e - j * dch) * 8;
    float ok[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ov[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < Lq; ++i) {
      const float x = dS[i][j], p = P[i][j];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        ok[u] += x * Q[i][cc + u];
        ov[u] += p * G[i][cc + u];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) ok[u] *= scale;
    *(bf16x8*)(dk + ((long long)b * Lk + j) * ldk + h * D + cc) = sm_pack8(ok);
    *(bf16x8*)(dv + ((long long)b * Lk + j) * ldv + h * D + cc) = sm_pack8(ov);
  }
}

// MFMA form of attn_small_fwd_vec_kernel for D = 64 (the decoder's T = 31
// self-attention and its cross-attention): one wave per (image, head).
//   S^T = K Q^T  (32 keys x 32 queries, 4 x v_mfma_f32_32x32x16_bf16; both
//                 fragments are 16-B row loads straight from global memory)
//   key j of query i sits in lane i (& 31), register-row j, so the softmax
//   over j is 16 registers + one lane-half exchange;
//   O^T = V^T P^T (2 d-tiles x 2 k-steps; V^T gathered from V rows staged in
//                 LDS): P^T is the accumulator itself,
//   rounded to bf16 (the stored weights, as the GEMM path uses them) and fed
//   as the B operand with no lane movement (its k order is the accumulator's
//   row order: element e of lane half h in k-step s is key 16s + 8(e>>2) +
//   4h + (e&3), so the V^T fragment gathers those keys).
// Same semantics as the VALU kernel: scale after the dot, additive -1e9
// mask, weights rounded to bf16 and zero-filled up to ldw.
__global__ __launch_bounds__(64) void attn_small_fwd_mfma_kernel(int H, int Lq, int Lk, float scale,
                                                                 const bf16* __restrict__ q, long long ldq,
                                                                 const bf16* __restrict__ k, long long ldk,
                                                                 const bf16* __restrict__ v, long long ldv,
                                                                 const float* __restrict__ mask, long long msb,
                                                                 long long msh, long long msi, long long msj,
                                                                 bf16* __restrict__ out, long long ldo,
                                                                 bf16* __restrict__ w, long long ldw) {
  const int b = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const int r = lane & 31, hf = lane >> 5;
  const bf16x8 zero8 = {};
  // fragments: A = K rows (key r), B = Q rows (query r), k = 16 s + 8 hf + e
  bf16x8 ka[4], qb[4];
  const bf16* kr = k + ((long long)b * Lk + min(r, Lk - 1)) * ldk + h * 64 + 8 * hf;
  const bf16* qr = q + ((long long)b * Lq + min(r, Lq - 1)) * ldq + h * 64 + 8 * hf;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    ka[s2] = *(const bf16x8*)(kr + 16 * s2);
    qb[s2] = *(const bf16x8*)(qr + 16 * s2);
  }
  if (r >= Lk)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) ka[s2] = zero8;
  // V^T fragments (gathered keys, column d = r of each 32-wide d-tile) from
  // V rows staged in LDS by 16-B loads (rows past Lk zero)
  __shared__ bf16x8 sV[32][8];
  const bf16* vb = v + (long long)b * Lk * ldv + h * 64;
#pragma unroll
  for (int c = 0; c < 4; ++c) sV[r][4 * hf + c] = r < Lk ? *(const bf16x8*)(vb + (long long)r * ldv + 8 * (4 * hf + c)) : zero8;
  __syncthreads();
  bf16x8 va[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = 16 * s2 + 8 * (e >> 2) + 4 * hf + (e & 3);
        const int d = 32 * t + r;
        va[t][s2][e] = sV[j][d >> 3][d & 7];
      }
  f32x16 st = {};
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[s2], qb[s2], st, 0, 0, 0);
  // row j of register g: j = (g & 3) + 8 (g >> 2) + 4 hf; column = query i = r
  const int i = r;
  const float* mb = mask ? mask + (long long)b * msb + (long long)h * msh + (long long)i * msi : nullptr;
  float mx = -INFINITY;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int j = (g & 3) + 8 * (g >> 2) + 4 * hf;
    float x = st[g] * scale;
    if (mb && j < Lk && i < Lq) x += mb[(long long)j * msj] * -1e9f;
    x = j < Lk ? x : -INFINITY;
    st[g] = x;
    mx = fmaxf(mx, x);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float e = st[g] == -INFINITY ? 0.f : expf(st[g] - mx);
    st[g] = e;
    sum += e;
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  bf16x8 pb[2];
  bf16* wrow = w + (((long long)b * H + h) * Lq + i) * ldw;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int j = (g & 3) + 8 * (g >> 2) + 4 * hf;
    const bf16 pt = (bf16)(j < Lk ? st[g] * inv : 0.f);
    pb[g >> 3][g & 7] = pt;
    if (i < Lq && j < (int)ldw) wrow[j] = pt;
  }
  f32x16 o[2] = {};
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[t][s2], pb[s2], o[t], 0, 0, 0);
  // O^T tile t: row d = 32 t + (g & 3) + 8 (g >> 2) + 4 hf, column i = r
  if (i < Lq) {
    bf16* orow = out + ((long long)b * Lq + i) * ldo + h * 64;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
        u16x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = __builtin_bit_cast(unsigned short, (bf16)o[t][4 * g4 + e]);
        *(u16x4*)(orow + 32 * t + 8 * g4 + 4 * hf) = pk;
      }
  }
}

// MFMA form of attn_small_bwd_vec_kernel for D = 64, one wave per (image,
// head). Two orientations of dP are formed so that every later product sums
// over its accumulator's ROW index (the operand-from-accumulator rule of
// attn_small_fwd_mfma_kernel, no lane movement):
//   dP^T = V dO^T  (rows j: with P^T, rowsum_i and dS^T; dQ^T = K^T dS^T)
//   dP   = dO V^T  (rows i: with P, dS;                  dK^T = Q^T dS)
//   dV^T = dO^T P  (P gathered straight into the B-fragment order)
// dS is rounded to bf16 before the products (as the GEMM path), dQ and dK
// scaled after the sum, outputs stored as 8-B runs of 4 columns. (P^T rows
// are unpacked from 8-B loads with shifts: __builtin_bit_cast of a u16
// vector element to bf16 returned element 0 for every element here.)
__global__ __launch_bounds__(64) void attn_small_bwd_mfma_kernel(int H, int Lq, int Lk, float scale,
                                                                 const bf16* __restrict__ q, long long ldq,
                                                                 const bf16* __restrict__ k, long long ldk,
                                                                 const bf16* __restrict__ v, long long ldv,
                                                                 const bf16* __restrict__ w, long long ldw,
                                                                 const bf16* __restrict__ dout, long long ldo,
                                                                 bf16* __restrict__ dq, bf16* __restrict__ dk,
                                                                 bf16* __restrict__ dv) {
  typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  const int b = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const int r = lane & 31, hf = lane >> 5;
  const bf16x8 zero8 = {};
  const long long qo = (long long)b * Lq * ldq + h * 64, ko = (long long)b * Lk * ldk + h * 64;
  const long long vo = (long long)b * Lk * ldv + h * 64, go = (long long)b * Lq * ldo + h * 64;
  const bf16* wb = w + ((long long)b * H + h) * Lq * ldw;
  // row fragments (16-B loads): V rows (key r), dO rows (query r)
  bf16x8 vrow[4], grow[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    vrow[s2] = *(const bf16x8*)(v + vo + (long long)min(r, Lk - 1) * ldv + 16 * s2 + 8 * hf);
    grow[s2] = *(const bf16x8*)(dout + go + (long long)min(r, Lq - 1) * ldo + 16 * s2 + 8 * hf);
  }
  if (r >= Lk)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) vrow[s2] = zero8;
  if (r >= Lq)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) grow[s2] = zero8;
  // accumulator row of register g (either orientation)
  auto arow = [&](int g) { return (g & 3) + 8 * (g >> 2) + 4 * hf; };
  // ---- dP^T (rows j = arow, column i = r) and P^T -------------------------
  f32x16 dpt = {};
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vrow[s2], grow[s2], dpt, 0, 0, 0);
  float pt[16];
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int j0 = 8 * g4 + 4 * hf;
    u32x2 pk = {0u, 0u};
    if (r < Lq && j0 + 4 <= (int)ldw) pk = *(const u32x2*)(wb + (long long)r * ldw + j0);
    pt[4 * g4 + 0] = __uint_as_float(pk[0] << 16);
    pt[4 * g4 + 1] = __uint_as_float(pk[0] & 0xffff0000u);
    pt[4 * g4 + 2] = __uint_as_float(pk[1] << 16);
    pt[4 * g4 + 3] = __uint_as_float(pk[1] & 0xffff0000u);
  }
  float rs = 0.f;
#pragma unroll
  for (int g = 0; g < 16; ++g) rs += pt[g] * dpt[g];
  rs += __shfl_xor(rs, 32, 64);  // rowsum of query i = r (both lane halves)
  bf16x8 dst[2];                  // dS^T as the B operand (k = j)
#pragma unroll
  for (int g = 0; g < 16; ++g) dst[g >> 3][g & 7] = (bf16)(pt[g] * (dpt[g] - rs));
  // ---- dP (rows i = arow, column j = r) and P -----------------------------
  f32x16 dp = {};
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(grow[s2], vrow[s2], dp, 0, 0, 0);
  bf16x8 ds[2], pj[2];
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int i = arow(g);
    const bf16 pv = (i < Lq && r < (int)ldw) ? wb[(long long)i * ldw + r] : (bf16)0.f;
    const float rsi = __shfl(rs, i, 64);
    pj[g >> 3][g & 7] = pv;
    ds[g >> 3][g & 7] = (bf16)((float)pv * (dp[g] - rsi));
  }
  // ---- gathered A operands X^T[d = r][k-slot] for the three products, from
  // K / Q / dO rows staged in LDS by 16-B loads (rows past Lk / Lq zero):
  // k-slot (s, e) of lane half hf = accumulator row 16 s + 8 (e >> 2) + 4 hf + (e & 3)
  __shared__ bf16x8 sK[32][8], sQ[32][8], sG[32][8];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int dc = 4 * hf + c;  // 8-column chunk
    sK[r][dc] = r < Lk ? *(const bf16x8*)(k + ko + (long long)r * ldk + 8 * dc) : zero8;
    sQ[r][dc] = r < Lq ? *(const bf16x8*)(q + qo + (long long)r * ldq + 8 * dc) : zero8;
    sG[r][dc] = r < Lq ? *(const bf16x8*)(dout + go + (long long)r * ldo + 8 * dc) : zero8;
  }
  __syncthreads();
  f32x16 dqt[2] = {}, dkt[2] = {}, dvt[2] = {};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int d = 32 * t + r;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 kt, qt, gt;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int x = 16 * s2 + 8 * (e >> 2) + 4 * hf + (e & 3);
        kt[e] = sK[x][d >> 3][d & 7];
        qt[e] = sQ[x][d >> 3][d & 7];
        gt[e] = sG[x][d >> 3][d & 7];
      }
      dqt[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt, dst[s2], dqt[t], 0, 0, 0);  // sum over j
      dkt[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qt, ds[s2], dkt[t], 0, 0, 0);   // sum over i
      dvt[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gt, pj[s2], dvt[t], 0, 0, 0);   // sum over i
    }
  }
  // ---- stores: column (query i or key j) = r, rows d = 32 t + 8 g4 + 4 hf + e
  auto put = [&](bf16* base, long long ld, const f32x16 (&acc)[2], float sc) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        u16x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = __builtin_bit_cast(unsigned short, (bf16)(sc * acc[t][4 * g4 + e]));
        *(u16x4*)(base + (long long)r * ld + 32 * t + 8 * g4 + 4 * hf) = pk;
      }
  };
  if (r < Lq) put(dq + qo, ldq, dqt, scale);
  if (r < Lk) {
    put(dk + ko, ldk, dkt, scale);
    put(dv + vo, ldv, dvt, 1.f);
  }
}

static bool small_vec(const fpnmt_attn_desc* d, std::initializer_list<const void*> ptrs) {
  if (d->dtype != FPNMT_BF16 || d->d % 8 || d->ldq % 8 || d->ldk % 8 || d->ldv % 8 || d->ldo % 8 || d->ldw % 8 ||
      d->ldw > SM_MAX_L)
    return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p & 15) return false;
  return true;
}

bool attn_small_ok(const fpnmt_attn_desc* d) {
  return d->lq >= 1 && d->lq <= SM_MAX_L && d->lk >= 1 && d->lk <= SM_MAX_L && d->d <= SM_MAX_D && d->h <= 65535 &&
         d->b <= 2147483647 && d->ldw <= 64;
}

int attn_small_fwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const float* mask, void* out,
                   void* weights, hipStream_t s) {
  const dim3 grid(d->b, d->h);
  if (d->d == 64 && small_vec(d, {q, k, v, out, weights}))
    hipLaunchKernelGGL(attn_small_fwd_mfma_kernel, grid, dim3(64), 0, s, d->h, d->lq, d->lk, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, mask, d->m_sb, d->m_sh,
                       d->m_si, d->m_sj, (bf16*)out, d->ldo, (bf16*)weights, d->ldw);
  else if (small_vec(d, {q, k, v, out, weights}))
    hipLaunchKernelGGL(attn_small_fwd_vec_kernel, grid, dim3(256), 0, s, d->h, d->lq, d->lk, d->d, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, mask, d->m_sb, d->m_sh,
                       d->m_si, d->m_sj, (bf16*)out, d->ldo, (bf16*)weights, d->ldw);
  else if (d->dtype == FPNMT_BF16)
    hipLaunchKernelGGL((attn_small_fwd_kernel<bf16>), grid, dim3(256), 0, s, d->h, d->lq, d->lk, d->d, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, mask, d->m_sb, d->m_sh,
                       d->m_si, d->m_sj, (bf16*)out, d->ldo, (bf16*)weights, d->ldw);
  else
    hipLaunchKernelGGL((attn_small_fwd_kernel<float>), grid, dim3(256), 0, s, d->h, d->lq, d->lk, d->d, d->scale,
                       (const float*)q, d->ldq, (const float*)k, d->ldk, (const float*)v, d->ldv, mask, d->m_sb,
                       d->m_sh, d->m_si, d->m_sj, (float*)out, d->ldo, (float*)weights, d->ldw);
  return check_launch("attention_small_fwd");
}

int attn_small_bwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const void* weights,
                   const void* dout, void* dq, void* dk, void* dv, hipStream_t s) {
  const dim3 grid(d->b, d->h);
  if (d->d == 64 && small_vec(d, {q, k, v, weights, dout, dq, dk, dv}))
    hipLaunchKernelGGL(attn_small_bwd_mfma_kernel, grid, dim3(64), 0, s, d->h, d->lq, d->lk, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, (const bf16*)weights,
                       d->ldw, (const bf16*)dout, d->ldo, (bf16*)dq, (bf16*)dk, (bf16*)dv);
  else if (small_vec(d, {q, k, v, weights, dout, dq, dk, dv}))
    hipLaunchKernelGGL(attn_small_bwd_vec_kernel, grid, dim3(256), 0, s, d->h, d->lq, d->lk, d->d, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, (const bf16*)weights,
                       d->ldw, (const bf16*)dout, d->ldo, (bf16*)dq, (bf16*)dk, (bf16*)dv);
  else if (d->dtype == FPNMT_BF16)
    hipLaunchKernelGGL((attn_small_bwd_kernel<bf16>), grid, dim3(256), 0, s, d->h, d->lq, d->lk, d->d, d->scale,
                       (const bf16*)q, d->ldq, (const bf16*)k, d->ldk, (const bf16*)v, d->ldv, (const bf16*)weights,
                       d->ldw, (const bf16*)dout, d->ldo, (bf16*)dq, (bf16*)dk, (bf16*)dv);
  else
    hipLaunchKernelGGL((attn_small_bwd_kernel<float>), grid, dim3(256), 0, s, d->h, d->lq, d->lk, d->d, d->scale,
                       (const float*)q, d->ldq, (const float*)k, d->ldk, (const float*)v, d->ldv,
                       (const float*)weights, d->ldw, (const float*)dout, d->ldo, (float*)dq, (float*)dk, (float*)dv);
  return check_launch("attention_small_bwd");
}

}  // namespace fpnmt
