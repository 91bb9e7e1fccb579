// Weight compute-copy preparation and the fused Keras-AMSGrad optimizer step.
//
// fpnmt_weight_prep: fp32 HWIO master -> OHWI (forward B operand) and flipped
//   IHWO (backward-data B operand) in the compute dtype, frozen-BN scale folded.
// fpnmt_grad_sumsq / fpnmt_amsgrad_step: per-tensor clip_by_norm (TF >= 2.4
//   OptimizerV2 semantics, utils/pipeline.py:30) + ResourceApplyAdamWithAmsgrad
//   over a flat parameter arena, lr from CustomSchedule (utils/utils.py:45-50)
//   evaluated on the device-resident `iterations` counter (graph-replay safe).
#include "common.h"

namespace fpnmt {

// OHWI: dst[k][r][s][c] = src[r][s][c][k]*scale[k]   (tiled 32x32 transpose of
// the (c,k) plane for every (r,s))
template <typename T>
__global__ __launch_bounds__(256) void wprep_ohwi_kernel(const float* __restrict__ src, int rs, int c, int k,
                                                         const float* __restrict__ scale, T* __restrict__ dst) {
  __shared__ float tile[32][33];
  const int rsi = blockIdx.z;
  const int c0 = blockIdx.y * 32, k0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const float* s = src + (long long)rsi * c * k;
  for (int yy = ty; yy < 32; yy += 8) {
    const int cc = c0 + yy, kk = k0 + tx;
    tile[yy][tx] = (cc < c && kk < k) ? s[(long long)cc * k + kk] * (scale ? scale[kk] : 1.f) : 0.f;
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    const int kk = k0 + yy, cc = c0 + tx;
    if (kk < k && cc < c) dst[((long long)kk * rs + rsi) * c + cc] = from_f32<T>(tile[tx][yy]);
  }
}

// flipped IHWO: dst[c][R-1-r][S-1-s][k] = src[r][s][c][k]*scale[k]  (k-contiguous copy)
template <typename T>
__global__ void wprep_flip_kernel(const float* __restrict__ src, int R, int Sd, int c, int k,
                                  const float* __restrict__ scale, T* __restrict__ dst, long long ldf) {
  const long long total = (long long)R * Sd * c * k;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % k);
    long long t = i / k;
    const int cc = (int)(t % c);
    t /= c;
    const int ss = (int)(t % Sd);
    const int rr = (int)(t / Sd);
    const long long o = (long long)cc * ldf + ((long long)(R - 1 - rr) * Sd + (Sd - 1 - ss)) * k + kk;
    dst[o] = from_f32<T>(src[i] * (scale ? scale[kk] : 1.f));
  }
}

// Batched prep: block = one 32x32 (c,k) tile of one (item, r, s); the tile is
// staged through LDS once and written to both the OHWI and flipped copies.
// Each thread owns four adjacent columns of a row: bf16 quads go out as one
// 8-B store when the destination is 8-B aligned (a quarter of the stores of
// one element per thread; 2-B stores were the kernel's limit).
template <typename T>
__device__ __forceinline__ void wprep_store4(T* d, const float (&v)[4], int valid) {
  if (sizeof(T) == 2 && valid == 4 && ((uintptr_t)d & 7) == 0) {
    typedef __attribute__((ext_vector_type(4))) T T4;
    T4 pv;
#pragma unroll
    for (int e = 0; e < 4; ++e) pv[e] = from_f32<T>(v[e]);
    *(T4*)d = pv;
  } else {
    for (int e = 0; e < valid; ++e) d[e] = from_f32<T>(v[e]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void wprep_batched_kernel(const fpnmt_wprep_item* __restrict__ items, int n) {
  __shared__ float tile[32][33];
  __shared__ int s_item;
  const long long b = blockIdx.x;
  if (threadIdx.x == 0) {
    int lo = 0, hi = n - 1;  // last item with tile_start <= b
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (items[mid].tile_start <= b) lo = mid; else hi = mid - 1;
    }
    s_item = lo;
  }
  __syncthreads();
  const fpnmt_wprep_item it = items[s_item];
  long long t = b - it.tile_start;
  const int tc = (it.c + 31) / 32, tk = (it.k + 31) / 32;
  const int kt = (int)(t % tk);
  t /= tk;
  const int ct = (int)(t % tc);
  const int rsi = (int)(t / tc);
  const int rr = rsi / it.s, ss = rsi % it.s;
  const int c0 = ct * 32, k0 = kt * 32;
  const int tx = (threadIdx.x & 7) * 4, ty = threadIdx.x >> 3;  // 8 column quads x 32 rows
  const float* src = it.w_hwio + (long long)rsi * it.c * it.k;
  const long long ldf = it.ld_flip ? it.ld_flip : (long long)it.r * it.s * it.k;
  {
    const int cc = c0 + ty, kk = k0 + tx;
    const int valid = cc < it.c ? max(0, min(4, it.k - kk)) : 0;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = e < valid ? src[(long long)cc * it.k + kk + e] * (it.scale ? it.scale[kk + e] : 1.f) : 0.f;
    if (it.w_flip && valid > 0)  // flipped IHWO: k contiguous, written straight from the read
      wprep_store4<T>((T*)it.w_flip + (long long)cc * ldf +
                          ((long long)(it.r - 1 - rr) * it.s + (it.s - 1 - ss)) * it.k + kk, v, valid);
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[ty][tx + e] = v[e];
  }
  __syncthreads();
  if (it.w_ohwi) {
    const int rs = it.r * it.s;
    const int kk = k0 + ty, cc = c0 + tx;
    const int valid = kk < it.k ? max(0, min(4, it.c - cc)) : 0;
    if (valid > 0) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = tile[tx + e][ty];
      wprep_store4<T>((T*)it.w_ohwi + ((long long)kk * rs + rsi) * it.c + cc, v, valid);
    }
  }
}

// Per-block partial ||g||^2 (block = a <= block_elems run of one segment);
// amsgrad_kernel sums a segment's partials in block order (no atomics: the
// clip factor, and so every update, is the same on every run).
__device__ __forceinline__ void sumsq_block(int blk, const int32_t* __restrict__ blk_seg,
                                            const long long* __restrict__ blk_start, int block_elems,
                                            const long long* __restrict__ off, const int32_t* __restrict__ seg_flags,
                                            const float* __restrict__ g, float gs, float* __restrict__ blk_part,
                                            float* red) {
  const int seg = blk_seg[blk];
  if (seg_flags && (seg_flags[seg] & 1)) return;
  const long long b0 = blk_start[blk];
  const long long b1 = min(b0 + block_elems, off[seg + 1]);
  // block starts are 4-element aligned (arena ALIGN / BLOCK_ELEMS): float4 body, scalar tail
  float s = 0.f;
  const long long nv = (b1 - b0) >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g + b0);
  for (long long i = threadIdx.x; i < nv; i += 256) {
    const float4 q = g4[i];
    const float a = q.x * gs, b = q.y * gs, c = q.z * gs, e = q.w * gs;
    s += a * a + b * b + c * c + e * e;
  }
  for (long long i = b0 + (nv << 2) + threadIdx.x; i < b1; i += 256) {
    const float v = g[i] * gs;
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) blk_part[blk] = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();  // red is reused by the block's next arena block
}

// one workgroup per arena block, or a persistent grid striding over them
// (gridDim.x < nblocks: the early optimizer part beside a running backward)
__global__ __launch_bounds__(256) void sumsq_kernel(int blk_first, int nblocks, const int32_t* __restrict__ blk_seg,
                                                    const long long* __restrict__ blk_start, int block_elems,
                                                    const long long* __restrict__ off,
                                                    const int32_t* __restrict__ seg_flags,
                                                    const float* __restrict__ g, float gs,
                                                    float* __restrict__ blk_part) {
  __shared__ float red[4];
  for (int b = (int)blockIdx.x; b < nblocks; b += (int)gridDim.x)
    sumsq_block(blk_first + b, blk_seg, blk_start, block_elems, off, seg_flags, g, gs, blk_part, red);
}

__device__ __forceinline__ float sched_lr(const fpnmt_adam_desc& d, float step) {
  if (d.sched_d_model <= 0.f) return d.const_lr;
  const float arg1 = rsqrtf(step) / fmaxf((step - d.sched_warmup) * d.sched_mult / (d.sched_warmup * 2.f), 1.f);
  const float arg2 = step * d.sched_warm_pow;
  return rsqrtf(d.sched_d_model) * fminf(arg1, arg2);
}

// Fused compute-copy refresh (PREP): a block of a conv / dense kernel segment
// (HWIO, k a power of two in [16, 4096], block_elems a multiple of k) covers
// whole k-rows q = (r*S + s)*C + c. Each thread writes the flipped copy of
// its float4 straight from registers (k-contiguous, 8-B stores) and parks the
// bf16 values in LDS ([row][k + 2]: the 4-B pad staggers the banks of the
// column reads below); after one barrier the block writes the OHWI copy
// (ohwi[kk][q], q-contiguous runs of the block's rows) from LDS.
constexpr int PREP_LDS = 16384 + 2 * 1024;  // bf16 elements: 16384 values + 2 per row (>= 16 per row)

__device__ __forceinline__ uint32_t prep_div_c(uint32_t q, const fpnmt_seg_prep& pp) {
  return (uint32_t)(((((uint64_t)q * pp.c_magic) >> 32) + q) >> pp.c_shift);
}

template <bool PREP>
__device__ __forceinline__ void amsgrad_block(const fpnmt_adam_desc& d, int blk, const int32_t* __restrict__ blk_seg,
                                              const long long* __restrict__ blk_start, int block_elems,
                                              const long long* __restrict__ off,
                                              const int32_t* __restrict__ seg_flags, float* __restrict__ param,
                                              const float* __restrict__ grad, float* __restrict__ m,
                                              float* __restrict__ v, float* __restrict__ vhat,
                                              const float* __restrict__ sumsq, const float* __restrict__ blk_part,
                                              const int32_t* __restrict__ seg_blk0,
                                              const long long* __restrict__ step,
                                              const fpnmt_seg_prep* __restrict__ preps, float& s_ss,
                                              unsigned short* s_prep) {
  const int seg = blk_seg[blk];
  const bool sparse_norm = seg_flags && (seg_flags[seg] & 1);
  if (d.clipnorm > 0.f && !sparse_norm && threadIdx.x < 64) {
    // the segment's ||g||^2: its blocks' partials in block order (wave 0)
    float t = 0.f;
    for (int b = seg_blk0[seg] + threadIdx.x; b < seg_blk0[seg + 1]; b += 64) t += blk_part[b];
    t = wave_sum(t);
    if (threadIdx.x == 0) s_ss = t;
  }
  __syncthreads();
  const long long b0 = blk_start[blk];
  const long long b1 = min(b0 + block_elems, off[seg + 1]);
  const float it = (float)(*step);
  const float lr = sched_lr(d, it);
  const float t = it + 1.f;
  const float b1p = powf(d.beta1, t), b2p = powf(d.beta2, t);
  const float alpha = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  // tf.clip_by_norm: g * clip / max(||g||, clip)  (||g|| = 0 -> factor 1)
  const float ss = d.clipnorm > 0.f ? (sparse_norm ? sumsq[seg] * d.grad_scale * d.grad_scale : s_ss) : 0.f;
  const float nrm = ss > 0.f ? sqrtf(ss) : 0.f;
  const bool sparse_form = seg_flags && (seg_flags[seg] & 2);
  auto upd = [&](float gr, float& pi, float& mi, float& vi, float& hi) {
    gr *= d.grad_scale;
    // per element as TF rounds it: (t * clip) / max(norm, clip), not t * factor
    const float g = d.clipnorm > 0.f ? (gr * d.clipnorm) / fmaxf(nrm, d.clipnorm) : gr;
    if (sparse_form) {
      mi = mi * d.beta1 + g * (1.f - d.beta1);
      vi = vi * d.beta2 + (g * g) * (1.f - d.beta2);
    } else {
      mi = mi + (g - mi) * (1.f - d.beta1);
      vi = vi + (g * g - vi) * (1.f - d.beta2);
    }
    hi = fmaxf(hi, vi);
    pi = pi - (mi * alpha) / (sqrtf(hi) + d.eps);
  };
  // float4 body (block starts are 4-element aligned), U vectors per thread in
  // flight per array (all 5U loads issued before the first use); streaming
  // (non-temporal) loads and stores: nothing here is re-read before the next
  // step. Scalar tail for the last < 4 elements of a segment.
  constexpr int U = 4;
  const long long nv = (b1 - b0) >> 2;
  float4* p4 = reinterpret_cast<float4*>(param + b0);
  const float4* g4 = reinterpret_cast<const float4*>(grad + b0);
  float4* m4 = reinterpret_cast<float4*>(m + b0);
  float4* v4 = reinterpret_cast<float4*>(v + b0);
  float4* h4 = reinterpret_cast<float4*>(vhat + b0);
  typedef __attribute__((ext_vector_type(4))) float nf4;
  auto ld = [](const float4* a) {
    const nf4 q = __builtin_nontemporal_load((const nf4*)a);
    return make_float4(q[0], q[1], q[2], q[3]);
  };
  auto st = [](float4* a, const float4& q) {
    const nf4 w = {q.x, q.y, q.z, q.w};
    __builtin_nontemporal_store(w, (nf4*)a);
  };
  // compute-copy refresh of this block (uniform per block)
  fpnmt_seg_prep pp{};
  bool prep = false;
  int lk = 0;
  long long l0 = 0;
  if constexpr (PREP) {
    pp = preps[seg];
    prep = pp.ohwi != nullptr;
    if (prep) {
      lk = __builtin_ctz((unsigned)pp.k);
      l0 = b0 - blk_start[seg_blk0[seg]];  // block start within the segment (a multiple of k)
    }
  }
  const long long ldf = pp.ld_flip ? pp.ld_flip : (long long)pp.r * pp.s * pp.k;
  // (r, s) of a tap index rsi < r*s <= 2^16 / s by a multiply: one division per block
  const uint32_t inv_s = prep ? (65536u + (uint32_t)pp.s - 1u) / (uint32_t)pp.s : 0u;
  auto prep4 = [&](long long i, const float4& q4) {
    // element el = 4i of the block: row ql, column kk (kk % 4 == 0)
    const int el = (int)(i << 2);
    const int ql = el >> lk, kk = el & (pp.k - 1);
    float sc[4] = {1.f, 1.f, 1.f, 1.f};
    if (pp.scale) {
      const float4 t = *(const float4*)(pp.scale + kk);
      sc[0] = t.x; sc[1] = t.y; sc[2] = t.z; sc[3] = t.w;
    }
    const bf16 w0 = from_f32<bf16>(q4.x * sc[0]), w1 = from_f32<bf16>(q4.y * sc[1]);
    const bf16 w2 = from_f32<bf16>(q4.z * sc[2]), w3 = from_f32<bf16>(q4.w * sc[3]);
    const uint32_t q = (uint32_t)((l0 >> lk) + ql);
    const uint32_t rsi = prep_div_c(q, pp);
    const int cc = (int)(q - rsi * (uint32_t)pp.c);
    const int rr = (int)((rsi * inv_s) >> 16), ss = (int)rsi - rr * pp.s;
    if (pp.flip) {
      typedef __attribute__((ext_vector_type(4))) bf16 b4;
      const b4 w = {w0, w1, w2, w3};
      *(b4*)((bf16*)pp.flip + (long long)cc * ldf + ((long long)(pp.r - 1 - rr) * pp.s + (pp.s - 1 - ss)) * pp.k + kk) = w;
    }
    unsigned short* dl = s_prep + ql * (pp.k + 2) + kk;
    *(uint32_t*)dl = (uint32_t)__builtin_bit_cast(unsigned short, w0) |
                     ((uint32_t)__builtin_bit_cast(unsigned short, w1) << 16);
    *(uint32_t*)(dl + 2) = (uint32_t)__builtin_bit_cast(unsigned short, w2) |
                           ((uint32_t)__builtin_bit_cast(unsigned short, w3) << 16);
  };
  for (long long i0 = threadIdx.x; i0 < nv; i0 += 256 * U) {
    float4 G[U], P[U], M[U], V[U], H[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = min(i0 + 256LL * u, nv - 1);  // clamped: unconditional loads
      G[u] = ld(g4 + i); P[u] = ld(p4 + i); M[u] = ld(m4 + i); V[u] = ld(v4 + i); H[u] = ld(h4 + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + 256LL * u;
      if (i >= nv) break;
      upd(G[u].x, P[u].x, M[u].x, V[u].x, H[u].x);
      upd(G[u].y, P[u].y, M[u].y, V[u].y, H[u].y);
      upd(G[u].z, P[u].z, M[u].z, V[u].z, H[u].z);
      upd(G[u].w, P[u].w, M[u].w, V[u].w, H[u].w);
      st(m4 + i, M[u]); st(v4 + i, V[u]); st(h4 + i, H[u]); st(p4 + i, P[u]);
      if constexpr (PREP) {
        if (prep) prep4(i, P[u]);
      }
    }
  }
  if constexpr (PREP) {
    if (prep) {  // prep segments have no scalar tail (their length is a multiple of k >= 16)
      __syncthreads();
      const int n = (int)(b1 - b0), nr = n >> lk, ng = (nr + 3) >> 2;
      const long long RSC = (long long)pp.r * pp.s * pp.c;
      const long long q0 = l0 >> lk;
      const bool vec = (RSC & 3) == 0 && (q0 & 3) == 0 && ((uintptr_t)pp.ohwi & 7) == 0;
      // full blocks have ng = 4096 / k items per k-row: a power of two
      const int lng = (ng & (ng - 1)) == 0 ? __builtin_ctz((unsigned)ng) : -1;
      for (int w = threadIdx.x; w < pp.k * ng; w += 256) {
        const int kk = lng >= 0 ? w >> lng : w / ng;
        const int ql = (w - kk * ng) << 2;
        const int cnt = min(4, nr - ql);
        bf16* dst = (bf16*)pp.ohwi + kk * RSC + q0 + ql;
        unsigned short e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = j < cnt ? s_prep[(ql + j) * (pp.k + 2) + kk] : (unsigned short)0;
        if (vec && cnt == 4) {
          typedef __attribute__((ext_vector_type(4))) unsigned short u4;
          const u4 o = {e[0], e[1], e[2], e[3]};
          *(u4*)dst = o;
        } else {
          for (int j = 0; j < cnt; ++j) ((unsigned short*)dst)[j] = e[j];
        }
      }
      return;
    }
  }
  for (long long i = b0 + (nv << 2) + threadIdx.x; i < b1; i += 256) {
    float pi = param[i], mi = m[i], vi = v[i], hi = vhat[i];
    upd(grad[i], pi, mi, vi, hi);
    m[i] = mi;
    v[i] = vi;
    vhat[i] = hi;
    param[i] = pi;
  }
}

// one workgroup per arena block, or a persistent grid striding over them
// (gridDim.x < nblocks: the early optimizer part, no compute-copy refresh,
// sharing the CUs with a running backward)
template <bool PREP>
__global__ __launch_bounds__(256) void amsgrad_kernel(fpnmt_adam_desc d, int blk_first, int nblocks,
                                                      const int32_t* __restrict__ blk_seg,
                                                      const long long* __restrict__ blk_start, int block_elems,
                                                      const long long* __restrict__ off,
                                                      const int32_t* __restrict__ seg_flags, float* __restrict__ param,
                                                      const float* __restrict__ grad, float* __restrict__ m,
                                                      float* __restrict__ v, float* __restrict__ vhat,
                                                      const float* __restrict__ sumsq,
                                                      const float* __restrict__ blk_part,
                                                      const int32_t* __restrict__ seg_blk0,
                                                      const long long* __restrict__ step,
                                                      const fpnmt_seg_prep* __restrict__ preps) {
  __shared__ float s_ss;
  __shared__ unsigned short s_prep[PREP ? PREP_LDS : 1];
  for (int b = (int)blockIdx.x; b < nblocks; b += (int)gridDim.x) {
    if (b != (int)blockIdx.x) __syncthreads();  // the previous block's LDS reads are done
    amsgrad_block<PREP>(d, blk_first + b, blk_seg, blk_start, block_elems, off, seg_flags, param, grad, m, v, vhat,
                        sumsq, blk_part, seg_blk0, step, preps, s_ss, s_prep);
  }
}

__global__ void step_inc_kernel(long long* step) { *step += 1; }

}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

int fpnmt_weight_prep(const float* w_hwio, int r, int s, int c, int k, const float* scale, int dtype,
                      void* w_ohwi, void* w_flip, long long ld_flip, fpnmt_stream_t stream) {
  const long long ldf = ld_flip ? ld_flip : (long long)r * s * k;
  if (ldf < (long long)r * s * k) return fail(FPNMT_E_ARG, "weight_prep: ld_flip < r*s*k");
  if (!w_hwio || r <= 0 || s <= 0 || c <= 0 || k <= 0) return fail(FPNMT_E_ARG, "weight_prep: bad args");
  hipStream_t st = S(stream);
  if (w_ohwi) {
    dim3 grid(cdiv(k, 32), cdiv(c, 32), r * s);
    if (dtype == FPNMT_BF16)
      hipLaunchKernelGGL((wprep_ohwi_kernel<bf16>), grid, dim3(256), 0, st, w_hwio, r * s, c, k, scale, (bf16*)w_ohwi);
    else
      hipLaunchKernelGGL((wprep_ohwi_kernel<float>), grid, dim3(256), 0, st, w_hwio, r * s, c, k, scale, (float*)w_ohwi);
    int e = check_launch("weight_prep_ohwi");
    if (e) return e;
  }
  if (w_flip) {
    long long total = (long long)r * s * c * k;
    int g = (int)std::min<long long>(4096, (total + 255) / 256);
    if (dtype == FPNMT_BF16)
      hipLaunchKernelGGL((wprep_flip_kernel<bf16>), dim3(g), dim3(256), 0, st, w_hwio, r, s, c, k, scale, (bf16*)w_flip, ldf);
    else
      hipLaunchKernelGGL((wprep_flip_kernel<float>), dim3(g), dim3(256), 0, st, w_hwio, r, s, c, k, scale, (float*)w_flip, ldf);
    return check_launch("weight_prep_flip");
  }
  return 0;
}

int fpnmt_weight_prep_batched(const fpnmt_wprep_item* items_dev, int n_items, long long total_tiles, int dtype,
                              fpnmt_stream_t stream) {
  if (n_items <= 0 || total_tiles <= 0) return 0;
  if (!items_dev) return fail(FPNMT_E_ARG, "weight_prep_batched: null table");
  if (total_tiles >= (1LL << 31)) return fail(FPNMT_E_UNSUPPORTED, "weight_prep_batched: too many tiles");
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((wprep_batched_kernel<bf16>), dim3((unsigned)total_tiles), dim3(256), 0, S(stream), items_dev,
                       n_items);
  else
    hipLaunchKernelGGL((wprep_batched_kernel<float>), dim3((unsigned)total_tiles), dim3(256), 0, S(stream), items_dev,
                       n_items);
  return check_launch("weight_prep_batched");
}

int fpnmt_grad_sumsq_part(int blk_first, int nblocks, int max_grid, const int32_t* blk_seg,
                          const long long* blk_start, int block_elems, const long long* off,
                          const int32_t* seg_flags, const float* g, float grad_scale, float* blk_part,
                          fpnmt_stream_t stream) {
  if (nblocks <= 0) return 0;
  if (!blk_part) return fail(FPNMT_E_ARG, "grad_sumsq: null partials");
  if (blk_first < 0 || max_grid < 0) return fail(FPNMT_E_ARG, "grad_sumsq: negative first block / grid");
  const int grid = max_grid > 0 ? std::min(nblocks, max_grid) : nblocks;
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid), dim3(256), 0, S(stream), blk_first, nblocks, blk_seg, blk_start,
                     block_elems, off, seg_flags, g, grad_scale, blk_part);
  return check_launch("grad_sumsq");
}

int fpnmt_grad_sumsq(int nblocks, const int32_t* blk_seg, const long long* blk_start, int block_elems,
                     const long long* off, const int32_t* seg_flags, const float* g, float grad_scale,
                     float* blk_part, fpnmt_stream_t stream) {
  return fpnmt_grad_sumsq_part(0, nblocks, 0, blk_seg, blk_start, block_elems, off, seg_flags, g, grad_scale,
                               blk_part, stream);
}

int fpnmt_amsgrad_step_part(const fpnmt_adam_desc* d, int blk_first, int nblocks, int inc_step, int max_grid,
                            const int32_t* blk_seg, const long long* blk_start, int block_elems,
                            const long long* off, const int32_t* seg_flags, float* param, const float* grad,
                            float* m, float* v, float* vhat, const float* sumsq, const float* blk_part,
                            const int32_t* seg_blk0, long long* step, const fpnmt_seg_prep* preps,
                            fpnmt_stream_t stream) {
  if (!d || !step) return fail(FPNMT_E_ARG, "amsgrad: null");
  if (blk_first < 0 || max_grid < 0) return fail(FPNMT_E_ARG, "amsgrad: negative first block / grid");
  const int grid = max_grid > 0 ? std::min(nblocks, max_grid) : nblocks;
  if (d->clipnorm > 0.f && nblocks > 0 && (!blk_part || !seg_blk0 || !sumsq))
    return fail(FPNMT_E_ARG, "amsgrad: clipnorm needs the norms (sumsq, blk_part, seg_blk0)");
  if (preps && (!seg_blk0 || block_elems > 16384 || block_elems % 4096))
    return fail(FPNMT_E_ARG, "amsgrad_prep: needs seg_blk0 and block_elems a multiple of 4096 (<= 16384)");
  if (nblocks > 0) {
    if (preps)
      hipLaunchKernelGGL(amsgrad_kernel<true>, dim3(grid), dim3(256), 0, S(stream), *d, blk_first, nblocks, blk_seg,
                         blk_start, block_elems, off, seg_flags, param, grad, m, v, vhat, sumsq, blk_part, seg_blk0,
                         step, preps);
    else
      hipLaunchKernelGGL(amsgrad_kernel<false>, dim3(grid), dim3(256), 0, S(stream), *d, blk_first, nblocks, blk_seg,
                         blk_start, block_elems, off, seg_flags, param, grad, m, v, vhat, sumsq, blk_part, seg_blk0,
                         step, (const fpnmt_seg_prep*)nullptr);
  }
  if (inc_step) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, S(stream), step);
  return check_launch("amsgrad");
}

int fpnmt_amsgrad_step_prep(const fpnmt_adam_desc* d, int nblocks, const int32_t* blk_seg,
                            const long long* blk_start, int block_elems, const long long* off,
                            const int32_t* seg_flags, float* param, const float* grad, float* m, float* v,
                            float* vhat, const float* sumsq, const float* blk_part, const int32_t* seg_blk0,
                            long long* step, const fpnmt_seg_prep* preps, fpnmt_stream_t stream) {
  return fpnmt_amsgrad_step_part(d, 0, nblocks, 1, 0, blk_seg, blk_start, block_elems, off, seg_flags, param, grad,
                                 m, v, vhat, sumsq, blk_part, seg_blk0, step, preps, stream);
}

int fpnmt_amsgrad_step(const fpnmt_adam_desc* d, int nblocks, const int32_t* blk_seg, const long long* blk_start,
                       int block_elems, const long long* off, const int32_t* seg_flags, float* param,
                       const float* grad, float* m, float* v, float* vhat, const float* sumsq,
                       const float* blk_part, const int32_t* seg_blk0, long long* step, fpnmt_stream_t stream) {
  return fpnmt_amsgrad_step_prep(d, nblocks, blk_seg, blk_start, block_elems, off, seg_flags, param, grad, m, v,
                                 vhat, sumsq, blk_part, seg_blk0, step, nullptr, stream);
}

}  // extern "C"
