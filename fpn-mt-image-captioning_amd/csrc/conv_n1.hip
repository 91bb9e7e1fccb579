// Single-filter convolutions (k == 1): the FeatureExtractor's regression head,
// Conv2D(256, 1, 3x3, 'same') over the five pyramid levels, whose output is
// the co-attention's spatial score (reference models/retinanet.py:287,
// coattention.py:24-30). As an implicit GEMM it has N = 1: a 64x64 MFMA tile
// wastes 63/64 of its work and the weight gradient (M = 2304, N = 1, K =
// every pixel) ran at ~1 TFLOP/s. Here each pass is a streaming kernel over
// the input at the HBM roofline:
//   fwd        y[p]     = act(scale * sum_{tap,c} x[p+tap][c] w[tap][c] + b)
//   bwd-data   dx[p][c] = sum_tap dz[p-tap] w[tap][c]  (* act_in'(y_in[p][c]));
//              w read from the flipped bwd-data copy
//   bwd-filter dw[tap][c] += sum_p x[p+tap][c] dz[p]   (block partials, then
//              act_colsum's chunk-ordered sum: deterministic)
// Stride 1, r, s <= 3, channels a power-of-two multiple of 16 B. Several
// levels (grouped launches) are one pixel range; a level is found by prefix.
#include "common.h"

namespace fpnmt {

namespace {

constexpr int N1_MAXL = 6;
constexpr int N1_TAPS = 9;

struct N1Args {
  const void* x[N1_MAXL];   // fwd / wgrad: input; bwd-data: dz (n, ho, wo, 1)
  void* y[N1_MAXL];         // fwd: output (n, ho, wo, 1); bwd-data: dx
  const void* m[N1_MAXL];   // bwd-data: y_in of the act' mask (optional); wgrad: dz
  int H[N1_MAXL], W[N1_MAXL], Ho[N1_MAXL], Wo[N1_MAXL];
  int p0[N1_MAXL + 1];  // first pixel of each level (output grid for fwd / wgrad, input grid for bwd-data)
  int P;                // pixels in total (host: P * C / 16 B < 2^31, 32-bit index math)
  int nl, C, R, S, pt, pl;
};

template <typename T> struct N1V;
template <> struct N1V<bf16> { typedef bf16x8 V; static constexpr int n = 8; };
template <> struct N1V<float> { typedef f32x4 V; static constexpr int n = 4; };

struct N1Level {
  const void* x;
  void* y;
  const void* m;
  int H, W, Ho, Wo;
  int p0;
};

// static-index selection of pixel p's level (no dynamic indexing of the
// kernarg arrays, which would copy the struct to scratch)
__device__ __forceinline__ N1Level n1_level(const N1Args& a, int p) {
  N1Level L{a.x[0], a.y[0], a.m[0], a.H[0], a.W[0], a.Ho[0], a.Wo[0], a.p0[0]};
#pragma unroll
  for (int i = 1; i < N1_MAXL; ++i)
    if (i < a.nl && p >= a.p0[i]) L = N1Level{a.x[i], a.y[i], a.m[i], a.H[i], a.W[i], a.Ho[i], a.Wo[i], a.p0[i]};
  return L;
}

// XCD-aware block order: dispatch sends block b to XCD b % 8; remapped, each
// XCD gets one contiguous 1/8 of the logical blocks, so a block's halo rows
// (the 3x3 taps reach one image row up / down) are mostly in its own XCD's L2
__device__ __forceinline__ int n1_xcd_block(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// ---- VALU-lean arithmetic: the kernels are VALU-bound (a wave64 VALU op
// issues over 4 cycles on a 16-lane SIMD), not HBM-bound, so bf16 products go
// through v_dot2_f32_bf16 (2 MACs, no unpacking) and fp32 ones through packed
// v_pk_fma_f32; out-of-range taps read a zero page instead of masking lanes.
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;

__device__ __forceinline__ float dot16b(const bf16x8& x, const bf16x8& w, float acc) {
  // constant-index sub-vectors (a bit_cast through u32x4 lanes was miscompiled
  // into four dot2s of the same pair)
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 0, 1), __builtin_shufflevector(w, w, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 2, 3), __builtin_shufflevector(w, w, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 4, 5), __builtin_shufflevector(w, w, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 6, 7), __builtin_shufflevector(w, w, 6, 7), acc, false);
  return acc;
}
__device__ __forceinline__ float dot16b(const f32x4& x, const f32x4& w, float acc) {
#pragma unroll
  for (int h = 0; h < 4; ++h) acc = fmaf(x[h], w[h], acc);
  return acc;
}
// 16 B of T as VN/2 float pairs
__device__ __forceinline__ void to_pairs(const bf16x8& v, f32x2_t (&o)[4]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) o[h] = f32x2_t{(float)v[2 * h], (float)v[2 * h + 1]};
}
__device__ __forceinline__ void to_pairs(const f32x4& v, f32x2_t (&o)[2]) {
  o[0] = f32x2_t{v[0], v[1]};
  o[1] = f32x2_t{v[2], v[3]};
}

// fwd: LPP lanes per pixel, NCH 16-B channel chunks per lane (C = LPP*NCH*VN);
// 64 / LPP pixels per wave, lanes of a pixel reduced by xor shuffles; U pixel
// groups per round with all their tap loads issued before the dot products.
template <typename T, int LPP, int NCH>
__global__ __launch_bounds__(256) void n1_fwd_kernel(const N1Args a, const T* __restrict__ w, const float* scale,
                                                     const float* bias, int act, float alpha, const T* zp) {
  typedef typename N1V<T>::V VT;
  constexpr int VN = N1V<T>::n;
  constexpr int PPW = 64 / LPP;
  constexpr int U = NCH == 1 ? 2 : 1;
  const int lane = threadIdx.x & 63, sub = lane % LPP, pw = lane / LPP;
  const int C = a.C, taps = a.R * a.S;
  VT wr[N1_TAPS][NCH];
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
    for (int k = 0; k < NCH; ++k) wr[t][k] = *(const VT*)(t < taps ? w + (long long)t * C + (sub + k * LPP) * VN : zp);
  const float sc = scale ? scale[0] : 1.f, bi = bias ? bias[0] : 0.f;
  const int P = a.P;
  // block-contiguous pixel ranges (rounds of 4 waves x PPW x U pixels), XCD-aware
  constexpr int RP = 4 * PPW * U;
  const int rounds = (P + RP - 1) / RP;
  const int per = (rounds + gridDim.x - 1) / gridDim.x;
  const int vb = n1_xcd_block(blockIdx.x, gridDim.x);
  const int b_end = min(P, (vb + 1) * per * RP);
  for (int base = vb * per * RP + (threadIdx.x >> 6) * PPW * U; base < b_end; base += RP) {
    VT v[U][N1_TAPS][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pu = base + u * PPW + pw;
      const bool live = pu < b_end;
      const N1Level L = n1_level(a, live ? pu : 0);
      const int q = (live ? pu : 0) - L.p0;
      const int hw = L.Ho * L.Wo;
      const int n = q / hw, rem = q - n * hw;
      const int oh = rem / L.Wo, ow = rem - oh * L.Wo;
      const T* xb = (const T*)L.x + (long long)n * L.H * L.W * C + sub * VN;
#pragma unroll
      for (int t = 0; t < N1_TAPS; ++t) {
        const int ih = oh + t / a.S - a.pt, iw = ow + t % a.S - a.pl;
        const bool ok = live && t < taps && ih >= 0 && ih < L.H && iw >= 0 && iw < L.W;
        const T* xr = xb + ((long long)ih * L.W + iw) * C;
#pragma unroll
        for (int k = 0; k < NCH; ++k) v[u][t][k] = *(const VT*)(ok ? xr + k * LPP * VN : zp);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pu = base + u * PPW + pw;
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
        for (int k = 0; k < NCH; ++k) acc = dot16b(v[u][t][k], wr[t][k], acc);
#pragma unroll
      for (int o = LPP / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (pu < b_end && sub == 0) {
        const N1Level L = n1_level(a, pu);
        ((T*)L.y)[pu - L.p0] = from_f32<T>(act_apply(acc * sc + bi, act, alpha));
      }
    }
  }
}

// bwd-data: one thread per (input pixel, 16-B channel chunk): coalesced dx
// stores. The block stages the weights from the flipped bwd-data copy,
// w_flip[c][R-1-r][S-1-s][0], into LDS as [tap][c] (one coalesced read); each
// thread keeps its chunk's taps as float pairs (packed FMAs).
template <typename T>
__global__ __launch_bounds__(256) void n1_bwd_data_kernel(const N1Args a, const T* __restrict__ w, int act_in,
                                                          const T* zp) {
  typedef typename N1V<T>::V VT;
  constexpr int VN = N1V<T>::n;
  constexpr int NP = VN / 2;
  __shared__ float ws[N1_TAPS * 1024];
  const int C = a.C, CV = C / VN, taps = a.R * a.S;
  for (int e = threadIdx.x; e < taps * C; e += 256) {
    const int c = e / taps, tf = e - c * taps;  // e = c * taps + (taps - 1 - t)
    ws[(taps - 1 - tf) * C + c] = to_f32(w[e]);
  }
  __syncthreads();
  const int total = a.P * CV;
  // block-contiguous ranges of 256-item rounds (256 a multiple of CV, a power
  // of two <= 128: a thread's chunk is fixed), XCD-aware block order
  const int rounds = (total + 255) / 256;
  const int per = (rounds + gridDim.x - 1) / gridDim.x;
  const int vb = n1_xcd_block(blockIdx.x, gridDim.x);
  const int i_end = min(total, (vb + 1) * per * 256);
  int i = vb * per * 256 + threadIdx.x;
  const int ch = i % CV;
  f32x2_t wr[N1_TAPS][NP];
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
    for (int h = 0; h < NP; ++h)
      wr[t][h] = t < taps ? f32x2_t{ws[t * C + ch * VN + 2 * h], ws[t * C + ch * VN + 2 * h + 1]} : f32x2_t{0.f, 0.f};
  for (; i < i_end; i += 256) {
    const int p = i / CV;
    const N1Level L = n1_level(a, p);
    const int q = p - L.p0;
    const int hw = L.H * L.W;
    const int n = q / hw, rem = q - n * hw;
    const int ih = rem / L.W, iw = rem - ih * L.W;
    const T* dzb = (const T*)L.x + (long long)n * L.Ho * L.Wo;
    float g[N1_TAPS];
#pragma unroll
    for (int t = 0; t < N1_TAPS; ++t) {
      const int oh = ih - t / a.S + a.pt, ow = iw - t % a.S + a.pl;
      const bool ok = t < taps && oh >= 0 && oh < L.Ho && ow >= 0 && ow < L.Wo;
      g[t] = to_f32(*(ok ? dzb + oh * L.Wo + ow : zp));
    }
    const long long off = (long long)q * C + ch * VN;
    VT yv;
    if (L.m) yv = *(const VT*)((const T*)L.m + off);
    f32x2_t acc[NP];
#pragma unroll
    for (int h = 0; h < NP; ++h) acc[h] = f32x2_t{0.f, 0.f};
#pragma unroll
    for (int t = 0; t < N1_TAPS; ++t) {
      const f32x2_t gg = {g[t], g[t]};
#pragma unroll
      for (int h = 0; h < NP; ++h) acc[h] = __builtin_elementwise_fma(gg, wr[t][h], acc[h]);
    }
    VT o;
#pragma unroll
    for (int h = 0; h < NP; ++h) {
      float v0 = acc[h][0], v1 = acc[h][1];
      if (L.m) {
        v0 *= act_mask_from_y(to_f32(yv[2 * h]), act_in);
        v1 *= act_mask_from_y(to_f32(yv[2 * h + 1]), act_in);
      }
      o[2 * h] = from_f32<T>(v0);
      o[2 * h + 1] = from_f32<T>(v1);
    }
    *(VT*)((T*)L.y + off) = o;
  }
}

// bwd-filter, input-pixel form: dw[t][c] += sum_p x[p][c] dz[p - off_t]. A
// block = PL pixel lanes x CV channel chunks; a thread loads its x chunk ONCE
// per input pixel (as float pairs) and the pixel's taps-many dz values, and
// accumulates taps x VN products (packed FMAs) over the block's pixel range.
// The pixel lanes are summed through LDS in lane order and the block writes
// its [taps][C] partial row (summed in block order by act_colsum).
template <typename T>
__global__ __launch_bounds__(256) void n1_bwd_filter_kernel(const N1Args a, float* __restrict__ part,
                                                            int pix_per_block, const T* zp) {
  typedef typename N1V<T>::V VT;
  constexpr int VN = N1V<T>::n;
  constexpr int NP = VN / 2;
  __shared__ float red[256 * VN];
  const int C = a.C, CV = C / VN, PL = 256 / CV, taps = a.R * a.S;
  const int ch = threadIdx.x % CV, pl = threadIdx.x / CV;
  const int P = a.P;
  const int vb = n1_xcd_block(blockIdx.x, gridDim.x);
  const int pb = vb * pix_per_block;
  const int pe = min(P, pb + pix_per_block);
  f32x2_t acc[N1_TAPS][NP];
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
    for (int h = 0; h < NP; ++h) acc[t][h] = f32x2_t{0.f, 0.f};
  constexpr int U = 2;  // two pixels' loads in flight per round
  for (int p0 = pb + pl; p0 < pe; p0 += U * PL) {
    VT xv[U];
    float g[U][N1_TAPS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * PL;
      const bool live = p < pe;
      const N1Level L = n1_level(a, live ? p : pb);
      const int q = (live ? p : pb) - L.p0;
      const int hw = L.H * L.W;
      const int n = q / hw, rem = q - n * hw;
      const int ih = rem / L.W, iw = rem - ih * L.W;
      xv[u] = *(const VT*)(live ? (const T*)L.x + (long long)q * C + ch * VN : zp);
      const T* dzb = (const T*)L.m + (long long)n * L.Ho * L.Wo;
#pragma unroll
      for (int t = 0; t < N1_TAPS; ++t) {
        const int oh = ih - t / a.S + a.pt, ow = iw - t % a.S + a.pl;
        const bool ok = live && t < taps && oh >= 0 && oh < L.Ho && ow >= 0 && ow < L.Wo;
        g[u][t] = to_f32(*(ok ? dzb + oh * L.Wo + ow : zp));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x2_t xp[NP];
      to_pairs(xv[u], xp);
#pragma unroll
      for (int t = 0; t < N1_TAPS; ++t) {
        const f32x2_t gg = {g[u][t], g[u][t]};
#pragma unroll
        for (int h = 0; h < NP; ++h) acc[t][h] = __builtin_elementwise_fma(xp[h], gg, acc[t][h]);
      }
    }
  }
  float* out = part + (long long)vb * taps * C;
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t) {
    if (t < taps) {  // block-uniform
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        red[threadIdx.x * VN + 2 * h] = acc[t][h][0];
        red[threadIdx.x * VN + 2 * h + 1] = acc[t][h][1];
      }
      __syncthreads();
      if (pl == 0) {
        float sm[VN];
#pragma unroll
        for (int j = 0; j < VN; ++j) sm[j] = red[ch * VN + j];
        for (int r = 1; r < PL; ++r)
#pragma unroll
          for (int j = 0; j < VN; ++j) sm[j] += red[(r * CV + ch) * VN + j];
#pragma unroll
        for (int j = 0; j < VN; ++j) out[(long long)t * C + ch * VN + j] = sm[j];
      }
      __syncthreads();
    }
  }
}

template <typename T>
bool n1_shape_ok(const fpnmt_conv_desc* d) {
  constexpr int VN = N1V<T>::n;
  if (d->k != 1 || d->stride_h != 1 || d->stride_w != 1 || d->r > 3 || d->s > 3 || d->c % VN) return false;
  const int cv = d->c / VN;
  return (cv & (cv - 1)) == 0 && cv >= 8 && cv <= 128;
}

bool n1_aligned(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <typename T>
int n1_fwd_t(const N1Args& a, const void* w, const float* scale, const float* bias, int act, float alpha,
             hipStream_t s) {
  constexpr int VN = N1V<T>::n;
  const int cv = a.C / VN;
  const long long P = a.P;
  const int LPP = cv >= 64 ? 64 : cv;
  const long long waves = (P * LPP + 63) / 64;
  // ~4 waves per SIMD over the chip, each looping over ~4 rounds
  const int grid = (int)std::min<long long>(1024, std::max<long long>(1, (waves + 7) / 8));
  const T* wt = (const T*)w;
  const T* zp = (const T*)zero16_ptr();
  switch (cv) {
    case 8: hipLaunchKernelGGL((n1_fwd_kernel<T, 8, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha, zp); break;
    case 16: hipLaunchKernelGGL((n1_fwd_kernel<T, 16, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha, zp); break;
    case 32: hipLaunchKernelGGL((n1_fwd_kernel<T, 32, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha, zp); break;
    case 64: hipLaunchKernelGGL((n1_fwd_kernel<T, 64, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha, zp); break;
    default: hipLaunchKernelGGL((n1_fwd_kernel<T, 64, 2>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha, zp); break;
  }
  return check_launch("n1_fwd_kernel");
}

template <typename T>
int n1_bwd_data_t(const N1Args& a, const void* w, int act_in, hipStream_t s) {
  constexpr int VN = N1V<T>::n;
  const int cv = a.C / VN;
  const long long total = (long long)a.P * cv;
  // grid * 256 a multiple of cv (a power of two <= 128): every thread keeps one
  // chunk; 2 pixels per thread (the LDS weight staging per block vs the
  // serial rounds' memory latency)
  const int grid = (int)std::min<long long>(8192, std::max<long long>(1, (total + 511) / 512));
  hipLaunchKernelGGL((n1_bwd_data_kernel<T>), dim3(grid), dim3(256), 0, s, a, (const T*)w, act_in,
                     (const T*)zero16_ptr());
  return check_launch("n1_bwd_data_kernel");
}

template <typename T>
int n1_bwd_filter_t(const N1Args& a, float* dw, hipStream_t s) {
  const long long P = a.P;
  if (P <= 0) return 0;
  const int cols = a.R * a.S * a.C;
  long long nb = std::min<long long>(1024, std::max<long long>(1, P / 16));
  const long long ppb = (P + nb - 1) / nb;
  nb = (P + ppb - 1) / ppb;
  float* part = partial_f32(nb * cols);
  if (!part) return fail(FPNMT_E_ARG, "conv2d_bwd_filter (k = 1): needs the process workspace (fpnmt_set_workspace)");
  hipLaunchKernelGGL((n1_bwd_filter_kernel<T>), dim3((unsigned)nb), dim3(256), 0, s, a, part, (int)ppb,
                     (const T*)zero16_ptr());
  const int st = check_launch("n1_bwd_filter_kernel");
  if (st) return st;
  colsum_launch((int)nb, cols, part, dw, s);
  return check_launch("n1_bwd_filter colsum");
}

// level table over `lv` (skipping empty levels); grid = the fwd / wgrad output
// grid (out_grid) or the bwd-data input grid
int n1_args(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv, int pass, int act_in, N1Args& a) {
  const bool out_grid = pass == 0;  // fwd walks output pixels; bwd-data / bwd-filter input pixels
  a = N1Args{};
  a.C = d->c; a.R = d->r; a.S = d->s; a.pt = d->pad_t; a.pl = d->pad_l;
  long long p = 0;
  for (int i = 0; i < n_levels; ++i) {
    const fpnmt_conv_level& L = lv[i];
    const int ho = (L.h + d->pad_t + d->pad_b - d->r) + 1, wo = (L.w + d->pad_l + d->pad_r - d->s) + 1;
    const long long pix = out_grid ? (long long)L.n * ho * wo : (long long)L.n * L.h * L.w;
    if (L.n <= 0 || ho <= 0 || wo <= 0 || L.h <= 0 || L.w <= 0 || pix <= 0) continue;
    if (a.nl == N1_MAXL) return -1;
    if (pass == 0 && L.residual) return -1;  // fwd residual: the GEMM epilogue has it
    a.x[a.nl] = L.x; a.y[a.nl] = L.y;
    a.m[a.nl] = pass == 2 ? L.dz : (pass == 1 && act_in != FPNMT_ACT_NONE ? L.residual : nullptr);
    a.H[a.nl] = L.h; a.W[a.nl] = L.w; a.Ho[a.nl] = ho; a.Wo[a.nl] = wo;
    a.p0[a.nl] = (int)p;
    p += pix;
    ++a.nl;
    if (p * d->c >= (1LL << 31)) return -1;  // 32-bit pixel x channel offsets in the kernels
  }
  a.p0[a.nl] = (int)p;
  for (int i = a.nl + 1; i <= N1_MAXL; ++i) a.p0[i] = (int)p;
  a.P = (int)p;
  return 0;
}

bool n1_ptrs_aligned(const N1Args& a, bool x, bool y, bool m) {
  for (int i = 0; i < a.nl; ++i)
    if ((x && !n1_aligned(a.x[i])) || (y && !n1_aligned(a.y[i])) || (m && a.m[i] && !n1_aligned(a.m[i])))
      return false;
  return true;
}

}  // namespace

// Dispatch hooks called by the conv entry points (api.hip): 1 = launched,
// 0 = not handled (the implicit GEMM runs), < 0 = error.
int conv_n1(int pass, const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv, const void* w,
            const float* scale, const float* bias, int act_in, float* dw, hipStream_t s) {
  const bool bf = d->dtype == FPNMT_BF16;
  if (bf ? !n1_shape_ok<bf16>(d) : !n1_shape_ok<float>(d)) return 0;
  if ((pass != 2 && !n1_aligned(w)) || !zero16_ptr()) return 0;  // the zero page: the process workspace
  N1Args a;
  if (n1_args(d, n_levels, lv, pass, act_in, a)) return 0;
  if (a.nl == 0) return 0;  // nothing to compute: the generic path handles empty outputs
  int st = 0;
  if (pass == 0) {  // fwd: lv.x input, lv.y output
    if (!n1_ptrs_aligned(a, true, false, false)) return 0;
    st = bf ? n1_fwd_t<bf16>(a, w, scale, bias, d->act, d->act_alpha, s)
            : n1_fwd_t<float>(a, w, scale, bias, d->act, d->act_alpha, s);
  } else if (pass == 1) {  // bwd-data: lv.x dz, lv.y dx, lv.dz = y_in (mask) or null
    if (!n1_ptrs_aligned(a, false, true, true)) return 0;
    st = bf ? n1_bwd_data_t<bf16>(a, w, act_in, s) : n1_bwd_data_t<float>(a, w, act_in, s);
  } else {  // bwd-filter: lv.x input, lv.dz output gradient
    if (scale || !n1_ptrs_aligned(a, true, false, false)) return 0;
    st = bf ? n1_bwd_filter_t<bf16>(a, dw, s) : n1_bwd_filter_t<float>(a, dw, s);
  }
  return st ? st : 1;
}

}  // namespace fpnmt
