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
  long long p0[N1_MAXL + 1];  // first pixel of each level (output grid for fwd / wgrad, input grid for bwd-data)
  long long P;                // pixels in total
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
  long long p0;
};

// static-index selection of pixel p's level (no dynamic indexing of the
// kernarg arrays, which would copy the struct to scratch)
__device__ __forceinline__ N1Level n1_level(const N1Args& a, long long p) {
  N1Level L{a.x[0], a.y[0], a.m[0], a.H[0], a.W[0], a.Ho[0], a.Wo[0], a.p0[0]};
#pragma unroll
  for (int i = 1; i < N1_MAXL; ++i)
    if (i < a.nl && p >= a.p0[i]) L = N1Level{a.x[i], a.y[i], a.m[i], a.H[i], a.W[i], a.Ho[i], a.Wo[i], a.p0[i]};
  return L;
}

// LPP lanes per pixel, NCH 16-B channel chunks per lane (C = LPP*NCH*VN);
// 64 / LPP pixels per wave, lanes of a pixel reduced by xor shuffles
template <typename T, int LPP, int NCH>
__global__ __launch_bounds__(256) void n1_fwd_kernel(const N1Args a, const T* __restrict__ w, const float* scale,
                                                     const float* bias, int act, float alpha) {
  typedef typename N1V<T>::V VT;
  constexpr int VN = N1V<T>::n;
  constexpr int PPW = 64 / LPP;
  const int lane = threadIdx.x & 63, sub = lane % LPP, pw = lane / LPP;
  const int C = a.C, taps = a.R * a.S;
  float wr[N1_TAPS][NCH][VN];
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      VT v = t < taps ? *(const VT*)(w + (long long)t * C + (sub + k * LPP) * VN) : VT{};
#pragma unroll
      for (int j = 0; j < VN; ++j) wr[t][k][j] = to_f32(v[j]);
    }
  const float sc = scale ? scale[0] : 1.f, bi = bias ? bias[0] : 0.f;
  const long long P = a.P;
  const long long stride = (long long)gridDim.x * 4 * PPW;
  for (long long base = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * PPW; base < P; base += stride) {
    const long long p = base + pw;
    const bool valid = p < P;
    float acc = 0.f;
    if (valid) {
      const N1Level L = n1_level(a, p);
      const long long q = p - L.p0;
      const int hw = L.Ho * L.Wo;
      const int n = (int)(q / hw), rem = (int)(q - (long long)n * hw);
      const int oh = rem / L.Wo, ow = rem - oh * L.Wo;
      const T* xb = (const T*)L.x + (long long)n * L.H * L.W * C;
#pragma unroll
      for (int t = 0; t < N1_TAPS; ++t) {
        if (t >= taps) break;
        const int ih = oh + t / a.S - a.pt, iw = ow + t % a.S - a.pl;
        if (ih < 0 || ih >= L.H || iw < 0 || iw >= L.W) continue;
        const T* xr = xb + ((long long)ih * L.W + iw) * C;
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          const VT v = *(const VT*)(xr + (sub + k * LPP) * VN);
#pragma unroll
          for (int j = 0; j < VN; ++j) acc += to_f32(v[j]) * wr[t][k][j];
        }
      }
    }
#pragma unroll
    for (int o = LPP / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (valid && sub == 0) {
      const N1Level L = n1_level(a, p);
      ((T*)L.y)[p - L.p0] = from_f32<T>(act_apply(acc * sc + bi, act, alpha));
    }
  }
}

// one thread per (input pixel, 16-B channel chunk): coalesced dx stores
template <typename T>
__global__ __launch_bounds__(256) void n1_bwd_data_kernel(const N1Args a, const T* __restrict__ w, int act_in) {
  typedef typename N1V<T>::V VT;
  constexpr int VN = N1V<T>::n;
  const int C = a.C, CV = C / VN, taps = a.R * a.S;
  const long long P = a.P;
  const long long total = P * CV;
  const long long stride = (long long)gridDim.x * 256;  // a multiple of CV (host): the chunk is fixed
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int ch = (int)(i % CV);
  // w is the bwd-data operand, the flipped IHWO copy: w_flip[c][R-1-r][S-1-s][0]
  float wr[N1_TAPS][VN];
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
    for (int j = 0; j < VN; ++j)
      wr[t][j] = t < taps ? to_f32(w[(long long)(ch * VN + j) * taps + (taps - 1 - t)]) : 0.f;
  for (; i < total; i += stride) {
    const long long p = i / CV;
    const N1Level L = n1_level(a, p);
    const long long q = p - L.p0;
    const int hw = L.H * L.W;
    const int n = (int)(q / hw), rem = (int)(q - (long long)n * hw);
    const int ih = rem / L.W, iw = rem - ih * L.W;
    const T* dzb = (const T*)L.x + (long long)n * L.Ho * L.Wo;
    float acc[VN];
#pragma unroll
    for (int j = 0; j < VN; ++j) acc[j] = 0.f;
#pragma unroll
    for (int t = 0; t < N1_TAPS; ++t) {
      if (t >= taps) break;
      const int oh = ih - t / a.S + a.pt, ow = iw - t % a.S + a.pl;
      if (oh < 0 || oh >= L.Ho || ow < 0 || ow >= L.Wo) continue;
      const float g = to_f32(dzb[(long long)oh * L.Wo + ow]);
#pragma unroll
      for (int j = 0; j < VN; ++j) acc[j] += g * wr[t][j];
    }
    const long long off = q * C + (long long)ch * VN;
    if (L.m) {
      const VT yv = *(const VT*)((const T*)L.m + off);
#pragma unroll
      for (int j = 0; j < VN; ++j) acc[j] *= act_mask_from_y(to_f32(yv[j]), act_in);
    }
    VT o;
#pragma unroll
    for (int j = 0; j < VN; ++j) o[j] = from_f32<T>(acc[j]);
    *(VT*)((T*)L.y + off) = o;
  }
}

// Block = PL pixel lanes x CV channel chunks; every thread accumulates its
// chunk's taps x VN products over the block's pixel range, the pixel lanes
// are summed through LDS in lane order, and the block writes its partial
// [taps][C] row to part[blockIdx.x] (summed in block order by act_colsum).
template <typename T>
__global__ __launch_bounds__(256) void n1_bwd_filter_kernel(const N1Args a, float* __restrict__ part,
                                                            long long pix_per_block) {
  typedef typename N1V<T>::V VT;
  constexpr int VN = N1V<T>::n;
  __shared__ float red[256 * VN];
  const int C = a.C, CV = C / VN, PL = 256 / CV, taps = a.R * a.S;
  const int ch = threadIdx.x % CV, pl = threadIdx.x / CV;
  const long long P = a.P;
  const long long pb = (long long)blockIdx.x * pix_per_block;
  const long long pe = min(P, pb + pix_per_block);
  float acc[N1_TAPS][VN];
#pragma unroll
  for (int t = 0; t < N1_TAPS; ++t)
#pragma unroll
    for (int j = 0; j < VN; ++j) acc[t][j] = 0.f;
  for (long long p = pb + pl; p < pe; p += PL) {
    const N1Level L = n1_level(a, p);
    const long long q = p - L.p0;
    const int hw = L.Ho * L.Wo;
    const int n = (int)(q / hw), rem = (int)(q - (long long)n * hw);
    const int oh = rem / L.Wo, ow = rem - oh * L.Wo;
    const float g = to_f32(((const T*)L.m)[q]);
    const T* xb = (const T*)L.x + (long long)n * L.H * L.W * C + ch * VN;
#pragma unroll
    for (int t = 0; t < N1_TAPS; ++t) {
      if (t >= taps) break;
      const int ih = oh + t / a.S - a.pt, iw = ow + t % a.S - a.pl;
      if (ih < 0 || ih >= L.H || iw < 0 || iw >= L.W) continue;
      const VT v = *(const VT*)(xb + ((long long)ih * L.W + iw) * C);
#pragma unroll
      for (int j = 0; j < VN; ++j) acc[t][j] += to_f32(v[j]) * g;
    }
  }
  float* out = part + (long long)blockIdx.x * taps * C;
  for (int t = 0; t < taps; ++t) {
#pragma unroll
    for (int j = 0; j < VN; ++j) red[threadIdx.x * VN + j] = acc[t][j];
    __syncthreads();
    if (pl == 0) {
      float s[VN];
#pragma unroll
      for (int j = 0; j < VN; ++j) s[j] = red[ch * VN + j];
      for (int r = 1; r < PL; ++r)
#pragma unroll
        for (int j = 0; j < VN; ++j) s[j] += red[(r * CV + ch) * VN + j];
#pragma unroll
      for (int j = 0; j < VN; ++j) out[(long long)t * C + ch * VN + j] = s[j];
    }
    __syncthreads();
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
  const long long P = a.p0[a.nl];
  const int LPP = cv >= 64 ? 64 : cv;
  const long long waves = (P * LPP + 63) / 64;
  const int grid = (int)std::min<long long>(2048, std::max<long long>(1, (waves + 3) / 4));
  const T* wt = (const T*)w;
  switch (cv) {
    case 8: hipLaunchKernelGGL((n1_fwd_kernel<T, 8, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha); break;
    case 16: hipLaunchKernelGGL((n1_fwd_kernel<T, 16, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha); break;
    case 32: hipLaunchKernelGGL((n1_fwd_kernel<T, 32, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha); break;
    case 64: hipLaunchKernelGGL((n1_fwd_kernel<T, 64, 1>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha); break;
    default: hipLaunchKernelGGL((n1_fwd_kernel<T, 64, 2>), dim3(grid), dim3(256), 0, s, a, wt, scale, bias, act, alpha); break;
  }
  return check_launch("n1_fwd_kernel");
}

template <typename T>
int n1_bwd_data_t(const N1Args& a, const void* w, int act_in, hipStream_t s) {
  constexpr int VN = N1V<T>::n;
  const int cv = a.C / VN;
  const long long total = a.p0[a.nl] * cv;
  // grid * 256 a multiple of cv (a power of two <= 128): every thread keeps one chunk
  const int grid = (int)std::min<long long>(4096, std::max<long long>(1, (total + 255) / 256));
  hipLaunchKernelGGL((n1_bwd_data_kernel<T>), dim3(grid), dim3(256), 0, s, a, (const T*)w, act_in);
  return check_launch("n1_bwd_data_kernel");
}

template <typename T>
int n1_bwd_filter_t(const N1Args& a, float* dw, hipStream_t s) {
  const long long P = a.p0[a.nl];
  if (P <= 0) return 0;
  const int cols = a.R * a.S * a.C;
  long long nb = std::min<long long>(512, std::max<long long>(1, P / 32));
  const long long ppb = (P + nb - 1) / nb;
  nb = (P + ppb - 1) / ppb;
  float* part = scratch_f32(nb * cols);
  if (!part) return fail(FPNMT_E_ARG, "conv2d_bwd_filter (k = 1): needs the process workspace (fpnmt_set_workspace)");
  hipLaunchKernelGGL((n1_bwd_filter_kernel<T>), dim3((unsigned)nb), dim3(256), 0, s, a, part, ppb);
  const int st = check_launch("n1_bwd_filter_kernel");
  if (st) return st;
  colsum_launch((int)nb, cols, part, dw, s);
  return check_launch("n1_bwd_filter colsum");
}

// level table over `lv` (skipping empty levels); grid = the fwd / wgrad output
// grid (out_grid) or the bwd-data input grid
int n1_args(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv, int pass, int act_in, N1Args& a) {
  const bool out_grid = pass != 1;
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
    a.p0[a.nl] = p;
    p += pix;
    ++a.nl;
  }
  a.p0[a.nl] = p;
  for (int i = a.nl + 1; i <= N1_MAXL; ++i) a.p0[i] = p;
  a.P = p;
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
  if (!n1_aligned(w)) return 0;
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
