// Kernels of the MobileNetV2 backbone (the reference FeatureExtractor's
// default, models/retinanet.py:274 -> models/mobilenet.py:43-72, Keras
// MobileNetV2): BatchNormalization in training mode (batch statistics,
// moving averages) fused with ReLU6 / the residual add, and the 3x3
// depthwise convolution. All NHWC, HBM-bound: 16-B vectors per lane, and
// every reduction is per-block partials summed in a fixed order (no
// atomics: bitwise-repeatable gradients and statistics).
#include "common.h"

namespace fpnmt {

template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* v) {
    const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)t[j];
  }
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    bf16x8 t;
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = (bf16)v[j];
    *(bf16x8*)p = t;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[j + 4]; }
    *(f32x4*)p = a;
    *(f32x4*)(p + 4) = b;
  }
};

__device__ __forceinline__ float act6(float v, int act) {
  if (act == FPNMT_ACT_RELU6) return fminf(fmaxf(v, 0.f), 6.f);
  return act_apply(v, act, 0.f);
}
// derivative from the activation output (relu6: 0 < y < 6)
__device__ __forceinline__ float act6_grad(float y, int act) {
  if (act == FPNMT_ACT_RELU6) return (y > 0.f && y < 6.f) ? 1.f : 0.f;
  return act_grad_from_y(y, act, 0.f);
}

// ---------------------------------------------------------------------------
// Column-partial reductions over (rows, c) NHWC activations. Block = 256
// threads = RL row lanes x GT groups of 8 channels; grid (column tiles, row
// chunks); each block writes part[chunk][k][c] for its K quantities.
struct ColGrid {
  int gx, gy, rpc, GT, RL;
};
static ColGrid col_grid(long long rows, int c) {
  ColGrid G;
  const int groups = c / 8;
  G.GT = groups < 256 ? groups : 256;
  G.RL = 256 / G.GT;
  G.gx = cdiv(groups, G.GT);
  long long chunks = 512 / G.gx;
  const long long max_chunks = (rows + 4LL * G.RL - 1) / (4LL * G.RL);
  chunks = std::max(1LL, std::min(chunks, max_chunks));
  G.rpc = (int)((rows + chunks - 1) / chunks);
  G.gy = (int)((rows + G.rpc - 1) / G.rpc);
  return G;
}

// BN statistics pass 1: shifted sums (shift = row 0's value of the channel)
// S1 = sum(x - K), S2 = sum((x - K)^2), accumulated in fp64: HBM-bound, so
// the fp64 adds are free, and the variance and the backward's channel sums
// feed a cancellation (training-mode BN backward) that fp32 sums amplify
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_part_kernel(long long rows, int c, int rpc, const T* __restrict__ x,
                                                            double* __restrict__ part) {
  __shared__ double red[2][256 * 8];
  const int groups = c / 8;
  const int GT = groups < 256 ? groups : 256, RL = 256 / GT;
  const int tg = threadIdx.x % GT, tr = threadIdx.x / GT;
  const int g = blockIdx.x * GT + tg;
  const bool active = tr < RL && g < groups;
  const long long r0 = (long long)blockIdx.y * rpc, r1 = min(rows, r0 + rpc);
  double s1[8], s2[8];
  float k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.0;
  if (active) {
    Vec8<T>::load(x + (long long)g * 8, k);
    for (long long r = r0 + tr; r < r1; r += RL) {
      float v[8];
      Vec8<T>::load(x + r * c + (long long)g * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double d = (double)v[j] - (double)k[j];
        s1[j] += d;
        s2[j] += d * d;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * 8 + j] = s1[j];
    red[1][threadIdx.x * 8 + j] = s2[j];
  }
  __syncthreads();
  if (tr == 0 && g < groups) {
    for (int q = 1; q < RL; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += red[0][(q * GT + tg) * 8 + j];
        s2[j] += red[1][(q * GT + tg) * 8 + j];
      }
    double* dst = part + (long long)blockIdx.y * 2 * c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dst[g * 8 + j] = s1[j];
      dst[c + g * 8 + j] = s2[j];
    }
  }
}

// pass 2 (block per 64 channels x 4 chunk lanes): chunk partials in a fixed
// order -> batch mean / biased variance; moving averages (Keras:
// moving = moving * momentum + value * (1 - momentum), the variance with
// Bessel's correction as fused batch norm reports it)
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_final_kernel(long long rows, int c, int chunks,
                                                             const T* __restrict__ x,
                                                             const double* __restrict__ part,
                                                             float* __restrict__ mean, float* __restrict__ var,
                                                             float* __restrict__ mmean, float* __restrict__ mvar,
                                                             float momentum) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, kl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  double a = 0.0, b = 0.0;
  if (col < c)
    for (int k = kl; k < chunks; k += 4) {
      a += part[(long long)k * 2 * c + col];
      b += part[(long long)k * 2 * c + c + col];
    }
  red[0][kl][cl] = a;
  red[1][kl][cl] = b;
  __syncthreads();
  if (kl == 0 && col < c) {
    const double s1 = ((red[0][0][cl] + red[0][1][cl]) + red[0][2][cl]) + red[0][3][cl];
    const double s2 = ((red[1][0][cl] + red[1][1][cl]) + red[1][2][cl]) + red[1][3][cl];
    const double n = (double)rows;
    const double d = s1 / n;
    const double v = fmax(s2 / n - d * d, 0.0);
    const float m = (float)((double)to_f32(x[col]) + d);
    mean[col] = m;
    var[col] = (float)v;
    if (mmean) {
      const float unb = (float)(rows > 1 ? v * (n / (n - 1.0)) : v);
      mmean[col] = mmean[col] * momentum + m * (1.f - momentum);
      mvar[col] = mvar[col] * momentum + unb * (1.f - momentum);
    }
  }
}

// y = act((x - mean) * rsqrt(var + eps) * gamma + beta) [+ residual]
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(long long n8, int c, const T* __restrict__ x,
                                                       const float* __restrict__ mean, const float* __restrict__ var,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps, int act,
                                                       const T* __restrict__ res, T* __restrict__ y) {
  const int g8 = c / 8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % g8) * 8;
    float v[8], r[8];
    Vec8<T>::load(x + i * 8, v);
    if (res) Vec8<T>::load(res + i * 8, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = (v[j] - mean[ch + j]) * rsqrtf(var[ch + j] + eps) * gamma[ch + j] + beta[ch + j];
      o = act6(o, act);
      v[j] = res ? o + r[j] : o;
    }
    Vec8<T>::store(y + i * 8, v);
  }
}

// BN backward pass 1: per-chunk sums of g = dy * act'(y) and g * xhat
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_part_kernel(long long rows, int c, int rpc, const T* __restrict__ x,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ var, float eps, int act,
                                                          const T* __restrict__ y, const T* __restrict__ dy,
                                                          double* __restrict__ part) {
  __shared__ double red[2][256 * 8];
  const int groups = c / 8;
  const int GT = groups < 256 ? groups : 256, RL = 256 / GT;
  const int tg = threadIdx.x % GT, tr = threadIdx.x / GT;
  const int g = blockIdx.x * GT + tg;
  const bool active = tr < RL && g < groups;
  const long long r0 = (long long)blockIdx.y * rpc, r1 = min(rows, r0 + rpc);
  double sb[8], sg[8];
  float mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sb[j] = sg[j] = 0.0;
  if (active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = mean[g * 8 + j];
      rs[j] = rsqrtf(var[g * 8 + j] + eps);
    }
    for (long long r = r0 + tr; r < r1; r += RL) {
      float xv[8], yv[8], dv[8];
      const long long o = r * c + (long long)g * 8;
      Vec8<T>::load(x + o, xv);
      Vec8<T>::load(dy + o, dv);
      if (act != FPNMT_ACT_NONE) Vec8<T>::load(y + o, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gr = act != FPNMT_ACT_NONE ? dv[j] * act6_grad(yv[j], act) : dv[j];
        sb[j] += (double)gr;
        sg[j] += (double)gr * (double)((xv[j] - mu[j]) * rs[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * 8 + j] = sb[j];
    red[1][threadIdx.x * 8 + j] = sg[j];
  }
  __syncthreads();
  if (tr == 0 && g < groups) {
    for (int q = 1; q < RL; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sb[j] += red[0][(q * GT + tg) * 8 + j];
        sg[j] += red[1][(q * GT + tg) * 8 + j];
      }
    double* dst = part + (long long)blockIdx.y * 2 * c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dst[g * 8 + j] = sb[j];
      dst[c + g * 8 + j] = sg[j];
    }
  }
}

// pass 2: sums[c] = dbeta, sums[c + col] = dgamma (fixed order); += into the grads
__global__ __launch_bounds__(256) void bn_bwd_final_kernel(int c, int chunks, const double* __restrict__ part,
                                                           float* __restrict__ sums, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, kl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  double a = 0.0, b = 0.0;
  if (col < c)
    for (int k = kl; k < chunks; k += 4) {
      a += part[(long long)k * 2 * c + col];
      b += part[(long long)k * 2 * c + c + col];
    }
  red[0][kl][cl] = a;
  red[1][kl][cl] = b;
  __syncthreads();
  if (kl == 0 && col < c) {
    const float sb = (float)(((red[0][0][cl] + red[0][1][cl]) + red[0][2][cl]) + red[0][3][cl]);
    const float sg = (float)(((red[1][0][cl] + red[1][1][cl]) + red[1][2][cl]) + red[1][3][cl]);
    sums[col] = sb;
    sums[c + col] = sg;
    if (dbeta) dbeta[col] += sb;
    if (dgamma) dgamma[col] += sg;
  }
}

// pass 3: dx = gamma * rstd * (g - sum(g)/n - xhat * sum(g xhat)/n)
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(long long rows, int c, const T* __restrict__ x,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ var,
                                                        const float* __restrict__ gamma, float eps, int act,
                                                        const T* __restrict__ y, const T* __restrict__ dy,
                                                        const float* __restrict__ sums, float inv_n,
                                                        const float* __restrict__ inv_n_dev, T* __restrict__ dx) {
  const int g8 = c / 8;
  if (inv_n_dev) inv_n = *inv_n_dev;  // sync BN: 1 / the all-reduced row count
  const long long n8 = rows * g8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % g8) * 8;
    float xv[8], yv[8], dv[8], o[8];
    Vec8<T>::load(x + i * 8, xv);
    Vec8<T>::load(dy + i * 8, dv);
    if (act != FPNMT_ACT_NONE) Vec8<T>::load(y + i * 8, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float rs = rsqrtf(var[ch + j] + eps);
      const float gr = act != FPNMT_ACT_NONE ? dv[j] * act6_grad(yv[j], act) : dv[j];
      const float xh = (xv[j] - mean[ch + j]) * rs;
      o[j] = gamma[ch + j] * rs * (gr - sums[ch + j] * inv_n - xh * sums[c + ch + j] * inv_n);
    }
    Vec8<T>::store(dx + i * 8, o);
  }
}

// ---------------------------------------------------------------------------
// Cross-replica ("sync") BatchNorm for data parallelism: each rank reduces its
// own rows to fp64 sums, the caller all-reduces them (SUM over the ranks),
// and the statistics / the backward's channel sums are the global batch's
// (Keras BatchNormalization over the whole global batch, what the reference
// computes on one device: models/mobilenet.py:61, SURVEY 8(e) "Batch norm").
//
// forward sums, plain (shift-0) form so that ranks with different shifts
// add: sums[col] = sum x, sums[c + col] = sum x^2, sums[2c] = rows
// (converted from the shifted partials in fp64: S1 + n K, S2 + 2 K S1 + n K^2)
template <typename T>
__global__ __launch_bounds__(256) void bn_sums_final_kernel(long long rows, int c, int chunks, const T* __restrict__ x,
                                                            const double* __restrict__ part,
                                                            double* __restrict__ sums) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, kl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  double a = 0.0, b = 0.0;
  if (col < c)
    for (int k = kl; k < chunks; k += 4) {
      a += part[(long long)k * 2 * c + col];
      b += part[(long long)k * 2 * c + c + col];
    }
  red[0][kl][cl] = a;
  red[1][kl][cl] = b;
  __syncthreads();
  if (kl == 0 && col < c) {
    const double s1 = ((red[0][0][cl] + red[0][1][cl]) + red[0][2][cl]) + red[0][3][cl];
    const double s2 = ((red[1][0][cl] + red[1][1][cl]) + red[1][2][cl]) + red[1][3][cl];
    const double n = (double)rows, K = (double)to_f32(x[col]);
    sums[col] = s1 + n * K;
    sums[c + col] = s2 + 2.0 * K * s1 + n * K * K;
    if (col == 0) sums[2 * c] = n;
  }
}

// statistics of the (all-reduced) sums: batch mean / biased variance and the
// Keras moving averages (unbiased variance), as bn_stats_final_kernel
__global__ __launch_bounds__(256) void bn_stats_from_sums_kernel(int c, const double* __restrict__ sums,
                                                                 float* __restrict__ mean, float* __restrict__ var,
                                                                 float* __restrict__ mmean, float* __restrict__ mvar,
                                                                 float momentum) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= c) return;
  const double n = sums[2 * c];
  const double m = sums[col] / n;
  const double v = fmax(sums[c + col] / n - m * m, 0.0);
  mean[col] = (float)m;
  var[col] = (float)v;
  if (mmean) {
    const float unb = (float)(n > 1.0 ? v * (n / (n - 1.0)) : v);
    mmean[col] = mmean[col] * momentum + (float)m * (1.f - momentum);
    mvar[col] = mvar[col] * momentum + unb * (1.f - momentum);
  }
}

// backward sums of one rank: sums[col] = sum g, sums[c + col] = sum g * xhat
// (fp64, to be all-reduced), sums[2c] = rows; the rank's own parts are also
// added to dgamma / dbeta (the gradient exchange sums those over the ranks)
__global__ __launch_bounds__(256) void bn_bwd_sums_final_kernel(long long rows, int c, int chunks,
                                                                const double* __restrict__ part,
                                                                double* __restrict__ sums,
                                                                float* __restrict__ dgamma,
                                                                float* __restrict__ dbeta) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, kl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  double a = 0.0, b = 0.0;
  if (col < c)
    for (int k = kl; k < chunks; k += 4) {
      a += part[(long long)k * 2 * c + col];
      b += part[(long long)k * 2 * c + c + col];
    }
  red[0][kl][cl] = a;
  red[1][kl][cl] = b;
  __syncthreads();
  if (kl == 0 && col < c) {
    const double sb = ((red[0][0][cl] + red[0][1][cl]) + red[0][2][cl]) + red[0][3][cl];
    const double sg = ((red[1][0][cl] + red[1][1][cl]) + red[1][2][cl]) + red[1][3][cl];
    sums[col] = sb;
    sums[c + col] = sg;
    if (col == 0) sums[2 * c] = (double)rows;
    if (dbeta) dbeta[col] += (float)sb;
    if (dgamma) dgamma[col] += (float)sg;
  }
}

// global fp64 backward sums -> the float sums bn_bwd_dx_kernel reads, and
// out[2c] = 1 / the global row count (sums[2c], all-reduced with the sums)
__global__ __launch_bounds__(256) void bn_sums_to_f32_kernel(int c, const double* __restrict__ sums,
                                                             float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < 2 * c) out[i] = (float)sums[i];
  else if (i == 2 * c) out[i] = (float)(1.0 / fmax(sums[i], 1.0));
}

// ---------------------------------------------------------------------------
// Depthwise 3x3 (any kh x kw) conv, NHWC, weights (kh, kw, C) fp32 master
// layout (Keras (kh, kw, C, 1)). Thread per output pixel x 8 channels.
template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_kernel(int n, int h, int w, int c, int kh, int kw, int st, int pt,
                                                     int pl, int ho, int wo, const T* __restrict__ x,
                                                     const float* __restrict__ wt, T* __restrict__ y) {
  const int g8 = c / 8;
  const long long total = (long long)n * ho * wo * g8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % g8) * 8;
    long long t = i / g8;
    const int ow = (int)(t % wo);
    t /= wo;
    const int oh = (int)(t % ho);
    const int nn = (int)(t / ho);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int r = 0; r < kh; ++r) {
      const int ih = oh * st - pt + r;
      if (ih < 0 || ih >= h) continue;
      for (int s = 0; s < kw; ++s) {
        const int iw = ow * st - pl + s;
        if (iw < 0 || iw >= w) continue;
        float v[8];
        Vec8<T>::load(x + (((long long)nn * h + ih) * w + iw) * c + ch, v);
        const float* wp = wt + (r * kw + s) * c + ch;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j] * wp[j];
      }
    }
    Vec8<T>::store(y + i * 8, acc);
  }
}

// dx: gather form (thread per input pixel x 8 channels), no atomics
template <typename T>
__global__ __launch_bounds__(256) void dw_bwd_data_kernel(int n, int h, int w, int c, int kh, int kw, int st, int pt,
                                                          int pl, int ho, int wo, const T* __restrict__ dy,
                                                          const float* __restrict__ wt, T* __restrict__ dx) {
  const int g8 = c / 8;
  const long long total = (long long)n * h * w * g8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int ch = (int)(i % g8) * 8;
    long long t = i / g8;
    const int iw = (int)(t % w);
    t /= w;
    const int ih = (int)(t % h);
    const int nn = (int)(t / h);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int r = 0; r < kh; ++r) {
      const int a = ih + pt - r;  // = oh * st
      if (a < 0 || a % st) continue;
      const int oh = a / st;
      if (oh >= ho) continue;
      for (int s = 0; s < kw; ++s) {
        const int b = iw + pl - s;
        if (b < 0 || b % st) continue;
        const int ow = b / st;
        if (ow >= wo) continue;
        float v[8];
        Vec8<T>::load(dy + (((long long)nn * ho + oh) * wo + ow) * c + ch, v);
        const float* wp = wt + (r * kw + s) * c + ch;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j] * wp[j];
      }
    }
    Vec8<T>::store(dx + i * 8, acc);
  }
}

// dW[r][s][c] = sum over output pixels of x(tap) * dy: pass 1 per-chunk
// partials part[chunk][kh*kw][c] (thread = 8 channels of one chunk lane)
template <typename T>
__global__ __launch_bounds__(256) void dw_bwd_filter_part_kernel(int n, int h, int w, int c, int kh, int kw, int st,
                                                                 int pt, int pl, int ho, int wo, int ppc,
                                                                 const T* __restrict__ x, const T* __restrict__ dy,
                                                                 float* __restrict__ part) {
  constexpr int MAXT = 9;
  __shared__ float red[256][8];
  const int groups = c / 8;
  const int GT = groups < 256 ? groups : 256, RL = 256 / GT;
  const int tg = threadIdx.x % GT, tr = threadIdx.x / GT;
  const int g = blockIdx.x * GT + tg;
  const bool active = tr < RL && g < groups;
  const long long npix = (long long)n * ho * wo;
  const long long p0 = (long long)blockIdx.y * ppc, p1 = min(npix, p0 + ppc);
  float acc[MAXT][8];
#pragma unroll
  for (int q = 0; q < MAXT; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
  if (active) {
    for (long long pp = p0 + tr; pp < p1; pp += RL) {
      const int ow = (int)(pp % wo);
      const long long t = pp / wo;
      const int oh = (int)(t % ho);
      const int nn = (int)(t / ho);
      float d[8];
      Vec8<T>::load(dy + pp * c + (long long)g * 8, d);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int ih = oh * st - pt + r;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int iw = ow * st - pl + s;
          if (r >= kh || s >= kw || ih < 0 || ih >= h || iw < 0 || iw >= w) continue;
          float v[8];
          Vec8<T>::load(x + (((long long)nn * h + ih) * w + iw) * c + (long long)g * 8, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[r * 3 + s][j] += v[j] * d[j];
        }
      }
    }
  }
  float* dst = part + (long long)blockIdx.y * kh * kw * c;
  for (int r = 0; r < kh; ++r)
    for (int s = 0; s < kw; ++s) {
      const int q = r * 3 + s;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = acc[q][j];
      __syncthreads();
      if (tr == 0 && g < groups) {
        float sum[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[j] = red[tg][j];
        for (int l = 1; l < RL; ++l)
#pragma unroll
          for (int j = 0; j < 8; ++j) sum[j] += red[l * GT + tg][j];
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[(r * kw + s) * c + g * 8 + j] = sum[j];
      }
    }
}

// pass 2: dw[e] += sum over chunks (fixed order), e over kh*kw*c
__global__ __launch_bounds__(256) void dw_bwd_filter_final_kernel(int chunks, int ne, const float* __restrict__ part,
                                                                  float* __restrict__ dw) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= ne) return;
  float s = 0.f;
  for (int k = 0; k < chunks; ++k) s += part[(long long)k * ne + e];
  dw[e] += s;
}

static int grid_n(long long work) { return (int)std::max<long long>(1, std::min<long long>(8192, (work + 255) / 256)); }

}  // namespace fpnmt

using namespace fpnmt;

// typed launches (the C-ABI takes void* activations)
template <typename T>
static void bn_stats_t(const ColGrid& G, long long rows, int c, const void* x, double* part, float* mean, float* var,
                       float* mm, float* mv, float momentum, hipStream_t s) {
  hipLaunchKernelGGL((bn_stats_part_kernel<T>), dim3(G.gx, G.gy), dim3(256), 0, s, rows, c, G.rpc, (const T*)x, part);
  hipLaunchKernelGGL((bn_stats_final_kernel<T>), dim3(cdiv(c, 64)), dim3(256), 0, s, rows, c, G.gy, (const T*)x,
                     (const double*)part, mean, var, mm, mv, momentum);
}
template <typename T>
static void bn_apply_t(long long n8, int c, const void* x, const float* mean, const float* var, const float* gamma,
                       const float* beta, float eps, int act, const void* res, void* y, hipStream_t s) {
  hipLaunchKernelGGL((bn_apply_kernel<T>), dim3(grid_n(n8)), dim3(256), 0, s, n8, c, (const T*)x, mean, var, gamma,
                     beta, eps, act, (const T*)res, (T*)y);
}
template <typename T>
static void bn_bwd_t(const ColGrid& G, long long rows, int c, const void* x, const float* mean, const float* var,
                     const float* gamma, float eps, int act, const void* y, const void* dy, void* dx, double* part,
                     float* sums, float* dgamma, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL((bn_bwd_part_kernel<T>), dim3(G.gx, G.gy), dim3(256), 0, s, rows, c, G.rpc, (const T*)x, mean,
                     var, eps, act, (const T*)y, (const T*)dy, part);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(c, 64)), dim3(256), 0, s, c, G.gy, (const double*)part, sums,
                     dgamma, dbeta);
  const long long n8 = rows * (c / 8);
  hipLaunchKernelGGL((bn_bwd_dx_kernel<T>), dim3(grid_n(n8)), dim3(256), 0, s, rows, c, (const T*)x, mean, var, gamma,
                     eps, act, (const T*)y, (const T*)dy, (const float*)sums, 1.f / (float)rows, nullptr, (T*)dx);
}
template <typename T>
static void dw_fwd_t(long long work, int n, int h, int w, int c, int kh, int kw, int st, int pt, int pl, int ho,
                     int wo, const void* x, const float* wt, void* y, hipStream_t s) {
  hipLaunchKernelGGL((dw_fwd_kernel<T>), dim3(grid_n(work)), dim3(256), 0, s, n, h, w, c, kh, kw, st, pt, pl, ho, wo,
                     (const T*)x, wt, (T*)y);
}
template <typename T>
static void dw_bwd_data_t(long long work, int n, int h, int w, int c, int kh, int kw, int st, int pt, int pl, int ho,
                          int wo, const void* dy, const float* wt, void* dx, hipStream_t s) {
  hipLaunchKernelGGL((dw_bwd_data_kernel<T>), dim3(grid_n(work)), dim3(256), 0, s, n, h, w, c, kh, kw, st, pt, pl, ho,
                     wo, (const T*)dy, wt, (T*)dx);
}
template <typename T>
static void dw_bwd_filter_t(const ColGrid& G, int n, int h, int w, int c, int kh, int kw, int st, int pt, int pl,
                            int ho, int wo, const void* x, const void* dy, float* part, float* dw, hipStream_t s) {
  const int ne = kh * kw * c;
  hipLaunchKernelGGL((dw_bwd_filter_part_kernel<T>), dim3(G.gx, G.gy), dim3(256), 0, s, n, h, w, c, kh, kw, st, pt,
                     pl, ho, wo, G.rpc, (const T*)x, (const T*)dy, part);
  hipLaunchKernelGGL(dw_bwd_filter_final_kernel, dim3(cdiv(ne, 256)), dim3(256), 0, s, G.gy, ne, (const float*)part,
                     dw);
}

static int bn_check(int dtype, long long rows, int c) {
  if (dtype != FPNMT_BF16 && dtype != FPNMT_F32) return fail(FPNMT_E_ARG, "batchnorm: bad dtype");
  if (c <= 0 || c % 8) return fail(FPNMT_E_UNSUPPORTED, "batchnorm: channels must be a positive multiple of 8");
  if (rows < 0) return fail(FPNMT_E_ARG, "batchnorm: negative rows");
  return 0;
}

extern "C" {

int fpnmt_bn_stats(int dtype, long long rows, int c, const void* x, float* mean, float* var, float* moving_mean,
                   float* moving_var, float momentum, fpnmt_stream_t stream) {
  int e = bn_check(dtype, rows, c);
  if (e) return e;
  if (rows == 0) return 0;
  if (!x || !mean || !var || (!moving_mean != !moving_var)) return fail(FPNMT_E_ARG, "bn_stats: null pointer");
  const ColGrid G = col_grid(rows, c);
  double* part = (double*)scratch_f32((long long)G.gy * 4 * c);
  if (!part) return fail(FPNMT_E_ARG, "bn_stats: needs the fpnmt workspace");
  if (dtype == FPNMT_BF16)
    bn_stats_t<bf16>(G, rows, c, x, part, mean, var, moving_mean, moving_var, momentum, S(stream));
  else
    bn_stats_t<float>(G, rows, c, x, part, mean, var, moving_mean, moving_var, momentum, S(stream));
  return check_launch("bn_stats");
}

int fpnmt_bn_apply(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                   const float* gamma, const float* beta, float eps, int act, const void* residual, void* y,
                   fpnmt_stream_t stream) {
  int e = bn_check(dtype, rows, c);
  if (e) return e;
  if (rows == 0) return 0;
  if (!x || !mean || !var || !gamma || !beta || !y) return fail(FPNMT_E_ARG, "bn_apply: null pointer");
  const long long n8 = rows * (c / 8);
  if (dtype == FPNMT_BF16)
    bn_apply_t<bf16>(n8, c, x, mean, var, gamma, beta, eps, act, residual, y, S(stream));
  else
    bn_apply_t<float>(n8, c, x, mean, var, gamma, beta, eps, act, residual, y, S(stream));
  return check_launch("bn_apply");
}

int fpnmt_bn_bwd(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                 const float* gamma, float eps, int act, const void* y, const void* dy, void* dx, float* dgamma,
                 float* dbeta, fpnmt_stream_t stream) {
  int e = bn_check(dtype, rows, c);
  if (e) return e;
  if (rows == 0) return 0;
  if (!x || !mean || !var || !gamma || !dy || !dx || (act != FPNMT_ACT_NONE && !y))
    return fail(FPNMT_E_ARG, "bn_bwd: null pointer");
  const ColGrid G = col_grid(rows, c);
  float* ws = scratch_f32((long long)G.gy * 4 * c + 2 * c);
  if (!ws) return fail(FPNMT_E_ARG, "bn_bwd: needs the fpnmt workspace");
  double* part = (double*)ws;
  float* sums = ws + (long long)G.gy * 4 * c;
  if (dtype == FPNMT_BF16)
    bn_bwd_t<bf16>(G, rows, c, x, mean, var, gamma, eps, act, y, dy, dx, part, sums, dgamma, dbeta, S(stream));
  else
    bn_bwd_t<float>(G, rows, c, x, mean, var, gamma, eps, act, y, dy, dx, part, sums, dgamma, dbeta, S(stream));
  return check_launch("bn_bwd");
}

int fpnmt_bn_stats_sums(int dtype, long long rows, int c, const void* x, double* sums, fpnmt_stream_t stream) {
  int e = bn_check(dtype, rows, c);
  if (e) return e;
  if (!sums) return fail(FPNMT_E_ARG, "bn_stats_sums: null pointer");
  if (rows == 0) return zero_fill(sums, (size_t)(2 * c + 1) * sizeof(double), S(stream));
  if (!x) return fail(FPNMT_E_ARG, "bn_stats_sums: null pointer");
  const ColGrid G = col_grid(rows, c);
  double* part = (double*)scratch_f32((long long)G.gy * 4 * c);
  if (!part) return fail(FPNMT_E_ARG, "bn_stats_sums: needs the fpnmt workspace");
  if (dtype == FPNMT_BF16) {
    hipLaunchKernelGGL((bn_stats_part_kernel<bf16>), dim3(G.gx, G.gy), dim3(256), 0, S(stream), rows, c, G.rpc,
                       (const bf16*)x, part);
    hipLaunchKernelGGL((bn_sums_final_kernel<bf16>), dim3(cdiv(c, 64)), dim3(256), 0, S(stream), rows, c, G.gy,
                       (const bf16*)x, (const double*)part, sums);
  } else {
    hipLaunchKernelGGL((bn_stats_part_kernel<float>), dim3(G.gx, G.gy), dim3(256), 0, S(stream), rows, c, G.rpc,
                       (const float*)x, part);
    hipLaunchKernelGGL((bn_sums_final_kernel<float>), dim3(cdiv(c, 64)), dim3(256), 0, S(stream), rows, c, G.gy,
                       (const float*)x, (const double*)part, sums);
  }
  return check_launch("bn_stats_sums");
}

int fpnmt_bn_stats_finalize(int c, const double* sums, float* mean, float* var, float* moving_mean,
                            float* moving_var, float momentum, fpnmt_stream_t stream) {
  if (c <= 0 || c % 8) return fail(FPNMT_E_UNSUPPORTED, "bn_stats_finalize: channels must be a positive multiple of 8");
  if (!sums || !mean || !var || (!moving_mean != !moving_var)) return fail(FPNMT_E_ARG, "bn_stats_finalize: null pointer");
  hipLaunchKernelGGL(bn_stats_from_sums_kernel, dim3(cdiv(c, 256)), dim3(256), 0, S(stream), c, sums, mean, var,
                     moving_mean, moving_var, momentum);
  return check_launch("bn_stats_finalize");
}

int fpnmt_bn_bwd_sums(int dtype, long long rows, int c, const void* x, const float* mean, const float* var, float eps,
                      int act, const void* y, const void* dy, double* sums, float* dgamma, float* dbeta,
                      fpnmt_stream_t stream) {
  int e = bn_check(dtype, rows, c);
  if (e) return e;
  if (!sums) return fail(FPNMT_E_ARG, "bn_bwd_sums: null pointer");
  if (rows == 0) return zero_fill(sums, (size_t)(2 * c + 1) * sizeof(double), S(stream));
  if (!x || !mean || !var || !dy || (act != FPNMT_ACT_NONE && !y)) return fail(FPNMT_E_ARG, "bn_bwd_sums: null pointer");
  const ColGrid G = col_grid(rows, c);
  double* part = (double*)scratch_f32((long long)G.gy * 4 * c);
  if (!part) return fail(FPNMT_E_ARG, "bn_bwd_sums: needs the fpnmt workspace");
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((bn_bwd_part_kernel<bf16>), dim3(G.gx, G.gy), dim3(256), 0, S(stream), rows, c, G.rpc,
                       (const bf16*)x, mean, var, eps, act, (const bf16*)y, (const bf16*)dy, part);
  else
    hipLaunchKernelGGL((bn_bwd_part_kernel<float>), dim3(G.gx, G.gy), dim3(256), 0, S(stream), rows, c, G.rpc,
                       (const float*)x, mean, var, eps, act, (const float*)y, (const float*)dy, part);
  hipLaunchKernelGGL(bn_bwd_sums_final_kernel, dim3(cdiv(c, 64)), dim3(256), 0, S(stream), rows, c, G.gy,
                     (const double*)part, sums, dgamma, dbeta);
  return check_launch("bn_bwd_sums");
}

int fpnmt_bn_bwd_dx(int dtype, long long rows, int c, const void* x, const float* mean, const float* var,
                    const float* gamma, float eps, int act, const void* y, const void* dy, const double* sums,
                    void* dx, fpnmt_stream_t stream) {
  int e = bn_check(dtype, rows, c);
  if (e) return e;
  if (rows == 0) return 0;
  if (!x || !mean || !var || !gamma || !dy || !dx || !sums || (act != FPNMT_ACT_NONE && !y))
    return fail(FPNMT_E_ARG, "bn_bwd_dx: null pointer");
  float* fs = scratch_f32(2 * c + 1);
  if (!fs) return fail(FPNMT_E_ARG, "bn_bwd_dx: needs the fpnmt workspace");
  hipLaunchKernelGGL(bn_sums_to_f32_kernel, dim3(cdiv(2 * c + 1, 256)), dim3(256), 0, S(stream), c, sums, fs);
  const long long n8 = rows * (c / 8);
  const float* inv_n = fs + 2 * c;
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((bn_bwd_dx_kernel<bf16>), dim3(grid_n(n8)), dim3(256), 0, S(stream), rows, c, (const bf16*)x,
                       mean, var, gamma, eps, act, (const bf16*)y, (const bf16*)dy, (const float*)fs, 0.f, inv_n,
                       (bf16*)dx);
  else
    hipLaunchKernelGGL((bn_bwd_dx_kernel<float>), dim3(grid_n(n8)), dim3(256), 0, S(stream), rows, c, (const float*)x,
                       mean, var, gamma, eps, act, (const float*)y, (const float*)dy, (const float*)fs, 0.f, inv_n,
                       (float*)dx);
  return check_launch("bn_bwd_dx");
}

static int dw_check(int dtype, int n, int h, int w, int c, int kh, int kw, int st) {
  if (dtype != FPNMT_BF16 && dtype != FPNMT_F32) return fail(FPNMT_E_ARG, "depthwise: bad dtype");
  if (c <= 0 || c % 8) return fail(FPNMT_E_UNSUPPORTED, "depthwise: channels must be a positive multiple of 8");
  if (kh < 1 || kw < 1 || kh > 3 || kw > 3 || st < 1) return fail(FPNMT_E_UNSUPPORTED, "depthwise: kernel <= 3x3");
  if (n < 0 || h < 0 || w < 0) return fail(FPNMT_E_ARG, "depthwise: negative size");
  return 0;
}

int fpnmt_depthwise_fwd(int dtype, int n, int h, int w, int c, int kh, int kw, int stride, int pad_t, int pad_b,
                        int pad_l, int pad_r, const void* x, const float* w_hwc, void* y, fpnmt_stream_t stream) {
  int e = dw_check(dtype, n, h, w, c, kh, kw, stride);
  if (e) return e;
  const int ho = (h + pad_t + pad_b - kh) / stride + 1, wo = (w + pad_l + pad_r - kw) / stride + 1;
  if (n == 0 || ho <= 0 || wo <= 0) return 0;
  if (!x || !w_hwc || !y) return fail(FPNMT_E_ARG, "depthwise_fwd: null pointer");
  const long long work = (long long)n * ho * wo * (c / 8);
  if (dtype == FPNMT_BF16)
    dw_fwd_t<bf16>(work, n, h, w, c, kh, kw, stride, pad_t, pad_l, ho, wo, x, w_hwc, y, S(stream));
  else
    dw_fwd_t<float>(work, n, h, w, c, kh, kw, stride, pad_t, pad_l, ho, wo, x, w_hwc, y, S(stream));
  return check_launch("depthwise_fwd");
}

int fpnmt_depthwise_bwd_data(int dtype, int n, int h, int w, int c, int kh, int kw, int stride, int pad_t, int pad_b,
                             int pad_l, int pad_r, const void* dy, const float* w_hwc, void* dx,
                             fpnmt_stream_t stream) {
  int e = dw_check(dtype, n, h, w, c, kh, kw, stride);
  if (e) return e;
  const int ho = (h + pad_t + pad_b - kh) / stride + 1, wo = (w + pad_l + pad_r - kw) / stride + 1;
  if ((long long)n * h * w == 0) return 0;
  if (!dy || !w_hwc || !dx) return fail(FPNMT_E_ARG, "depthwise_bwd_data: null pointer");
  const long long work = (long long)n * h * w * (c / 8);
  if (dtype == FPNMT_BF16)
    dw_bwd_data_t<bf16>(work, n, h, w, c, kh, kw, stride, pad_t, pad_l, std::max(ho, 0), std::max(wo, 0), dy, w_hwc,
                        dx, S(stream));
  else
    dw_bwd_data_t<float>(work, n, h, w, c, kh, kw, stride, pad_t, pad_l, std::max(ho, 0), std::max(wo, 0), dy, w_hwc,
                         dx, S(stream));
  return check_launch("depthwise_bwd_data");
}

int fpnmt_depthwise_bwd_filter(int dtype, int n, int h, int w, int c, int kh, int kw, int stride, int pad_t,
                               int pad_b, int pad_l, int pad_r, const void* x, const void* dy, float* dw_hwc,
                               fpnmt_stream_t stream) {
  int e = dw_check(dtype, n, h, w, c, kh, kw, stride);
  if (e) return e;
  const int ho = (h + pad_t + pad_b - kh) / stride + 1, wo = (w + pad_l + pad_r - kw) / stride + 1;
  if (n == 0 || ho <= 0 || wo <= 0) return 0;
  if (!x || !dy || !dw_hwc) return fail(FPNMT_E_ARG, "depthwise_bwd_filter: null pointer");
  const long long npix = (long long)n * ho * wo;
  const ColGrid G = col_grid(npix, c);
  const int ne = kh * kw * c;
  float* part = scratch_f32((long long)G.gy * ne);
  if (!part) return fail(FPNMT_E_ARG, "depthwise_bwd_filter: needs the fpnmt workspace");
  if (dtype == FPNMT_BF16)
    dw_bwd_filter_t<bf16>(G, n, h, w, c, kh, kw, stride, pad_t, pad_l, ho, wo, x, dy, part, dw_hwc, S(stream));
  else
    dw_bwd_filter_t<float>(G, n, h, w, c, kh, kw, stride, pad_t, pad_l, ho, wo, x, dy, part, dw_hwc, S(stream));
  return check_launch("depthwise_bwd_filter");
}

}  // extern "C"
