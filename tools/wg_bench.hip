// Weight-gradient kernel variants (dW += im2col(x)^T dz, bf16 in, fp32 out) on
// the C2 step's wgrad shapes (batch 32): gemm_pipe_wg_kernel (the library's
// current choice) against gemm_wide_wg_kernel. Correctness: one split with
// fp32 atomics into a zeroed dW against a naive fp32 reference; timing: the
// split count the library's launcher would pick (one wave of blocks over the
// chip), partial slabs into a scratch buffer (the ordered slab reduce is a
// separate, shared kernel and is not timed). HIP events, 20 launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/wg_bench.hip -o tools/wg_bench
// Not part of the library.
#include "gemm_wide.h"
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <functional>

namespace fpnmt {
SplitWs g_split_ws;
}
using namespace fpnmt;

// n, h, w: input; c -> k channels, r x r, stride; mode A_IM2COL_T (r x r) or A_COL (1x1 rows)
struct Shape { const char* name; int n, h, w, c, k, r, stride; };

static void setup(GemmParams& p, const Shape& s, const void* x, const void* dz, void* dw, const void* zero) {
  memset(&p, 0, sizeof(p));
  const int pad = s.stride == 1 ? s.r / 2 : 0;
  const int ho = (s.h + 2 * pad - s.r) / s.stride + 1, wo = (s.w + 2 * pad - s.r) / s.stride + 1;
  p.M = s.r * s.r * s.c; p.N = s.k; p.K = s.n * ho * wo;
  p.A = x; p.B = dz; p.C = dw; p.lda = s.c; p.ldb = s.k; p.ldc = s.k;
  p.batch_inner = 1; p.alpha = 1.f;
  p.H = s.h; p.W = s.w; p.Cc = s.c; p.Ho = ho; p.Wo = wo; p.Rk = s.r; p.Sk = s.r; p.sh = p.sw = s.stride;
  p.pt = p.pl = pad;
  p.fd_HoWo = make_fastdiv(ho * wo); p.fd_Wo = make_fastdiv(wo); p.fd_C = make_fastdiv(s.c); p.fd_S = make_fastdiv(s.r);
  p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
  p.accumulate = 2; p.c_f32 = 1; p.zero16 = zero;
}

__global__ void ref_kernel(GemmParams p, float* out) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= (long long)p.M * p.N) return;
  const int m = (int)(e / p.N), n = (int)(e % p.N);
  const int tap = m / p.Cc, ch = m % p.Cc, r = tap / p.Sk, s = tap % p.Sk;
  const bf16* x = (const bf16*)p.A;
  const bf16* dz = (const bf16*)p.B;
  float acc = 0.f;
  for (int k = 0; k < p.K; ++k) {
    const int img = k / (p.Ho * p.Wo), rem = k % (p.Ho * p.Wo), ho = rem / p.Wo, wo = rem % p.Wo;
    const int hi = ho * p.sh - p.pt + r, wi = wo * p.sw - p.pl + s;
    if (hi < 0 || hi >= p.H || wi < 0 || wi >= p.W) continue;
    acc += (float)x[(((long long)img * p.H + hi) * p.W + wi) * p.Cc + ch] * (float)dz[(long long)k * p.N + n];
  }
  out[e] = acc;
}

__global__ void diff_kernel(const float* y, const float* ref, long long n, float* out2) {
  __shared__ float smax[256], sref[256];
  float md = 0.f, mr = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    md = fmaxf(md, fabsf(y[i] - ref[i]));
    mr = fmaxf(mr, fabsf(ref[i]));
  }
  smax[threadIdx.x] = md; sref[threadIdx.x] = mr;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 256; ++i) { md = fmaxf(md, smax[i]); mr = fmaxf(mr, sref[i]); }
    atomicMax((int*)&out2[0], __float_as_int(md));
    atomicMax((int*)&out2[1], __float_as_int(mr));
  }
}

static float* g_slab = nullptr;

// splits: 0 = the library's choice (>= 4 K-tiles per split, one wave of blocks), 1 = atomics
template <int BM, int BN, int AM, bool WIDE, int WM, int WN, int SPREAD = 0, int MF = 32>
static void run(GemmParams p, hipStream_t st, int splits) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  const long long tiles = (long long)p.tiles_m * p.tiles_n;
  const long long tot_kt = (p.K + 63) / 64;
  long long kt_per = tot_kt;
  if (splits == 0) kt_per = std::max<long long>(4, (tot_kt + std::max<long long>(1, 256 / tiles) - 1) / std::max<long long>(1, 256 / tiles));
  p.k_per_split = (int)(kt_per * 64);
  p.split_k = (int)((tot_kt + kt_per - 1) / kt_per);
  if (p.split_k > 1) {
    p.C = g_slab; p.ldc = p.N; p.c_split = (long long)p.M * p.N; p.accumulate = 0; p.alpha = 1.f;
  }
  const dim3 grid((unsigned)(tiles * p.split_k));
  if constexpr (WIDE)
    hipLaunchKernelGGL((gemm_wide_wg_kernel<BM, BN, WM, WN, AM>), grid, dim3(64 * WM * WN), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_pipe_wg_kernel<BM, BN, WM, WN, AM, SPREAD, MF>), grid, dim3(64 * WM * WN), 0, st, p);
}

// the library's former path for the 64-channel shapes: gemm_kernel 64x64, BK 64,
// register-staged, split = 768 / blocks (>= 4 K-tiles each), partial slabs
template <int AM>
static void run_old(GemmParams p, hipStream_t st, int splits) {
  p.tiles_m = (p.M + 63) / 64; p.tiles_n = (p.N + 63) / 64;
  const long long blocks = (long long)p.tiles_m * p.tiles_n;
  const int nkt = (p.K + 63) / 64;
  int split = splits == 1 ? 1 : (int)((768 + blocks - 1) / blocks);
  split = std::max(1, std::min(split, nkt / 4));
  const int kt_per = (nkt + split - 1) / split;
  p.k_per_split = kt_per * 64;
  p.split_k = (nkt + kt_per - 1) / kt_per;
  if (p.split_k > 1) {
    p.C = g_slab; p.ldc = p.N; p.c_split = (long long)p.M * p.N; p.c_si = p.c_split; p.c_so = p.c_split;
    p.accumulate = 0; p.alpha = 1.f;
  }
  hipLaunchKernelGGL((gemm_kernel<bf16, 64, 64, 2, 2, AM, B_KN, true, 64>), dim3((unsigned)blocks, p.split_k, 1),
                     dim3(256), 0, st, p);
}

#if defined(WB_HALO)
#include "wg_halo.h"
static void* g_zero_h = nullptr;
// the halo-staged 3x3 kernel on one level (splits 1: straight into dw)
static void run_halo(GemmParams p, hipStream_t st, int splits) {
  HaloArgs a{};
  const int H = p.H, W = p.W, n = p.K / (p.Ho * p.Wo);
  int WS = 8, lws = 3;
  while (WS < W) { WS <<= 1; ++lws; }
  const int RT = 64 / WS;
  a.lv[0] = HaloLevel{(const bf16*)p.A, (const bf16*)p.B, H, W, WS, lws, RT, (H + RT - 1) / RT, 0};
  a.nlv = 1; a.n = n; a.C = p.Cc; a.N = p.N;
  a.tot_kt = n * a.lv[0].rowtiles;
  a.cgroups = p.Cc / 32; a.ngroups = p.N / 128;
  const int tiles = a.cgroups * a.ngroups;
  const int sp = splits == 1 ? 1 : std::max(1, 256 / tiles);
  a.kt_per = (a.tot_kt + sp - 1) / sp;
  a.splits = (a.tot_kt + a.kt_per - 1) / a.kt_per;
  a.slab = a.splits == 1 ? (float*)p.C : g_slab;
  a.zero = g_zero_h;
  hipLaunchKernelGGL(wg_halo3x3_kernel<3>, dim3(tiles * a.splits), dim3(576), 0, st, a);
}
#endif

#if defined(WB_LW)
// the loader-wave form (gemm_pipe_wg_kernel with NLW loader waves), same split choice as run()
template <int BM, int BN, int AM, int WM, int WN, int NLW, int MF = 32>
static void run_lw(GemmParams p, hipStream_t st, int splits) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  const long long tiles = (long long)p.tiles_m * p.tiles_n;
  const long long tot_kt = (p.K + 63) / 64;
  long long kt_per = tot_kt;
  if (splits == 0) kt_per = std::max<long long>(4, (tot_kt + std::max<long long>(1, 256 / tiles) - 1) / std::max<long long>(1, 256 / tiles));
  p.k_per_split = (int)(kt_per * 64);
  p.split_k = (int)((tot_kt + kt_per - 1) / kt_per);
  if (p.split_k > 1) {
    p.C = g_slab; p.ldc = p.N; p.c_split = (long long)p.M * p.N; p.accumulate = 0; p.alpha = 1.f;
  }
  const dim3 grid((unsigned)(tiles * p.split_k));
  hipLaunchKernelGGL((gemm_pipe_wg_kernel<BM, BN, WM, WN, AM, 0, MF, NLW>), grid, dim3(64 * (WM * WN + NLW)), 0, st, p);
}
#endif

struct Var { const char* name; int bm; std::function<void(GemmParams, hipStream_t, int)> t3, col; };

int main() {
  std::vector<Shape> shapes = {
#if defined(WB_HALO)
      {"P3 head 3x3 256->256 @28", 32, 28, 28, 256, 256, 3, 1},
      {"FE out 3x3 256->512 @14", 32, 14, 14, 256, 512, 3, 1},
      {"r3 3x3 128->128 @28", 32, 28, 28, 128, 128, 3, 1},
      {"r4 3x3 256->256 @14", 32, 14, 14, 256, 256, 3, 1},
      {"r5 3x3 512->512 @7", 32, 7, 7, 512, 512, 3, 1},
  };
  if (0) shapes = {
#endif
#if defined(WB_W64)
      {"r2 3x3 64->64 @56", 32, 56, 56, 64, 64, 3, 1},
      {"r2 1x1 256->64 @56", 32, 56, 56, 256, 64, 1, 1},
      {"r2 1x1 64->256 @56", 32, 56, 56, 64, 256, 1, 1},
      {"r3 3x3 128->128 @28", 32, 28, 28, 128, 128, 3, 1},
      {"r5 3x3 512->512 @7", 32, 7, 7, 512, 512, 3, 1},
      {"r5 1x1 2048->512 @7", 32, 7, 7, 2048, 512, 1, 1},
      {"r5 1x1 512->2048 @7", 32, 7, 7, 512, 2048, 1, 1},
  };
  if (0) shapes = {
#endif
      {"P3 head 3x3 256->256 @28", 32, 28, 28, 256, 256, 3, 1},
      {"FE out 3x3 256->512 @14", 32, 14, 14, 256, 512, 3, 1},
      {"r3 3x3 128->128 @28", 32, 28, 28, 128, 128, 3, 1},
      {"r4 3x3 256->256 @14", 32, 14, 14, 256, 256, 3, 1},
      {"r5 3x3 512->512 @7", 32, 7, 7, 512, 512, 3, 1},
      {"P4 head 3x3 256->256 @14", 32, 14, 14, 256, 256, 3, 1},
      {"r4 1x1 1024->256 @14", 32, 14, 14, 1024, 256, 1, 1},
      {"r3 1x1 512->128 @28", 32, 28, 28, 512, 128, 1, 1},
      {"r4 1x1 256->1024 @14", 32, 14, 14, 256, 1024, 1, 1},
      {"r5 1x1 2048->512 @7", 32, 7, 7, 2048, 512, 1, 1},
  };
  std::vector<Var> vars = {
#if defined(WB_LW)
      // round 6: loader waves own the ring's LDS-DMA (gemm_pipe_wg_kernel NLW > 0)
      {"pipe_wg 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4>, run<128, 128, A_COL, false, 2, 4>},
      {"pipe_wg 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2>, run<256, 128, A_COL, false, 4, 2>},
      {"pipe_wg 128x256 w2x4 s3", 128, run<128, 256, A_IM2COL_T, false, 2, 4>, run<128, 256, A_COL, false, 2, 4>},
      {"lw4 128x128 w2x4", 128, run_lw<128, 128, A_IM2COL_T, 2, 4, 4>, run_lw<128, 128, A_COL, 2, 4, 4>},
      {"lw4 128x128 w2x2", 128, run_lw<128, 128, A_IM2COL_T, 2, 2, 4>, run_lw<128, 128, A_COL, 2, 2, 4>},
      {"lw4 256x128 w4x2", 256, run_lw<256, 128, A_IM2COL_T, 4, 2, 4>, run_lw<256, 128, A_COL, 4, 2, 4>},
      {"lw4 128x256 w2x4", 128, run_lw<128, 256, A_IM2COL_T, 2, 4, 4>, run_lw<128, 256, A_COL, 2, 4, 4>},
      {"lw8 128x256 w2x4", 128, run_lw<128, 256, A_IM2COL_T, 2, 4, 8>, run_lw<128, 256, A_COL, 2, 4, 8>},
#elif defined(WB_HALO)
      // round 5: the halo-staged 3x3 kernel (tools/wg_halo.h) against the shipped tiles
      {"pipe_wg 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4>, run<128, 128, A_COL, false, 2, 4>},
      {"pipe_wg 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2>, run<256, 128, A_COL, false, 4, 2>},
      {"pipe_wg 256x256 w4x2 s2", 256, run<256, 256, A_IM2COL_T, false, 4, 2>, run<256, 256, A_COL, false, 4, 2>},
      {"pipe_wg 128x256 w2x4 s3", 128, run<128, 256, A_IM2COL_T, false, 2, 4>, run<128, 256, A_COL, false, 2, 4>},
      {"pipe_wg 128x256 w2x2 s3", 128, run<128, 256, A_IM2COL_T, false, 2, 2>, run<128, 256, A_COL, false, 2, 2>},
      {"pipe_wg 256x128 w2x2 s3", 256, run<256, 128, A_IM2COL_T, false, 2, 2>, run<256, 128, A_COL, false, 2, 2>},
      {"pipe_wg 128x128 w2x2 s4", 128, run<128, 128, A_IM2COL_T, false, 2, 2>, run<128, 128, A_COL, false, 2, 2>},
#elif defined(WB_W64)
      // round 5: 64-wide tile sides (8-chunk LDS rows) and per-chunk filter
      // taps for the 64-channel convs, against the register-staged kernel
      {"old gemm 64x64x64", 64, run_old<A_IM2COL_T>, run_old<A_COL>},
      {"pipe_wg 128x64 w2x2", 128, run<128, 64, A_IM2COL_T, false, 2, 2>, run<128, 64, A_COL, false, 2, 2>},
      {"pipe_wg 256x64 w4x1", 256, run<256, 64, A_IM2COL_T, false, 4, 1>, run<256, 64, A_COL, false, 4, 1>},
      {"pipe_wg 64x256 w1x4", 64, run<64, 256, A_IM2COL_T, false, 1, 4>, run<64, 256, A_COL, false, 1, 4>},
      {"pipe_wg 64x128 w1x2", 64, run<64, 128, A_IM2COL_T, false, 1, 2>, run<64, 128, A_COL, false, 1, 2>},
      {"pipe_wg 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4>, run<128, 128, A_COL, false, 2, 4>},
      {"pipe_wg 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2>, run<256, 128, A_COL, false, 4, 2>},
#elif defined(WB_SPREAD)
      // round 4: the next K-tile's DMA spread between the k-steps (1), + MFMA priority (2)
      {"pipe_wg 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4>, run<128, 128, A_COL, false, 2, 4>},
      {"spread 128x128", 128, run<128, 128, A_IM2COL_T, false, 2, 4, 1>, run<128, 128, A_COL, false, 2, 4, 1>},
      {"spread+prio 128x128", 128, run<128, 128, A_IM2COL_T, false, 2, 4, 2>, run<128, 128, A_COL, false, 2, 4, 2>},
      {"pipe_wg 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2>, run<256, 128, A_COL, false, 4, 2>},
      {"spread 256x128", 256, run<256, 128, A_IM2COL_T, false, 4, 2, 1>, run<256, 128, A_COL, false, 4, 2, 1>},
      {"spread+prio 256x128", 256, run<256, 128, A_IM2COL_T, false, 4, 2, 2>, run<256, 128, A_COL, false, 4, 2, 2>},
#elif defined(WB_MF16)
      // round 5: the 16x16x32 MFMA form (MF 16) against the shipped 32x32x16
      {"pipe_wg 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4>, run<128, 128, A_COL, false, 2, 4>},
      {"mf16 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4, 0, 16>, run<128, 128, A_COL, false, 2, 4, 0, 16>},
      {"pipe_wg 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2>, run<256, 128, A_COL, false, 4, 2>},
      {"mf16 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2, 0, 16>, run<256, 128, A_COL, false, 4, 2, 0, 16>},
      {"mf16 256x128 spread+prio", 256, run<256, 128, A_IM2COL_T, false, 4, 2, 2, 16>,
       run<256, 128, A_COL, false, 4, 2, 2, 16>},
#else
      {"pipe_wg 128x128 w2x4", 128, run<128, 128, A_IM2COL_T, false, 2, 4>, run<128, 128, A_COL, false, 2, 4>},
      {"pipe_wg 256x128 w4x2", 256, run<256, 128, A_IM2COL_T, false, 4, 2>, run<256, 128, A_COL, false, 4, 2>},
      {"wide_wg 128x128 w2x2", 128, run<128, 128, A_IM2COL_T, true, 2, 2>, run<128, 128, A_COL, true, 2, 2>},
      {"wide_wg 256x128 w2x2", 256, run<256, 128, A_IM2COL_T, true, 2, 2>, run<256, 128, A_COL, true, 2, 2>},
      {"wide_wg 128x256 w2x2", 128, run<128, 256, A_IM2COL_T, true, 2, 2>, run<128, 256, A_COL, true, 2, 2>},
#endif
  };
  const size_t maxe = 32ull * 56 * 56 * 256;
  bf16 *x, *dz;
  float *dw, *ref, *d2;
  hipMalloc(&x, maxe * 2); hipMalloc(&dz, maxe * 2); hipMalloc(&dw, 16ull << 20); hipMalloc(&ref, 16ull << 20);
  hipMalloc(&d2, 8); hipMalloc(&g_slab, 256ull << 20);
  std::vector<bf16> h(maxe);
  for (size_t i = 0; i < maxe; ++i) h[i] = (bf16)(((i * 2654435761u) % 2001) / 1000.f - 1.f);
  hipMemcpy(x, h.data(), maxe * 2, hipMemcpyHostToDevice);
  for (size_t i = 0; i < maxe; ++i) h[i] = (bf16)((((i + 77) * 40503u) % 2001) / 1000.f - 1.f);
  hipMemcpy(dz, h.data(), maxe * 2, hipMemcpyHostToDevice);
  void* zp;
  hipMalloc(&zp, 256); hipMemset(zp, 0, 256);
#if defined(WB_HALO)
  g_zero_h = zp;
#endif
  hipStream_t st; hipStreamCreate(&st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* filt = getenv("WB_FILTER");
  const int iters = 20;
  for (auto& s : shapes) {
    if (filt && !strstr(s.name, filt)) continue;
    GemmParams p;
    setup(p, s, x, dz, dw, zp);
    const bool col = s.r == 1 && s.stride == 1;
    const long long outs = (long long)p.M * p.N;
    hipLaunchKernelGGL(ref_kernel, dim3((unsigned)((outs + 255) / 256)), dim3(256), 0, st, p, ref);
    hipStreamSynchronize(st);
    const double flop = 2.0 * p.M * p.N * (double)p.K;
    for (auto& v : vars) {
      if (s.c % 8 && !col) continue;  // a chunk's 8 m rows must stay inside one tap
      auto fn = col ? v.col : v.t3;
      hipMemsetAsync(dw, 0, outs * 4, st);
      fn(p, st, 1);
      hipMemsetAsync(d2, 0, 8, st);
      hipLaunchKernelGGL(diff_kernel, dim3(1024), dim3(256), 0, st, dw, ref, outs, d2);
      float hd[2];
      hipMemcpy(hd, d2, 8, hipMemcpyDeviceToHost);
      for (int i = 0; i < 3; ++i) fn(p, st, 0);
      hipStreamSynchronize(st);
      hipEventRecord(e0, st);
      for (int i = 0; i < iters; ++i) fn(p, st, 0);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= iters;
      if (hipGetLastError() != hipSuccess) { printf("launch error\n"); return 1; }
      printf("%-26s %-24s %8.1f us %7.1f TF  err %.2e%s\n", s.name, v.name, ms * 1e3, flop / (ms * 1e-3) / 1e12,
             hd[0] / hd[1], hd[0] / hd[1] > 1e-3 ? "  BAD" : "");
      fflush(stdout);
    }
  }
  return 0;
}
