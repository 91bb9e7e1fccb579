// Microbenchmark of the row-GEMM paths for the transformer's short-M shapes
// (encoder baseline rows M = 32, decoder rows M = 992; bf16, A_ROW x B_NK,
// bias epilogue). Each variant is captured 100x into one hipGraph and
// replayed, so the figure includes the in-graph launch gaps of the real step.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/small_bench.hip -o gpurun_out/small_bench
// Not part of the library.
#include "../fpn-mt-image-captioning_amd/csrc/gemm_skinny.h"
#if defined(SB_PIPE)
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"
#endif
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <functional>
#include <cmath>

namespace fpnmt {
SplitWs g_split_ws;
void set_error(const std::string&) {}
int fail(int code, const std::string&) { return code; }
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : -3; }
}  // namespace fpnmt
using namespace fpnmt;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Shape { const char* name; int m, n, k; };

static GemmParams setup(const Shape& s, const void* a, const void* b, void* c, const float* bias) {
  GemmParams p;
  memset(&p, 0, sizeof(p));
  p.M = s.m; p.N = s.n; p.K = s.k;
  p.A = a; p.B = b; p.C = c; p.lda = s.k; p.ldb = s.k; p.ldc = s.n; p.ldr = s.n;
  p.batch_inner = 1; p.alpha = 1.f; p.bias = bias;
  p.fd_HoWo = p.fd_Wo = p.fd_C = p.fd_S = p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
  p.split_k = 1; p.k_per_split = s.k;
  return p;
}

static void small8(GemmParams p, hipStream_t st) {
  hipLaunchKernelGGL((gemm_small_kernel<bf16, 8>), dim3(((p.M + 31) / 32) * ((p.N + 63) / 64), 1, 1), dim3(512), 0, st, p);
}
static void small4(GemmParams p, hipStream_t st) {
  hipLaunchKernelGGL((gemm_small_kernel<bf16, 4>), dim3(((p.M + 31) / 32) * ((p.N + 63) / 64), 1, 1), dim3(256), 0, st, p);
}
template <int NW, int CT>
static void skinny(GemmParams p, hipStream_t st) {
  hipLaunchKernelGGL((gemm_skinny_kernel<NW, CT>), dim3(((p.M + 31) / 32) * ((p.N + CT - 1) / CT), 1, 1),
                     dim3(64 * NW), 0, st, p);
}

struct Var { const char* name; std::function<void(GemmParams, hipStream_t)> fn; };

#if defined(SB_PIPE)
// the LDS-DMA pipe kernel on the decoder's short-row shapes (round 5): the
// library's 64x64 4-stage ring (128 blocks at N = 512) against 16x16x32
// MFMA forms and smaller tiles that spread the same GEMM over more CUs
static const void* g_zero = nullptr;
template <int BM, int BN, int WM, int WN, int ST, int SPREAD, int MF>
static void pipe(GemmParams p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  p.zero16 = g_zero;
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, WM, WN, A_ROW, 64 * WM * WN, ST, 1, 64, SPREAD, MF>),
                     dim3(p.tiles_m * p.tiles_n, 1, 1), dim3(64 * WM * WN), 0, st, p);
}
// round 6: the loader-wave kernel (csrc/gemm_pipe.h gemm_pipe_lw_kernel)
template <int BM, int BN, int WM, int WN, int NLW, int ST>
static void lw(GemmParams p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  p.zero16 = g_zero;
  hipLaunchKernelGGL((gemm_pipe_lw_kernel<BM, BN, WM, WN, A_ROW, NLW, ST>), dim3(p.tiles_m * p.tiles_n, 1, 1),
                     dim3(64 * (WM * WN + NLW)), 0, st, p);
}
#endif

// weight-gradient form of the encoder's M = 32-row Dense layers:
// C (in x out, fp32, read-modify-write) += x^T (in x 32) . dy (32 x out)
template <int BM, int BN, int WM, int WN>
static void wg(GemmParams p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  p.k_per_split = ((p.K + 31) / 32) * 32; p.split_k = 1;
  hipLaunchKernelGGL((gemm_kernel<bf16, BM, BN, WM, WN, A_COL, B_KN, true, 0>), dim3(p.tiles_m * p.tiles_n, 1, 1),
                     dim3(64 * WM * WN), 0, st, p);
}
static void wgrad_bench(bf16* a, bf16* b, float* c, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  struct W { int m, n, k; } ws[] = {{512, 512, 32}, {2048, 512, 32}, {512, 2048, 32}, {512, 512, 128}};
  std::vector<Var> vars = {{"wg 64x64", wg<64, 64, 2, 2>}, {"wg 32x32", wg<32, 32, 1, 1>},
                           {"wg 64x32?", wg<64, 64, 2, 2>}};
  for (auto& w : ws) {
    for (int vi = 0; vi < 2; ++vi) {
      auto& v = vars[vi];
      GemmParams p;
      memset(&p, 0, sizeof(p));
      p.M = w.m; p.N = w.n; p.K = w.k;
      p.A = a; p.B = b; p.C = c; p.lda = w.m; p.ldb = w.n; p.ldc = w.n;
      p.batch_inner = 1; p.alpha = 1.f; p.accumulate = 1; p.c_f32 = 1;
      p.fd_HoWo = p.fd_Wo = p.fd_C = p.fd_S = p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int r = 0; r < 100; ++r) v.fn(p, st);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int it = 0; it < 5; ++it) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("wgrad %4dx%4dx%3d %-12s %7.2f us\n", w.m, w.n, w.k, v.name, ms * 1e3 / 500);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
}

int main() {
  std::vector<Shape> shapes = {
      {"enc q/o  32x512x512", 32, 512, 512},     {"enc ffn1 32x2048x512", 32, 2048, 512},
      {"enc ffn2 32x512x2048", 32, 512, 2048},   {"enc qall 32x2048x512", 32, 2048, 512},
      {"dec 992x512x512", 992, 512, 512},        {"dec ffn2 992x512x2048", 992, 512, 2048},
      {"dec ffn1 992x2048x512", 992, 2048, 512}, {"dec qkv 992x1536x512", 992, 1536, 512},
      {"k=16 32x512x16", 32, 512, 16},
  };
#if defined(SB_PIPE)
  shapes = {{"dec 992x512x512", 992, 512, 512}, {"dec ffn2 992x512x2048", 992, 512, 2048},
            {"dec ffn1 992x2048x512", 992, 2048, 512}, {"dec qkv 992x1536x512", 992, 1536, 512},
#if defined(SB_LW)
            // C5 decode steps: 256 images x beam 8 rows
            {"c5 2048x512x512", 2048, 512, 512}, {"c5 ffn2 2048x512x2048", 2048, 512, 2048},
            {"c5 ffn1 2048x2048x512", 2048, 2048, 512}, {"c5 qkv 2048x1536x512", 2048, 1536, 512},
#endif
  };
  std::vector<Var> vars = {{"small<8>", small8},
                           {"pipe64x64 s4 (lib)", pipe<64, 64, 2, 2, 4, 1, 32>},
                           {"pipe64x64 s4 mf16", pipe<64, 64, 2, 2, 4, 1, 16>},
                           {"pipe32x64 s4 mf16", pipe<32, 64, 2, 2, 4, 1, 16>},
                           {"pipe64x32 s4 mf16", pipe<64, 32, 2, 2, 4, 1, 16>},
                           {"pipe32x32 s4 mf16 w1x2", pipe<32, 32, 1, 2, 4, 1, 16>},
                           {"pipe32x64 s8 mf16", pipe<32, 64, 2, 2, 8, 1, 16>},
                           {"pipe64x64 s8 mf16", pipe<64, 64, 2, 2, 8, 1, 16>},
#if defined(SB_LW)
                           {"lw1 64x32 s4", lw<64, 32, 2, 2, 1, 4>},
                           {"lw2 64x32 s4", lw<64, 32, 2, 2, 2, 4>},
                           {"lw2 64x32 s3", lw<64, 32, 2, 2, 2, 3>},
                           {"lw2 64x64 s4", lw<64, 64, 2, 2, 2, 4>},
                           {"lw4 64x64 s4", lw<64, 64, 2, 2, 4, 4>},
                           {"lw2 32x64 s4", lw<32, 64, 2, 2, 2, 4>},
                           {"lw4 128x128 s3", lw<128, 128, 2, 2, 4, 3>},
                           {"lw4 128x64 s4", lw<128, 64, 2, 2, 4, 4>},
                           {"lw2 64x64 s3", lw<64, 64, 2, 2, 2, 3>},
#endif
  };
  {
    void* z;
    CK(hipMalloc(&z, 256));
    CK(hipMemset(z, 0, 256));
    g_zero = z;
  }
#else
  std::vector<Var> vars = {{"small<8>", small8}, {"small<4>", small4},
                           {"skinny<4,32>", skinny<4, 32>}, {"skinny<8,32>", skinny<8, 32>},
                           {"skinny<16,32>", skinny<16, 32>}, {"skinny<8,64>", skinny<8, 64>}};
#endif
  const size_t maxe = 2048ull * 2048;
  bf16 *a, *b, *c, *c_ref;
  float* bias;
  CK(hipMalloc(&a, maxe * 2)); CK(hipMalloc(&b, 2048ull * 2048 * 2));
  CK(hipMalloc(&c, maxe * 2)); CK(hipMalloc(&c_ref, maxe * 2)); CK(hipMalloc(&bias, 2048 * 4));
  {
    std::vector<bf16> h(2048ull * 2048);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (bf16)((float)((i * 2654435761u) % 2001) / 1000.f - 1.f);
    CK(hipMemcpy(a, h.data(), maxe * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, h.data(), 2048ull * 2048 * 2, hipMemcpyHostToDevice));
    std::vector<float> hb(2048);
    for (int i = 0; i < 2048; ++i) hb[i] = 0.01f * (i % 7);
    CK(hipMemcpy(bias, hb.data(), 2048 * 4, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int R = 100;
#if !defined(SB_PIPE)
  {
    float* cw;
    CK(hipMalloc(&cw, 2048ull * 2048 * 4));
    CK(hipMemset(cw, 0, 2048ull * 2048 * 4));
    wgrad_bench(a, b, cw, st, e0, e1);
  }
#endif
  for (auto& s : shapes) {
    // reference result: small<8>
    GemmParams pr = setup(s, a, b, c_ref, bias);
    small8(pr, st);
    CK(hipStreamSynchronize(st));
    std::vector<bf16> ref((size_t)s.m * s.n), got((size_t)s.m * s.n);
    CK(hipMemcpy(ref.data(), c_ref, ref.size() * 2, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
      GemmParams p = setup(s, a, b, c, bias);
      CK(hipMemsetAsync(c, 0, (size_t)s.m * s.n * 2, st));
      v.fn(p, st);
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(got.data(), c, got.size() * 2, hipMemcpyDeviceToHost));
      float md = 0.f;
      for (size_t i = 0; i < got.size(); ++i) md = fmaxf(md, fabsf((float)got[i] - (float)ref[i]));
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int r = 0; r < R; ++r) v.fn(p, st);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int it = 0; it < 5; ++it) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / (5 * R);
      printf("%-24s %-16s %7.2f us  %7.1f TF  maxdiff %.3g\n", s.name, v.name, us,
             2.0 * s.m * s.n * s.k / (us * 1e-6) / 1e12, md);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
