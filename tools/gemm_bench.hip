// Microbenchmark of gemm_kernel tile/BK variants on the hot conv shapes of the
// C2 step (bf16, B=32, 224^2). Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_bench.hip -o gpurun_out/gemm_bench
// Prints TFLOP/s per (shape, variant). Not part of the library.
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <functional>

namespace fpnmt {
SplitWs g_split_ws;
void set_error(const std::string&) {}
int fail(int code, const std::string&) { return code; }
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : -3; }
}  // namespace fpnmt
using namespace fpnmt;

struct Shape { const char* name; int mode; int n, h, w, c, k, r, stride, pad; int res = 0; };
static const void* g_res = nullptr;  // residual operand for shapes with res = 1

static void setup_fwd(GemmParams& p, const Shape& s, const void* x, const void* w, void* y) {
  memset(&p, 0, sizeof(p));
  int ho = (s.h + 2 * s.pad - s.r) / s.stride + 1, wo = (s.w + 2 * s.pad - s.r) / s.stride + 1;
  p.M = s.n * ho * wo; p.N = s.k; p.K = s.r * s.r * s.c;
  p.A = x; p.B = w; p.C = y; p.ldb = p.K; p.ldc = s.k; p.ldr = s.k;
  p.batch_inner = 1; p.alpha = 1.f;
  p.H = s.h; p.W = s.w; p.Cc = s.c; p.Ho = ho; p.Wo = wo; p.Rk = s.r; p.Sk = s.r; p.sh = p.sw = s.stride;
  p.pt = p.pl = s.pad;
  p.fd_HoWo = make_fastdiv(ho * wo); p.fd_Wo = make_fastdiv(wo); p.fd_C = make_fastdiv(s.c); p.fd_S = make_fastdiv(s.r);
  p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
  p.act = FPNMT_ACT_RELU; p.split_k = 1;
  if (s.res) p.R = g_res;
}
static void setup_wgrad(GemmParams& p, const Shape& s, const void* x, const void* dz, void* dw) {
  memset(&p, 0, sizeof(p));
  int ho = (s.h + 2 * s.pad - s.r) / s.stride + 1, wo = (s.w + 2 * s.pad - s.r) / s.stride + 1;
  p.M = s.r * s.r * s.c; p.N = s.k; p.K = s.n * ho * wo;
  p.A = x; p.B = dz; p.C = dw; p.ldb = s.k; p.ldc = s.k;
  p.batch_inner = 1; p.alpha = 1.f;
  p.H = s.h; p.W = s.w; p.Cc = s.c; p.Ho = ho; p.Wo = wo; p.Rk = s.r; p.Sk = s.r; p.sh = p.sw = s.stride;
  p.pt = p.pl = s.pad;
  p.fd_HoWo = make_fastdiv(ho * wo); p.fd_Wo = make_fastdiv(wo); p.fd_C = make_fastdiv(s.c); p.fd_S = make_fastdiv(s.r);
  p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
  p.accumulate = 2; p.c_f32 = 1;
}

template <int BM, int BN, int WM, int WN, int AM, int BMODE, int BK>
static void launch(GemmParams p, hipStream_t st, int split) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  const int nkt = (p.K + BK - 1) / BK;
  const int per = (nkt + split - 1) / split;
  p.k_per_split = per * BK; p.split_k = (nkt + per - 1) / per;
  hipLaunchKernelGGL((gemm_kernel<bf16, BM, BN, WM, WN, AM, BMODE, true, BK>), dim3(p.tiles_m * p.tiles_n, p.split_k, 1),
                     dim3(64 * WM * WN), 0, st, p);
}

static const void* g_zero = nullptr;
template <int BM, int BN, int WM, int WN, int NT = 512, int STAGES = 3>
static void launch_pipe(GemmParams p, hipStream_t st, int) {
  if (p.K % 64 || p.Cc % 64) return;
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  p.split_k = 1; p.k_per_split = p.K; p.zero16 = g_zero;
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, WM, WN, A_IM2COL, NT, STAGES>), dim3(p.tiles_m * p.tiles_n, 1, 1), dim3(NT), 0, st, p);
}
static void no_wgrad(GemmParams, hipStream_t, int) {}

struct Var { const char* name; std::function<void(GemmParams, hipStream_t, int)> fwd, wg; };

int main() {
  std::vector<Shape> shapes = {
      {"P3 subnet 3x3 256->256 @28", 0, 32, 28, 28, 256, 256, 3, 1, 1},
      {"res2 3x3 64->64 @56", 0, 32, 56, 56, 64, 64, 3, 1, 1},
      {"res3 3x3 128->128 @28", 0, 32, 28, 28, 128, 128, 3, 1, 1},
      {"res2 1x1 64->256 @56", 0, 32, 56, 56, 64, 256, 1, 1, 0},
      {"res4 3x3 256->256 @14", 0, 32, 14, 14, 256, 256, 3, 1, 1},
      {"res5 3x3 512->512 @7", 0, 32, 7, 7, 512, 512, 3, 1, 1},
      {"FE out 3x3 256->512 @14", 0, 32, 14, 14, 256, 512, 3, 1, 1},
      {"res2 1x1 64->256 @56 +R", 0, 32, 56, 56, 64, 256, 1, 1, 0, 1},
      {"res3 1x1 128->512 @28 +R", 0, 32, 28, 28, 128, 512, 1, 1, 0, 1},
      {"res4 1x1 256->1024 @14 +R", 0, 32, 14, 14, 256, 1024, 1, 1, 0, 1},
      {"res2 1x1 256->64 @56", 0, 32, 56, 56, 256, 64, 1, 1, 0},
      {"b64 res2 1x1 64->256 @56 +R", 0, 64, 56, 56, 64, 256, 1, 1, 0, 1},
      {"b64 res3 1x1 128->512 @28 +R", 0, 64, 28, 28, 128, 512, 1, 1, 0, 1},
      {"b64 res4 1x1 256->1024 @14 +R", 0, 64, 14, 14, 256, 1024, 1, 1, 0, 1},
      {"b64 res4 3x3 256->256 @14", 0, 64, 14, 14, 256, 256, 3, 1, 1},
      {"P5 3x3 256->256 @7", 0, 32, 7, 7, 256, 256, 3, 1, 1},
      {"P5-P7 3x3 256->256 @8", 0, 32, 8, 8, 256, 256, 3, 1, 1},
  };
  std::vector<Var> vars = {
      {"128x128 w2x2 BK32", launch<128, 128, 2, 2, A_IM2COL, B_NK, 32>, launch<128, 128, 2, 2, A_IM2COL_T, B_KN, 32>},
      {"128x128 w2x2 BK64", launch<128, 128, 2, 2, A_IM2COL, B_NK, 64>, launch<128, 128, 2, 2, A_IM2COL_T, B_KN, 64>},
      {"128x64 w2x2 BK32", launch<128, 64, 2, 2, A_IM2COL, B_NK, 32>, launch<128, 64, 2, 2, A_IM2COL_T, B_KN, 32>},
      {"128x64 w2x2 BK64", launch<128, 64, 2, 2, A_IM2COL, B_NK, 64>, launch<128, 64, 2, 2, A_IM2COL_T, B_KN, 64>},
      {"64x64 w2x2 BK32", launch<64, 64, 2, 2, A_IM2COL, B_NK, 32>, launch<64, 64, 2, 2, A_IM2COL_T, B_KN, 32>},
      {"64x64 w2x2 BK64", launch<64, 64, 2, 2, A_IM2COL, B_NK, 64>, launch<64, 64, 2, 2, A_IM2COL_T, B_KN, 64>},
      {"256x128 w4x2 BK32", launch<256, 128, 4, 2, A_IM2COL, B_NK, 32>, launch<256, 128, 4, 2, A_IM2COL_T, B_KN, 32>},
      {"128x256 w2x4 BK32", launch<128, 256, 2, 4, A_IM2COL, B_NK, 32>, launch<128, 256, 2, 4, A_IM2COL_T, B_KN, 32>},
      {"256x128 w4x2 BK64", launch<256, 128, 4, 2, A_IM2COL, B_NK, 64>, launch<256, 128, 4, 2, A_IM2COL_T, B_KN, 64>},
      {"pipe 128x256 glds3", launch_pipe<128, 256, 2, 4>, no_wgrad},
      {"pipe 256x128 glds3", launch_pipe<256, 128, 4, 2>, no_wgrad},
      {"pipe 256x64 glds3", launch_pipe<256, 64, 8, 1>, no_wgrad},
      {"pipe 64x64 nt256", launch_pipe<64, 64, 2, 2, 256>, no_wgrad},
      {"pipe 128x64 nt256", launch_pipe<128, 64, 2, 2, 256>, no_wgrad},
      {"pipe 64x128 nt256", launch_pipe<64, 128, 2, 2, 256>, no_wgrad},
      {"pipe 128x128 nt256", launch_pipe<128, 128, 2, 2, 256>, no_wgrad},
      {"pipe 64x64 nt256 s4", launch_pipe<64, 64, 2, 2, 256, 4>, no_wgrad},
      {"pipe 64x64 nt256 s5", launch_pipe<64, 64, 2, 2, 256, 5>, no_wgrad},
      {"pipe 64x128 nt256 s4", launch_pipe<64, 128, 2, 2, 256, 4>, no_wgrad},
      {"pipe 64x128 nt256 s5", launch_pipe<64, 128, 2, 2, 256, 5>, no_wgrad},
      {"pipe 128x64 nt256 s5", launch_pipe<128, 64, 2, 2, 256, 5>, no_wgrad},
  };
  const size_t maxe = 64ull * 56 * 56 * 256;
  bf16 *x, *w, *y;
  float* dw;
  hipMalloc(&x, maxe * 2); hipMalloc(&w, 9ull * 512 * 512 * 2); hipMalloc(&y, maxe * 2); hipMalloc(&dw, 9ull * 512 * 512 * 4);
  std::vector<bf16> hx(maxe);
  for (size_t i = 0; i < maxe; ++i) hx[i] = (bf16)(((i * 2654435761u) % 2001) / 1000.f - 1.f);
  hipMemcpy(x, hx.data(), maxe * 2, hipMemcpyHostToDevice);
  hipMemcpy(y, hx.data(), maxe * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hx.data(), 9ull * 512 * 512 * 2, hipMemcpyHostToDevice);
  bf16* res;
  hipMalloc(&res, maxe * 2);
  hipMemcpy(res, hx.data(), maxe * 2, hipMemcpyHostToDevice);
  g_res = res;
  void* zp;
  hipMalloc(&zp, 256);
  hipMemset(zp, 0, 256);
  g_zero = zp;
  hipStream_t st; hipStreamCreate(&st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* filt = getenv("GB_FILTER");
  const int passes = getenv("GB_FWD_ONLY") ? 1 : 2;
  for (auto& s : shapes) {
    if (filt && !strstr(s.name, filt)) continue;
    for (int pass = 0; pass < passes; ++pass) {
      for (auto& v : vars) {
        if (getenv("GB_VAR") && !strstr(v.name, getenv("GB_VAR"))) continue;
        GemmParams p;
        if (pass == 0) setup_fwd(p, s, x, w, y); else setup_wgrad(p, s, x, y, dw);
        double flop = 2.0 * p.M * p.N * (double)p.K;
        int split = 1;
        if (pass == 1) {  // split-K to fill the chip
          int tiles = 1;  // rough: aim at ~512 blocks
          (void)tiles;
          split = 8;
        }
        auto fn = pass == 0 ? v.fwd : v.wg;
        for (int i = 0; i < 3; ++i) fn(p, st, split);
        hipStreamSynchronize(st);
        const int it = 20;
        hipEventRecord(e0, st);
        for (int i = 0; i < it; ++i) fn(p, st, split);
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        if (hipGetLastError() != hipSuccess) { printf("launch error\n"); return 1; }
        printf("%-28s %-5s %-20s %8.1f us %7.1f TF\n", s.name, pass == 0 ? "fwd" : "wgrad", v.name, ms * 1e3,
               flop / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
