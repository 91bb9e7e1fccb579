// Variants of the halo-staged 3x3 conv kernel (csrc/gemm_halo.h) against the
// LDS-DMA im2col pipe kernel on the hot 3x3 shapes (bf16, random operands).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/halo_bench.hip -o gpurun_out/halo_bench
// PROBE 1 = no DMA in the K loop (compute structure alone), 2 = no MFMA
// (load pipeline alone). Prints us and TFLOP/s per (shape, variant).
#include "../fpn-mt-image-captioning_amd/csrc/gemm_halo.h"
#include <cstdio>
#include <cstring>
#include <vector>

namespace fpnmt {
SplitWs g_split_ws;
void set_error(const std::string&) {}
int fail(int code, const std::string&) { return code; }
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : -3; }
}  // namespace fpnmt
using namespace fpnmt;

struct Shape { const char* name; int n, h, w, c, k; };

static void setup(GemmParams& p, const Shape& s, const void* x, const void* w, void* y, const void* zero) {
  memset(&p, 0, sizeof(p));
  p.M = s.n * s.h * s.w; p.N = s.k; p.K = 9 * s.c;
  p.A = x; p.B = w; p.C = y; p.ldb = p.K; p.ldc = s.k; p.ldr = s.k;
  p.batch_inner = 1; p.alpha = 1.f;
  p.H = s.h; p.W = s.w; p.Cc = s.c; p.Ho = s.h; p.Wo = s.w; p.Rk = 3; p.Sk = 3; p.sh = p.sw = 1;
  p.pt = p.pl = 1;
  p.fd_HoWo = make_fastdiv(s.h * s.w); p.fd_Wo = make_fastdiv(s.w); p.fd_C = make_fastdiv(s.c); p.fd_S = make_fastdiv(3);
  p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
  p.act = FPNMT_ACT_RELU; p.split_k = 1; p.k_per_split = p.K;
  p.zero16 = zero;
}

template <int BM, int BN, int WM, int WN, int BST, int PROBE, int RD = 0, int PRIO = 0>
static void run_halo(GemmParams p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_halo_kernel<BM, BN, WM, WN, BST, RD, PRIO, PROBE>), dim3(p.tiles_m * p.tiles_n), dim3(512), 0, st, p);
}
template <int BM, int BN, int WM, int WN>
static void run_pipe(GemmParams p, hipStream_t st) {
  p.tiles_m = (p.M + BM - 1) / BM; p.tiles_n = (p.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, WM, WN, A_IM2COL, 512, 3>), dim3(p.tiles_m * p.tiles_n), dim3(512), 0, st, p);
}

int main() {
  const Shape shapes[] = {{"c2_p3_b32", 32, 28, 28, 256, 256}, {"fpn_p3_b64", 64, 28, 28, 256, 256},
                          {"r3_b64", 64, 28, 28, 128, 128}, {"r2_b64", 64, 56, 56, 64, 64}, {"p4_b64", 64, 14, 14, 256, 256}};
  size_t maxx = 0, maxw = 0, maxy = 0;
  for (auto& s : shapes) {
    maxx = std::max(maxx, (size_t)s.n * s.h * s.w * s.c);
    maxw = std::max(maxw, (size_t)9 * s.c * s.k);
    maxy = std::max(maxy, (size_t)s.n * s.h * s.w * s.k);
  }
  std::vector<unsigned short> hx(maxx), hw(maxw);
  unsigned st = 12345;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; float f = ((st >> 8) & 0xffff) / 32768.f - 1.f; unsigned u; memcpy(&u, &f, 4); return (unsigned short)(u >> 16); };
  for (auto& v : hx) v = rnd();
  for (auto& v : hw) v = rnd();
  void *x, *w, *y, *zero;
  hipMalloc(&x, maxx * 2); hipMalloc(&w, maxw * 2); hipMalloc(&y, maxy * 2); hipMalloc(&zero, 256);
  hipMemset(zero, 0, 256);
  hipMemcpy(x, hx.data(), maxx * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), maxw * 2, hipMemcpyHostToDevice);
  hipStream_t s; hipStreamCreate(&s);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  struct V { const char* name; void (*fn)(GemmParams, hipStream_t); bool wide; };
  const V vars[] = {
      {"pipe128x256", run_pipe<128, 256, 2, 4>, true},
      {"halo s3", run_halo<256, 128, 4, 2, 3, 0>, true},
      {"halo s4", run_halo<256, 128, 4, 2, 4, 0>, true},
      {"halo s4 rd", run_halo<256, 128, 4, 2, 4, 0, 1>, true},
      {"halo s4 prio", run_halo<256, 128, 4, 2, 4, 0, 0, 1>, true},
      {"halo s4 rd prio", run_halo<256, 128, 4, 2, 4, 0, 1, 1>, true},

      {"halo s3 noDMA", run_halo<256, 128, 4, 2, 3, 1>, true},
      {"halo s3 rd noDMA", run_halo<256, 128, 4, 2, 3, 1, 1>, true},
      {"halo s3 noMFMA", run_halo<256, 128, 4, 2, 3, 2>, true},
      {"halo s3 mfma-only", run_halo<256, 128, 4, 2, 3, 3>, true},
      {"halo s3 lds-only", run_halo<256, 128, 4, 2, 3, 4>, true},
      {"halo s3 rd lds-only", run_halo<256, 128, 4, 2, 3, 4, 1>, true},
      {"halo64 s3", run_halo<256, 64, 8, 1, 3, 0>, false},
      {"halo64 s4", run_halo<256, 64, 8, 1, 4, 0>, false},
      {"halo64 s4 rd", run_halo<256, 64, 8, 1, 4, 0, 1>, false},

      {"halo64 noDMA", run_halo<256, 64, 8, 1, 3, 1>, false},
  };
  for (int rep = 0; rep < 1; ++rep)
    for (auto& sh : shapes) {
      GemmParams p;
      setup(p, sh, x, w, y, zero);
      const double fl = 2.0 * p.M * p.N * p.K;
      for (auto& v : vars) {
        if (v.wide != (sh.k >= 128)) continue;
        for (int i = 0; i < 3; ++i) v.fn(p, s);
        hipEventRecord(e0, s);
        const int it = 20;
        for (int i = 0; i < it; ++i) v.fn(p, s);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        ms /= it;
        printf("%-11s %-15s %8.1f us %7.1f TF/s\n", sh.name, v.name, ms * 1e3, fl / ms / 1e9);
      }
    }
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
