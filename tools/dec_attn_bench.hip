// Decode-attention variants on the C5 shapes (256 images x beam 8 = 2048
// rows, 8 heads x depth 64, bf16): the self-attention over the K/V cache at
// lk = 1 .. 32 (cache rows through the src table, rows of the same image's
// beams) and the cross-attention over the 16 encoder positions of each image
// (row_div 8). Each variant: 50 launches captured into one hipGraph and
// replayed (in-graph gaps included), max |diff| against the lane-per-position
// kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dec_attn_bench.hip -o tools/bin_r6/dec_attn_bench
// Not part of the library.
#include "../fpn-mt-image-captioning_amd/csrc/decode.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>
#include <cmath>

namespace fpnmt {
void set_error(const std::string&) {}
int fail(int code, const std::string&) { return code; }
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : -3; }
}  // namespace fpnmt

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Case { const char* name; int lk; bool self; };
struct Args {
  int rows, heads, lk; float scale; const bf16* q; long long ldq; const bf16* kv; long long rs, ps, ko, vo;
  const int32_t* src; int src_ld, row_div; bf16* out; long long ldo;
};
typedef std::function<void(const Args&, hipStream_t)> Fn;

static void old_kernel(const Args& a, hipStream_t st) {
  hipLaunchKernelGGL((decode_attn_kernel<bf16>), dim3(a.rows), dim3(64 * a.heads), 0, st, a.rows, a.heads, 64, a.lk,
                     a.scale, a.q, a.ldq, a.kv, a.rs, a.ps, a.ko, a.vo, a.src, a.src_ld, a.row_div, a.out, a.ldo);
}
template <int PS, bool LATE, int MINW>
static void v_kernel(const Args& a, hipStream_t st) {
  hipLaunchKernelGGL((decode_attn_v_kernel<PS, LATE, MINW>), dim3(a.rows * a.heads), dim3(64), 0, st, a.rows, a.heads,
                     a.lk, a.scale, a.q, a.ldq, a.kv, a.rs, a.ps, a.ko, a.vo, a.src, a.src_ld, a.row_div, a.out, a.ldo);
}

int main() {
  const int R = 2048, H = 8, D = 64, d = H * D, T = 32, NI = 256, LENC = 16, L = 6;
  const long long self_elems = (long long)R * T * 2 * d, cross_elems = (long long)NI * LENC * 2 * L * d;
  std::vector<bf16> hq((size_t)R * d), hkv((size_t)std::max(self_elems, cross_elems));
  srand(7);
  for (auto& v : hq) v = (bf16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  for (auto& v : hkv) v = (bf16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  std::vector<int32_t> hsrc((size_t)R * T);
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < T; ++j) hsrc[(size_t)r * T + j] = (r / 8) * 8 + rand() % 8;
  bf16 *q, *kv, *o0, *o1;
  int32_t* src;
  CK(hipMalloc(&q, hq.size() * 2));
  CK(hipMalloc(&kv, hkv.size() * 2));
  CK(hipMalloc(&o0, (size_t)R * d * 2));
  CK(hipMalloc(&o1, (size_t)R * d * 2));
  CK(hipMalloc(&src, hsrc.size() * 4));
  CK(hipMemcpy(q, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(kv, hkv.data(), hkv.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(src, hsrc.data(), hsrc.size() * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<Case> cases = {{"self lk 1", 1, true},   {"self lk 8", 8, true},   {"self lk 16", 16, true},
                             {"self lk 24", 24, true}, {"self lk 32", 32, true}, {"cross lk 16", LENC, false}};
  std::vector<std::pair<const char*, Fn>> vars = {
      {"old lane/pos 512", old_kernel},
      {"v ps4 early w1", v_kernel<4, false, 1>},
      {"v ps2 early w8", v_kernel<2, false, 8>},
      {"v ps4 late w1", v_kernel<4, true, 1>},
      {"v ps8 early w1", v_kernel<8, false, 1>},  // round-6 table: profiles/r06/dec_attn.txt
  };
  std::vector<bf16> h0((size_t)R * d), h1((size_t)R * d);
  for (const Case& c : cases) {
    Args a;
    a.rows = R; a.heads = H; a.lk = c.lk; a.scale = 0.125f; a.q = q; a.ldq = d; a.kv = kv; a.out = o1; a.ldo = d;
    if (c.self) {
      a.rs = (long long)T * 2 * d; a.ps = 2 * d; a.ko = 0; a.vo = d; a.src = src; a.src_ld = T; a.row_div = 1;
    } else {
      a.rs = (long long)LENC * 2 * L * d; a.ps = 2 * L * d; a.ko = 2 * 3 * d; a.vo = 2 * 3 * d + d; a.src = nullptr;
      a.src_ld = 0; a.row_div = 8;
    }
    const double bytes = c.self ? (double)R * c.lk * 2 * d * 2 : (double)NI * LENC * 2 * d * 2;
    Args a0 = a;
    a0.out = o0;
    old_kernel(a0, st);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h0.data(), o0, h0.size() * 2, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
      v.second(a, st);
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(h1.data(), o1, h1.size() * 2, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < h0.size(); ++i) md = std::max(md, (double)fabsf((float)h0[i] - (float)h1[i]));
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int i = 0; i < 50; ++i) v.second(a, st);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, st));
      for (int it = 0; it < 4; ++it) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 200;
      printf("%-12s %-20s %8.2f us  %7.0f GB/s  maxdiff %.3g\n", c.name, v.first, us, bytes / us * 1e-3, md);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      CK(hipEventDestroy(e0));
      CK(hipEventDestroy(e1));
    }
  }
  return 0;
}
