// Fused identity bottleneck timing probes (csrc/bottleneck.hip built with
// BN_PROBE: bit 0 = no residual loads, bit 1 = no y stores — wrong results,
// where the time goes), batch 64, HIP events over 20 launches after 3.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBN_PROBE=<0..3> tools/bn_bench.hip -o tools/bin_r5/bn_bench<p>
// Not part of the library.
#include "../fpn-mt-image-captioning_amd/csrc/bottleneck.hip"
#include <cstdio>
#include <vector>

namespace fpnmt {
void set_error(const std::string&) {}
int fail(int code, const std::string&) { return code; }
int check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : -3; }
const void* zero16_ptr() { return nullptr; }
}  // namespace fpnmt

template <class F>
static float time_us(F f, hipStream_t st) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(e0, st);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / 20;
}

int main() {
  const int n = 64;
  const size_t xe = (size_t)n * 56 * 56 * 256;
  bf16 *x, *y, *w;
  float* b;
  void* zp;
  hipMalloc(&x, xe * 2); hipMalloc(&y, xe * 2); hipMalloc(&w, 4 << 20); hipMalloc(&b, 4096 * 4); hipMalloc(&zp, 256);
  hipMemset(zp, 0, 256);
  std::vector<bf16> h(xe);
  for (size_t i = 0; i < xe; ++i) h[i] = (bf16)(((i * 2654435761u) % 2001) / 1000.f - 1.f);
  hipMemcpy(x, h.data(), xe * 2, hipMemcpyHostToDevice);
  std::vector<bf16> hw(2 << 20);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (bf16)(((((i * 97) % 1009) / 1009.f) - 0.5f) * 0.05f);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  std::vector<float> hb(4096, 0.01f);
  hipMemcpy(b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  hipStream_t st; hipStreamCreate(&st);
  unsigned long long* dbg;
  hipMalloc(&dbg, 256 * 4 * 8);
  BnArgs a{x, w, w + (1 << 18), w + (1 << 19) + (1 << 18), b, b + 1024, b + 2048, y, (const bf16*)zp, n, dbg};
  auto buckets = [&](const char* name) {
    std::vector<unsigned long long> h(256 * 4);
    hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost);
    double s[4] = {0, 0, 0, 0};
    for (int blk = 0; blk < 256; ++blk)
      for (int q = 0; q < 4; ++q) s[q] += (double)h[blk * 4 + q] / 256;
    const double tot = s[0] + s[1] + s[2] + s[3];
    if (tot > 0)
      printf("  %s s_memtime cycles per block (last launch): wait+barrier %.0f (%.0f %%)  A %.0f (%.0f %%)  "
             "B %.0f (%.0f %%)  C %.0f (%.0f %%)\n", name, s[0], 100 * s[0] / tot, s[1], 100 * s[1] / tot, s[2],
             100 * s[2] / tot, s[3], 100 * s[3] / tot);
  };
  const float t2 = time_us([&] { launch_bottleneck<256, 64, 56, 56, 2, 128, 64, 3, 4, 4, 4, 3>(a, st); }, st);
  buckets("res2");
  const float t3 = time_us([&] { launch_bottleneck<512, 128, 28, 28, 2, 64, 64, 1, 4, 2, 4, 3>(a, st); }, st);
  buckets("res3 TR 2, 3 slots");
  const float t4 = time_us([&] { launch_bottleneck<512, 128, 28, 28, 4, 128, 64, 1, 4, 4, 4, 2>(a, st); }, st);
  buckets("res3 TR 4, 2 slots");
  const float t5 = time_us([&] { launch_bottleneck<256, 64, 56, 56, 2, 128, 64, 3, 4, 4, 4, 2>(a, st); }, st);
  buckets("res2 2 slots");
  printf("res3 TR4 2-slot %.1f us, res2 2-slot %.1f us\n", t4, t5);
  if (hipGetLastError() != hipSuccess) { printf("launch error\n"); return 1; }
  printf("BN_PROBE=%d  res2 56x56x256/64 b64 %.1f us   res3 28x28x512/128 b64 %.1f us\n", BN_PROBE, t2, t3);
  return 0;
}
