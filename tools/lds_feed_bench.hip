// What bounds the implicit-GEMM conv K loop on MI355X? A synthetic K loop with
// the pipe kernel's structure (LDS-DMA ring of STAGES K-tiles, one raw barrier
// per K-tile, counted vmcnt) where the per-K-tile work is set independently:
//   KB     bytes DMA'd into LDS per K-tile (L2-resident source, 16-B chunks)
//   NMF    v_mfma_f32_32x32x16_bf16 per wave per K-tile
//   NRD    ds_read_b128 per wave per K-tile (interleaved with the MFMAs)
// one 512-thread block per CU, 256 blocks, ITERS K-tiles each. Prints us per
// launch, us per K-tile, per-CU DMA GB/s and MFMA-pipe utilisation against
// 32 cycles per MFMA at the measured clock-free bound (cycles from s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lds_feed_bench.hip -o tools/lds_feed_bench
// Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int KB, int STAGES, int NMF, int NRD>
__global__ __launch_bounds__(512) void feed_kernel(const char* __restrict__ src, long long src_bytes, int iters,
                                                   float* __restrict__ out, long long* __restrict__ cyc) {
  constexpr int NT = 512;
  constexpr int STAGE = KB * 1024;
  constexpr int CH = STAGE / 16 / NT;  // 16-B DMA chunks per thread per K-tile
  static_assert(CH * 16 * NT == STAGE || KB == 0, "");
  constexpr int SM = STAGES * STAGE > 0 ? STAGES * STAGE : 16384;
  __shared__ __attribute__((aligned(1024))) char smem[SM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // each block walks its own window of the (L2-resident) source
  const long long win = (long long)blockIdx.x * 8192 * 16 % (src_bytes - (long long)STAGE - 16);
  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](int t, int stage) {
    if constexpr (KB > 0) {
      const long long base = (win + (long long)t * STAGE) % (src_bytes - STAGE);
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int q = i * NT + tid;
        __builtin_amdgcn_global_load_lds((const void*)(src + base + (long long)q * 16),
                                         (lds_void*)(smem + stage * STAGE + (i * NT + wave * 64) * 16), 16, 0, 0);
      }
    }
  };
  f32x16 acc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[a][i] = 0.f;
  bf16x8 fr[4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int i = 0; i < 8; ++i) fr[a][i] = (__bf16)(0.001f * (lane + i + a));
  const long long t0 = __builtin_amdgcn_s_memtime();
  constexpr int PER = CH;
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i) issue(i, i);
  for (int t = 0; t < iters; ++t) {
    wait_vmcnt<(STAGES - 2) * PER>();
    __builtin_amdgcn_s_barrier();
    issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    const char* sb = smem + (t % STAGES) * STAGE;
    // interleave: NRD reads spread over the NMF MFMAs
#pragma unroll
    for (int j = 0; j < (NMF > NRD ? NMF : NRD); ++j) {
      // fragments read two MFMAs ahead of their use (as the pipe kernel's
      // one-k-step-ahead prefetch)
      if (j < NRD) {
        const int off = ((j * 64 + lane) * 16) % (STAGE > 0 ? STAGE : 16384);
        fr[(j + 2) & 3] = *(const bf16x8*)(sb + off);
      }
      if (j < NMF) acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(j + 1) & 3], fr[j & 3], acc[j & 3], 0, 0, 0);
    }
  }
  wait_vmcnt<0>();
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[a][i];
  out[blockIdx.x * 512 + tid] = s;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KB, int STAGES, int NMF, int NRD>
static void run(const char* name, const char* src, long long bytes, float* out, long long* cyc) {
  const int iters = 256, blocks = 256;
  hipLaunchKernelGGL((feed_kernel<KB, STAGES, NMF, NRD>), dim3(blocks), dim3(512), 0, 0, src, bytes, iters, out, cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((feed_kernel<KB, STAGES, NMF, NRD>), dim3(blocks), dim3(512), 0, 0, src, bytes, iters, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(blocks);
  hipMemcpy(c.data(), cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
  long long med = c[blocks / 2];
  const double us = ms * 1e3 / reps;
  const double per_tile_us = us / iters;
  const double gbs = KB * 1024.0 / (per_tile_us * 1e-6) / 1e9;
  // MFMA pipe: 2 waves per SIMD x NMF x 32 cycles per K-tile; clock from the wall time of the cycles
  const double clk_ghz = med / (us * 1e3);
  const double mfma_cyc = 2.0 * NMF * 32.0;
  const double cyc_per_tile = (double)med / iters;
  std::printf("%-34s KB=%3d st=%d mfma/w=%3d rd/w=%3d  %8.2f us  %6.3f us/tile  %6.1f GB/s/CU  %7.0f cyc/tile  "
              "mfma-pipe %5.1f %%  clk %.2f GHz\n",
              name, KB, STAGES, NMF, NRD, us, per_tile_us, gbs, cyc_per_tile,
              mfma_cyc > 0 ? 100.0 * mfma_cyc / cyc_per_tile : 0.0, clk_ghz);
}

int main() {
  const long long bytes = 3ll << 20;  // 3 MB: L2-resident per XCD working set
  char* src;
  float* out;
  long long* cyc;
  hipMalloc(&src, bytes + (1 << 20));
  hipMemset(src, 1, bytes + (1 << 20));
  hipMalloc(&out, 256 * 512 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  // DMA alone: the L2 -> LDS feed per CU
  run<16, 2, 0, 0>("dma only", src, bytes, out, cyc);
  run<32, 2, 0, 0>("dma only", src, bytes, out, cyc);
  run<48, 2, 0, 0>("dma only", src, bytes, out, cyc);
  run<48, 3, 0, 0>("dma only", src, bytes, out, cyc);
  run<32, 4, 0, 0>("dma only", src, bytes, out, cyc);
  run<64, 2, 0, 0>("dma only", src, bytes, out, cyc);
  // MFMA alone, MFMA + reads (no DMA)
  run<0, 2, 16, 0>("mfma only (128x256 wave tile)", src, bytes, out, cyc);
  run<0, 2, 16, 16>("mfma + reads 1:1", src, bytes, out, cyc);
  run<0, 2, 32, 24>("mfma + reads 32:24", src, bytes, out, cyc);
  // the current 128x256 conv tile: 48 KB, 16 MFMA + 16 reads per wave
  run<48, 2, 16, 16>("pipe 128x256 s2", src, bytes, out, cyc);
  run<48, 3, 16, 16>("pipe 128x256 s3", src, bytes, out, cyc);
  // a 256x256 tile: 64 KB, 32 MFMA + 24 reads per wave
  run<64, 2, 32, 24>("256x256 s2", src, bytes, out, cyc);
  // 256x256 at BK 32: 32 KB per K-tile, 4 stages (128 KB)
  run<32, 4, 16, 12>("256x256 bk32 s4", src, bytes, out, cyc);
  run<32, 3, 16, 12>("256x256 bk32 s3", src, bytes, out, cyc);
  // halo-style 256x128: ~20 KB per K-tile, 16 MFMA + 16 reads
  run<16, 4, 16, 16>("halo-like 16KB s4", src, bytes, out, cyc);
  run<32, 3, 16, 16>("128x128x128? 32KB s3", src, bytes, out, cyc);
  hipFree(src);
  hipFree(out);
  hipFree(cyc);
  return 0;
}
