// Short-M row GEMM for the transformer's few-row problems (the encoder's
// baseline-token rows, M = 32 at batch 32): C (M x N) = A (M x K, rows
// k-contiguous) x B^T (B = N x K, k-contiguous), bf16 in, fp32 accumulate,
// the small kernel's epilogue (bias, residual, act, dropout, act' mask, RMW).
//
// Why a separate kernel: with 32 x 64 tiles an M = 32, N = 512 problem is 8
// blocks, each wave walking its K share behind one or two memory latencies;
// here a block owns a 32 x CT output tile (CT = 32 or 64: 16 .. 64 blocks for
// N = 512 .. 2048) and NW waves split K, so each wave issues ALL of its
// fragment loads (16 B per lane, straight from global memory) in one or two
// register rounds and the block waits out one latency. The NW partial tiles
// are summed through LDS in wave order (deterministic) and every thread runs
// the epilogue on its elements with all reads issued before the first store.
#pragma once
#include "gemm_impl.h"

namespace fpnmt {

template <int NW, int CT>
__global__ __launch_bounds__(64 * NW) void gemm_skinny_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int TN = CT / 32;
  constexpr int U = NW >= 16 ? 4 : 8;  // k-steps of 16 per register round
  static_assert(TN >= 1 && 32 * CT >= 64 * NW, "at least one output element per thread");
  __shared__ float red[NW][TN][16][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tiles_n = (p.N + CT - 1) / CT;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - (blockIdx.x / tiles_n) * tiles_n;
  const int m0 = tm * 32, n0 = tn * CT;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const T* __restrict__ Ag = (const T*)p.A + zo * p.a_so + zi * p.a_si;
  const T* __restrict__ Bg = (const T*)p.B + zo * p.b_so + zi * p.b_si;
  const int M = p.M, N = p.N, K = p.K;
  const int nks = (K + 15) / 16;
  const int per = (nks + NW - 1) / NW;
  const int ks0 = wave * per;
  const int ks1 = min(nks, ks0 + per);

  f32x16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  // rows >= M / columns >= N read row / column 0 (never stored); k beyond
  // the wave's range zeroes the A fragment after the load (no branch around
  // a load: all loads of a round stay in flight together)
  const int arow = m0 + lr;
  const T* ar = Ag + (long long)(arow < M ? arow : 0) * p.lda;
  const T* br[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int bcol = n0 + t * 32 + lr;
    br[t] = Bg + (long long)(bcol < N ? bcol : 0) * p.ldb;
  }
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  auto load_round = [&](int ks, bf16x8 (&av)[U], bf16x8 (&bv)[U][TN]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kq = (ks + u) * 16 + 8 * lh;
      const int kc = ((ks + u) < ks1 && kq < K) ? kq : 0;
      av[u] = *(const bf16x8*)(ar + kc);
#pragma unroll
      for (int t = 0; t < TN; ++t) bv[u][t] = *(const bf16x8*)(br[t] + kc);
    }
  };
  auto mma_round = [&](int ks, bf16x8 (&av)[U], bf16x8 (&bv)[U][TN]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kq = (ks + u) * 16 + 8 * lh;
      const unsigned keep = ((ks + u) < ks1 && kq < K) ? ~0u : 0u;
      const bf16x8 a = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, av[u]) & keep);
#pragma unroll
      for (int t = 0; t < TN; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv[u][t], acc[t], 0, 0, 0);
    }
  };
  bf16x8 aA[U], bA[U][TN], aB[U], bB[U][TN];
  int ks = ks0;
  if (ks < ks1) load_round(ks, aA, bA);
  while (ks < ks1) {
    if (ks + U < ks1) load_round(ks + U, aB, bB);
    mma_round(ks, aA, bA);
    ks += U;
    if (ks >= ks1) break;
    if (ks + U < ks1) load_round(ks + U, aA, bA);
    mma_round(ks, aB, bB);
    ks += U;
  }
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) red[wave][t][i][lane] = acc[t][i];
  __syncthreads();
  constexpr int NE = 32 * CT / (64 * NW);
  float ev[NE];
  int erow[NE], ecol[NE];
  bool eok[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int e = threadIdx.x + 64 * NW * j;
    const int t = e >> 10, i = (e >> 6) & 15, l = e & 63;
    ecol[j] = n0 + t * 32 + (l & 31);
    erow[j] = m0 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    eok[j] = ecol[j] < N && erow[j] < M;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w][t][i][l];
    ev[j] = s;
  }
  small_epilogue_n<T, NE>(p, ev, erow, ecol, eok, p.C, p.R, zo, zi);
}

}  // namespace fpnmt
