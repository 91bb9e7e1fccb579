// Weight-stationary streaming GEMM for the shallow 1x1 convs (stride 1, no
// padding) and row-major Dense layers with a small weight matrix: K <= 256,
// N <= 256 and N*K*2 <= 64 KB (ResNet res2 / res3 1x1 convs, the bwd-data of
// res2's 256->64 reduce, the FPN laterals of narrow inputs). Those GEMMs are
// HBM-bound (arithmetic intensity ~30-60 FLOP/B); the tiled kernels re-read
// the weights per block and, with one or two K-tiles, cannot overlap a
// block's load, MFMA and store phases.
//
// Structure: persistent blocks of 4 waves; the whole weight matrix (N x K,
// [row][64]-element images per 64-deep K slice, chunk slot XOR pipe_sw(row))
// is DMA'd into LDS once per block and stays there; each block then walks
// M-tiles of BM rows x all N columns: the tile's A rows come in by LDS-DMA
// (zero page past M), the residual rows (if any) into registers, MFMAs from
// LDS fragments, the direct epilogue (bias / residual / act / mask / dropout)
// stores from the accumulators. Several blocks per CU (48-64 KB of LDS each)
// overlap each other's load, MFMA and store phases.
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"

namespace fpnmt {

template <int BM, int N, int K, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void gemm_stream_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int NT = 64 * WM * WN;
  constexpr int NKT = K / 64;
  constexpr int A_IMG = BM * 128, B_IMG = N * 128;
  constexpr int A_BYTES = NKT * A_IMG, B_BYTES = NKT * B_IMG;
  constexpr int WTM = BM / WM, WTN = N / WN, TM = WTM / 32, TN = WTN / 32;
  static_assert(K % 64 == 0 && K <= 256 && TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "");
  static_assert((BM * 8) % NT == 0 && (N * 8) % 64 == 0, "whole waves of 16-B chunks");
  constexpr int NA = BM * 8 / NT;
  __shared__ __attribute__((aligned(1024))) char smem[A_BYTES + B_BYTES];
  char* As = smem;
  char* Bs = smem + A_BYTES;
  typedef __attribute__((address_space(3))) void lds_void;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int M = p.M;
  const T* __restrict__ Ag = (const T*)p.A;
  const T* __restrict__ Bg = (const T*)p.B;
  const T* zero = (const T*)p.zero16;

  // the weights, once: chunk q of image kt at byte q*16 (row q/8, slot q%8)
  for (int kt = 0; kt < NKT; ++kt)
    for (int q0 = wave * 64; q0 < N * 8; q0 += NT) {
      const int q = q0 + lane, row = q >> 3;
      const int kc = ((q & 7) ^ pipe_sw<64>(row)) * 8;
      __builtin_amdgcn_global_load_lds((const void*)(Bg + (long long)row * p.ldb + kt * 64 + kc),
                                       (lds_void*)(Bs + kt * B_IMG + q0 * 16), 16, 0, 0);
    }

  // this thread's A chunks: row, logical k chunk (fixed per tile row slot)
  int a_row[NA], a_kc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    a_row[i] = q >> 3;
    a_kc[i] = ((q & 7) ^ pipe_sw<64>(a_row[i])) * 8;
  }
  const T* Rg = p.R ? (const T*)p.R : nullptr;
  const int tiles = (M + BM - 1) / BM;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int m0 = t * BM;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int m = m0 + a_row[i];
        const T* src = m < M ? Ag + (long long)m * p.lda + kt * 64 + a_kc[i] : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(As + kt * A_IMG + (i * NT + wave * 64) * 16),
                                         16, 0, 0);
      }
    bf16x4 rv[TM][TN][4];
    if (Rg) prefetch_r_direct<TM, TN>(p, Rg, m0 + wm * WTM, wn * WTN, M, N, rv);
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's chunks landed (and, first tile, the weights)

    f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const char* Ak = As + kt * A_IMG;
      const char* Bk = Bs + kt * B_IMG;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int c = ks * 2 + lh;
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int row = wm * WTM + a * 32 + lr;
          fa[a] = *(const bf16x8*)(Ak + row * 128 + ((c ^ pipe_sw<64>(row)) << 4));
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int row = wn * WTN + b * 32 + lr;
          fb[b] = *(const bf16x8*)(Bk + row * 128 + ((c ^ pipe_sw<64>(row)) << 4));
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
      }
    }
    // every wave's fragment reads of this tile are done before any wave's
    // next-tile DMA overwrites the A images
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) (vmcnt, expcnt: no wait)
    __builtin_amdgcn_s_barrier();
    epilogue_direct<TM, TN>(p, acc, m0 + wm * WTM, wn * WTN, M, N, (char*)p.C, 0, Rg != nullptr, rv);
  }
}

}  // namespace fpnmt
