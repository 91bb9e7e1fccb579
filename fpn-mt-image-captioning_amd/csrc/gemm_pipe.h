// Pipelined bf16 MFMA GEMM for the large k-contiguous problems of the step:
// implicit-GEMM conv forward / stride-1 bwd-data (A = im2col of NHWC with
// C % 64 == 0, so every 64-deep K-tile lies inside one filter tap) and
// row-major Dense (A = rows, K % 64 == 0), both against B = (N, K) weights.
//
// Structure (cdna_hip_programming.md §5, "Pipelining across barriers"):
//   * 8 waves (512 threads), one block per CU, BM x BN tile, BK = 64 (the
//     64x64 / 4-wave form fills the chip on mid-size problems: 3 blocks/CU);
//   * operands move global -> LDS by LDS-DMA (global_load_lds_dwordx4), no
//     register staging; 3 LDS stages, two K-tiles in flight across each
//     barrier, retired with a counted `s_waitcnt vmcnt(N)` and a raw
//     s_barrier (a __syncthreads would drain the DMA queue);
//   * LDS images are [row][64] bf16 (128-B rows, lane-linear as the DMA
//     requires) with the 16-B chunk index XOR-swizzled by sw(row) =
//     (row >> 1) & 7 on the SOURCE address: two 128-B rows share a 256-B
//     bank line, and this swizzle gives each 16-lane ds_read_b128 group of
//     gfx950 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) 16 distinct 16-B
//     slots (row & 7 left 2-way conflicts: PMC bank-conflict/active 0.47);
//   * out-of-range rows / conv padding taps read a 16-B zero page;
//   * epilogue (bias, residual, act, dropout): EPI 1 = straight from the
//     accumulators (epilogue_direct below: the MFMA operands are swapped so
//     a lane holds four consecutive output columns of one row per register
//     group, stored as 8-B runs; no LDS, no barriers, so the LDS footprint is
//     the staging ring alone and more blocks fit a CU), EPI 0 = the shared
//     LDS-staged row epilogue (16-B stores).
#pragma once
#include <type_traits>
#include "gemm_impl.h"

namespace fpnmt {

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

// Direct epilogue for accumulators of the operand-swapped MFMA
// acc[a][b] = mfma_32x32x16(B-fragment b, A-fragment a): element i of lane l
// is output row row0 + a*32 + (l & 31), column col0 + b*32 + 8*(i >> 2) +
// 4*(l >> 5) + (i & 3), i.e. register group g = i >> 2 holds four consecutive
// columns. Needs N % 4 == 0, ldc % 4 == 0, ldr % 4 == 0 and 8-B aligned C / R
// (host-checked). The residual (or act-mask source) rows are loaded by
// prefetch_r_direct before the K loop: clamped addresses, no branches around
// the loads (a branch around a load makes hipcc wait vmcnt(0) per element).
template <int TM, int TN>
__device__ __forceinline__ void prefetch_r_direct(const GemmParams& p, const bf16* Rg, int row0, int col0, int M,
                                                  int N, bf16x4 (&rv)[TM][TN][4]) {
  const int lane = threadIdx.x & 63, lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const long long row = min(row0 + a * 32 + lr, M - 1);
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = min(col0 + b * 32 + 8 * g + 4 * lh, N - 4);
        rv[a][b][g] = *(const bf16x4*)(Rg + row * p.ldr + col);
      }
  }
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E). The
// epilogues index accumulator arrays with these, so a wave tile too large for
// the unroller's budget (64 x 128) still keeps its accumulators in registers
// (a runtime index sends the whole array to scratch)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// The epilogue operations on the four values of one (row, 4-column group):
// alpha * col_scale + bias, dropout, residual / act-mask operand, activation,
// the second mask operand M2 (see epilogue_direct).
struct EpiCols {
  float bi[4], cs[4];
};
__device__ __forceinline__ EpiCols epi_cols(const GemmParams& p, int col, bool bias_vec, bool scaled) {
  EpiCols e;
#pragma unroll
  for (int j = 0; j < 4; ++j) { e.bi[j] = 0.f; e.cs[j] = 1.f; }
  if (bias_vec) {
    const f32x4 t = *(const f32x4*)(p.bias + col);
    e.bi[0] = t[0]; e.bi[1] = t[1]; e.bi[2] = t[2]; e.bi[3] = t[3];
  } else if (p.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) e.bi[j] = p.bias[col + j];
  }
  if (scaled) {
#pragma unroll
    for (int j = 0; j < 4; ++j) e.cs[j] = (p.col_scale ? p.col_scale[col + j] : 1.f) * p.alpha;
  }
  return e;
}

// m2v: the M2 values of these four columns when the caller already holds
// them (tools/gemm_stream_lw.h stages M2 through LDS); null: read from p.M2
__device__ __forceinline__ void epi_values(const GemmParams& p, float (&v)[4], const EpiCols& e, int row, int col,
                                           int N, bool scaled, bool drop, unsigned long long key, float dsc,
                                           bool use_r, const bf16x4& rv, const bf16x4* m2v = nullptr) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = scaled ? v[j] * e.cs[j] + e.bi[j] : v[j] + e.bi[j];
  if (drop) {  // R + dropout(act(v)): residual after the mask
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a_ = act_apply(v[j], p.act, p.act_alpha);
      v[j] = uniform01(key, (uint64_t)row * (uint64_t)N + (uint64_t)(col + j)) >= p.drop_p ? a_ * dsc : 0.f;
    }
  }
  float r[4] = {0.f, 0.f, 0.f, 0.f};
  if (use_r) {
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = (float)rv[j];
    if (!p.r_mask) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += r[j];
    }
  }
  if (!drop) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = act_apply(v[j], p.act, p.act_alpha);
  }
  if (use_r && p.r_mask) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= act_mask_from_y(r[j], p.r_mask, p.act_alpha);
  }
  if (p.M2) {
    const bf16x4 y = m2v ? *m2v : *(const bf16x4*)((const bf16*)p.M2 + (long long)row * p.ldr + col);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= act_mask_from_y((float)y[j], p.m2_act);
  }
}

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int TM, int TN>
__device__ __forceinline__ void epilogue_direct(const GemmParams& p, f32x16 (&acc)[TM][TN], int row0, int col0, int M,
                                                int N, char* Cg, long long c_off, bool use_r,
                                                const bf16x4 (&rv)[TM][TN][4]) {
  const int lane = threadIdx.x & 63, lr = lane & 31, lh = lane >> 5;
  const bool bias_vec = p.bias && ((uintptr_t)p.bias & 15) == 0;
  const bool scaled = p.alpha != 1.f || p.col_scale;
  const bool drop = p.drop_p > 0.f;
  const unsigned long long key = drop ? drop_key(p) : 0ull;
  const float dsc = drop ? 1.f / (1.f - p.drop_p) : 1.f;
  // 16-B stores: lane l < 32 holds columns 8g..8g+3 of a row, lane l + 32
  // columns 8g+4..8g+7 of the same row; for a pair of groups (g, g+1) one
  // v_permlane32_swap per dword gives lanes 0-31 the 8 columns of group g and
  // lanes 32-63 those of group g+1 (cdna_hip_programming.md T21): half the
  // store instructions of the 8-B form (the store tail is issue-bound).
  const bool wide_ok = !p.c_f32 && p.accumulate != 1 && (((uintptr_t)Cg + 2 * c_off) & 15) == 0 && p.ldc % 8 == 0;
  static_for<0, TN>([&](auto bc) {
    constexpr int b = decltype(bc)::value;
    static_for<0, 2>([&](auto pc) {
      constexpr int g0 = 2 * decltype(pc)::value;
      const int colp = col0 + b * 32 + 8 * g0;  // first column of the group pair
      if (wide_ok && colp + 16 <= N) {          // wave-uniform
        const EpiCols e0 = epi_cols(p, colp + 4 * lh, bias_vec, scaled);
        const EpiCols e1 = epi_cols(p, colp + 8 + 4 * lh, bias_vec, scaled);
        static_for<0, TM>([&](auto ac) {
          constexpr int a = decltype(ac)::value;
          const int row = row0 + a * 32 + lr;
          float v0[4], v1[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v0[j] = acc[a][b][4 * g0 + j];
            v1[j] = acc[a][b][4 * g0 + 4 + j];
          }
          const int rowc = min(row, M - 1);  // every lane takes part in the swap
          epi_values(p, v0, e0, rowc, colp + 4 * lh, N, scaled, drop, key, dsc, use_r, rv[a][b][g0]);
          epi_values(p, v1, e1, rowc, colp + 8 + 4 * lh, N, scaled, drop, key, dsc, use_r, rv[a][b][g0 + 1]);
          const bf16x4 o0 = {(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]};
          const bf16x4 o1 = {(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
          u32x2 x = __builtin_bit_cast(u32x2, o0), y = __builtin_bit_cast(u32x2, o1);
          const auto s0 = __builtin_amdgcn_permlane32_swap(x[0], y[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(x[1], y[1], false, false);
          const u32x4 out = {s0[0], s1[0], s0[1], s1[1]};
          if (row < M) *(u32x4*)((bf16*)Cg + c_off + (long long)row * p.ldc + colp + 8 * lh) = out;
        });
        return;
      }
    static_for<g0, g0 + 2>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      const int col = col0 + b * 32 + 8 * g + 4 * lh;
      if (col >= N) return;
      const EpiCols e = epi_cols(p, col, bias_vec, scaled);
      static_for<0, TM>([&](auto ac) {
        constexpr int a = decltype(ac)::value;
        const int row = row0 + a * 32 + lr;
        if (row >= M) return;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[a][b][4 * g + j];
        epi_values(p, v, e, row, col, N, scaled, drop, key, dsc, use_r, rv[a][b][g]);
        const long long idx = c_off + (long long)row * p.ldc + col;
        if (p.c_f32) {
          f32x4* cp = (f32x4*)((float*)Cg + idx);
          f32x4 o = {v[0], v[1], v[2], v[3]};
          if (p.accumulate == 1) o += *cp;
          *cp = o;
        } else {
          bf16x4* cp = (bf16x4*)((bf16*)Cg + idx);
          bf16x4 o;
          if (p.accumulate == 1) {
            const bf16x4 old = *cp;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)(v[j] + (float)old[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
          }
          *cp = o;
        }
      });
    });
    });
  });
}

// Direct epilogue of the operand-swapped 16x16x32 MFMA acc[a][b] =
// mfma_16x16x32(B-fragment b, A-fragment a): lane l holds output row row0 +
// a*16 + (l & 15), columns col0 + b*16 + 4*(l >> 4) + j, j = 0..3 (four
// consecutive columns). Same epilogue operations and host preconditions as
// epilogue_direct. 16-B stores: for a pair of tiles (b, b+1) one
// v_permlane16_swap per dword (lanes 16-31 <-> 0-15 and 48-63 <-> 32-47 of the
// two registers) gives lane quarter q the 8 columns 8*(q >> 1) .. +7 of tile
// b + (q & 1).
template <int TM, int TN>
__device__ __forceinline__ void prefetch_r_direct16(const GemmParams& p, const bf16* Rg, int row0, int col0, int M,
                                                    int N, bf16x4 (&rv)[TM][TN]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const long long row = min(row0 + a * 16 + (lane & 15), M - 1);
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = min(col0 + b * 16 + 4 * (lane >> 4), N - 4);
      rv[a][b] = *(const bf16x4*)(Rg + row * p.ldr + col);
    }
  }
}

template <int TM, int TN>
__device__ __forceinline__ void epilogue_direct16(const GemmParams& p, f32x4 (&acc)[TM][TN], int row0, int col0, int M,
                                                  int N, char* Cg, long long c_off, bool use_r,
                                                  const bf16x4 (&rv)[TM][TN]) {
  const int lane = threadIdx.x & 63, q = lane >> 4;
  const bool bias_vec = p.bias && ((uintptr_t)p.bias & 15) == 0;
  const bool scaled = p.alpha != 1.f || p.col_scale;
  const bool drop = p.drop_p > 0.f;
  const unsigned long long key = drop ? drop_key(p) : 0ull;
  const float dsc = drop ? 1.f / (1.f - p.drop_p) : 1.f;
  const bool wide_ok = (TN % 2 == 0) && !p.c_f32 && p.accumulate != 1 &&
                       (((uintptr_t)Cg + 2 * c_off) & 15) == 0 && p.ldc % 8 == 0;
  static_for<0, (TN + 1) / 2>([&](auto pc) {
    constexpr int b0 = 2 * decltype(pc)::value;
    const int colp = col0 + b0 * 16;
    if constexpr (b0 + 1 < TN) {
      if (wide_ok && colp + 32 <= N) {  // wave-uniform
        const EpiCols e0 = epi_cols(p, colp + 4 * q, bias_vec, scaled);
        const EpiCols e1 = epi_cols(p, colp + 16 + 4 * q, bias_vec, scaled);
        static_for<0, TM>([&](auto ac) {
          constexpr int a = decltype(ac)::value;
          const int row = row0 + a * 16 + (lane & 15);
          const int rowc = min(row, M - 1);  // every lane takes part in the swap
          float v0[4], v1[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v0[j] = acc[a][b0][j];
            v1[j] = acc[a][b0 + 1][j];
          }
          epi_values(p, v0, e0, rowc, colp + 4 * q, N, scaled, drop, key, dsc, use_r, rv[a][b0]);
          epi_values(p, v1, e1, rowc, colp + 16 + 4 * q, N, scaled, drop, key, dsc, use_r, rv[a][b0 + 1]);
          const bf16x4 o0 = {(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]};
          const bf16x4 o1 = {(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
          u32x2 x = __builtin_bit_cast(u32x2, o0), y = __builtin_bit_cast(u32x2, o1);
          const auto s0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
          const u32x4 out = {s0[0], s1[0], s0[1], s1[1]};
          if (row < M)
            *(u32x4*)((bf16*)Cg + c_off + (long long)row * p.ldc + colp + 16 * (q & 1) + 8 * (q >> 1)) = out;
        });
        return;
      }
    }
    static_for<b0, (b0 + 2 < TN ? b0 + 2 : TN)>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      const int col = col0 + b * 16 + 4 * q;
      if (col >= N) return;
      const EpiCols e = epi_cols(p, col, bias_vec, scaled);
      static_for<0, TM>([&](auto ac) {
        constexpr int a = decltype(ac)::value;
        const int row = row0 + a * 16 + (lane & 15);
        if (row >= M) return;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[a][b][j];
        epi_values(p, v, e, row, col, N, scaled, drop, key, dsc, use_r, rv[a][b]);
        const long long idx = c_off + (long long)row * p.ldc + col;
        if (p.c_f32) {
          f32x4* cp = (f32x4*)((float*)Cg + idx);
          f32x4 o = {v[0], v[1], v[2], v[3]};
          if (p.accumulate == 1) o += *cp;
          *cp = o;
        } else {
          bf16x4* cp = (bf16x4*)((bf16*)Cg + idx);
          bf16x4 o;
          if (p.accumulate == 1) {
            const bf16x4 old = *cp;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)(v[j] + (float)old[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
          }
          *cp = o;
        }
      });
    });
  });
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  // gfx9 s_waitcnt encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14], expcnt[6:4]=7, lgkmcnt[11:8]=15
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// R image swizzle of EPI 2: 16-B chunk slot = chunk ^ pipe_rswz(row), so the
// epilogue's ds_read_b64 of 32 rows at one column spreads over the banks
template <int BN>
__device__ __forceinline__ int pipe_rswz(int row) {
  if constexpr (BN == 64) return (row >> 1) & 7;
  else return row & 15;
}

// LDS image geometry of one K-tile: [row][BK] bf16, 16-B chunk slots XOR
// pipe_sw(row) (conflict-free ds_read_b128 fragment reads for BK = 64 / 32:
// 128-B rows pair up on a 256-B bank line, 64-B rows four to a line)
template <int BK>
__device__ __forceinline__ int pipe_sw(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  else return (row >> 2) & 3;
}

// SPREAD = 1: the next K-tile's DMA instructions are issued in pieces between
// the k-steps of the current tile's MFMAs (after each k-step's fragment reads)
// instead of all at once after the barrier, so their issue cost overlaps the
// partner wave's MFMAs (MI355X_MICROARCH.md: 60-185 cycles per LDS-DMA
// wave-instruction); SPREAD = 2 also raises the wave's priority around its MFMAs;
// SPREAD = 3: the priority alone (the DMA issued after the barrier as with 0).
// MF = 16: v_mfma_f32_16x16x32_bf16 instead of 32x32x16 (same LDS image and
// bytes per MFMA cycle for a given wave tile; the loop holds a higher clock
// under load, MI355X_MICROARCH.md 'DVFS give-back' item 7), direct epilogue only.
template <int BM, int BN, int WM, int WN, int AM, int NT = 512, int STAGES = 3, int EPI = 1, int BK = 64,
          int SPREAD = 0, int MF = 32>
__global__ __launch_bounds__(NT) void gemm_pipe_kernel(const GemmParams p) {
  typedef bf16 T;
  static_assert(BK == 64 || BK == 32, "K-tile depth");
  constexpr int CPR = BK / 8, ROWB = BK * 2;  // 16-B chunks / bytes per LDS row
  static_assert(STAGES >= 1 && STAGES <= 8, "stages");
  static_assert(WM * WN * 64 == NT, "one wave per 64 threads");
  static_assert(AM == A_ROW || AM == A_IM2COL, "k-contiguous A only");
  static_assert(MF == 32 || (MF == 16 && EPI == 1), "16x16x32: direct epilogue only");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / MF, TN = WTN / MF;
  static_assert(TM >= 1 && TN >= 1, "");
  typedef typename std::conditional<MF == 32, f32x16, f32x4>::type accT;
  constexpr int NACC = MF == 32 ? 16 : 4, KS = MF == 32 ? 16 : 32;  // accumulators per lane, k per MFMA
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * CPR / NT, NB = BN * CPR / NT;  // 16-B DMA chunks per thread per stage
  static_assert((BM * CPR) % NT == 0 && (BN * CPR) % NT == 0 && NA >= 1 && NB >= 1, "");
  constexpr int EPI_BYTES = EPI ? 0 : (NT / 64) * 32 * (WTN + 4) * 4;
  // EPI 2: the residual / act-mask tile (BM x BN bf16) DMA'd into LDS behind
  // the staging ring at the kernel's start, read back by the direct epilogue
  constexpr int R_BYTES = EPI == 2 ? BM * BN * 2 : 0;
  constexpr int NR = R_BYTES / 16 / NT;
  static_assert(EPI != 2 || (BM * BN / 8) % NT == 0, "");
  constexpr int SMEM = (STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES) + R_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  const int ntile = p.tiles_m * p.tiles_n;
  const int bid = xcd_remap(blockIdx.x, ntile);
  int tmi = bid / p.tiles_n;
  const int tni = bid - tmi * p.tiles_n;
  const void* Ap = p.A;
  void* Cp0 = p.C;
  const void* Rp = p.R;
  int M = p.M;
  int gH = p.H, gW = p.W, gHo = p.Ho, gWo = p.Wo;
  FastDiv gfdHoWo = p.fd_HoWo, gfdWo = p.fd_Wo;
  if (p.ngroups > 0) {  // m-grouped launch (shared B)
    // static indices only (a dynamic index into the kernarg struct makes
    // the compiler copy the whole struct to scratch)
    GemmGroup G = p.groups[0];
#pragma unroll
    for (int q = 1; q < MAX_GROUPS; ++q)
      if (q < p.ngroups && tmi >= p.groups[q].start) G = p.groups[q];
    tmi -= G.start;
    Ap = G.A; Cp0 = G.C; Rp = G.R;
    M = G.M;
    gH = G.H; gW = G.W; gHo = G.Ho; gWo = G.Wo;
    gfdHoWo = G.fd_HoWo; gfdWo = G.fd_Wo;
  }
  const int N = p.N, K = p.K;
  const int m0 = tmi * BM, n0 = tni * BN;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const T* __restrict__ Ag = (const T*)Ap + zo * p.a_so + zi * p.a_si;
  const T* __restrict__ Bg = (const T*)p.B + zo * p.b_so + zi * p.b_si;
  const T* zero = (const T*)p.zero16;
  // split-K over blockIdx.y (partial slabs, see dispatch: C = the fp32 slab
  // base, split y writes y * c_split elements further)
  const int kt0 = (int)blockIdx.y * (p.k_per_split / BK);
  const int nk = max(0, min(K / BK - kt0, p.k_per_split / BK));

  // ---- per-thread DMA sources (rows fixed across K-tiles) ---------------
  // chunk q = i*NT + tid lands at LDS byte q*16: row q / CPR, slot q % CPR,
  // holding logical k-chunk (slot ^ pipe_sw(row)). Offsets are 32-bit element offsets
  // (host-checked); im2col rows keep the offset of their (hi0, wi0) pixel and
  // a bit per filter tap (r*S + s) that is inside the image, so a K-tile's
  // source is one add and one select per chunk (no branches in the loop).
  int a_off[NA];
  unsigned long long a_vm[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    const int row = q / CPR;
    const int kc = ((q % CPR) ^ pipe_sw<BK>(row)) * 8;
    const int m = m0 + row;
    if constexpr (AM == A_ROW) {
      a_off[i] = m * p.lda + kc;
      a_vm[i] = m < M ? 1ull : 0ull;
    } else {
      const uint32_t nimg = fdiv((uint32_t)min(m, M - 1), gfdHoWo);
      const int rem = min(m, M - 1) - (int)nimg * gHo * gWo;
      const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
      const int wo = rem - (int)ho * gWo;
      const int hi0 = (int)ho * p.sh - p.pt, wi0 = wo * p.sw - p.pl;
      a_off[i] = (((int)nimg * gH + hi0) * gW + wi0) * p.Cc + kc;
      unsigned long long vm = 0;
      if (m < M)
        for (int r = 0; r < p.Rk; ++r)
          for (int s2 = 0; s2 < p.Sk; ++s2)
            if (hi0 + r >= 0 && hi0 + r < gH && wi0 + s2 >= 0 && wi0 + s2 < gW) vm |= 1ull << (r * p.Sk + s2);
      a_vm[i] = vm;
    }
  }
  int b_off[NB];
  bool b_ok[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    const int row = q / CPR;
    const int kc = ((q % CPR) ^ pipe_sw<BK>(row)) * 8;
    b_ok[i] = n0 + row < N;
    b_off[i] = (n0 + row) * p.ldb + kc;
  }

  typedef __attribute__((address_space(3))) void lds_void;
  struct TileSrc { int k0, tap, tap_off; };
  auto tile_src = [&](int kt) {
    TileSrc ts;
    ts.k0 = (kt0 + kt) * BK;
    ts.tap = 0;
    ts.tap_off = ts.k0;
    if constexpr (AM == A_IM2COL) {
      // the whole K-tile sits in one filter tap (Cc % BK == 0)
      const uint32_t rs = fdiv((uint32_t)ts.k0, p.fd_C);
      const int cb = ts.k0 - (int)rs * p.Cc;
      const uint32_t r = fdiv(rs, p.fd_S);
      const int s2 = (int)rs - (int)r * p.Sk;
      ts.tap = (int)rs;
      ts.tap_off = ((int)r * gW + s2) * p.Cc + cb;
    }
    return ts;
  };
  // DMA instruction j of a stage: j < NA the A chunks, then the B chunks
  auto issue_range = [&](const TileSrc& ts, int stage, auto lo_c, auto hi_c) {
    constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
    char* sb = smem + stage * STAGE_BYTES;
    static_for<LO, HI>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j < NA) {
        const T* src = ((a_vm[j] >> ts.tap) & 1ull) ? Ag + (a_off[j] + ts.tap_off) : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (j * NT + wave * 64) * 16), 16, 0, 0);
      } else {
        constexpr int i = j - NA;
        const T* src = b_ok[i] ? Bg + (b_off[i] + ts.k0) : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + A_BYTES + (i * NT + wave * 64) * 16),
                                         16, 0, 0);
      }
    });
  };
  auto issue = [&](int kt, int stage) {
    issue_range(tile_src(kt), stage, std::integral_constant<int, 0>{}, std::integral_constant<int, NA + NB>{});
  };

  accT acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[a][b][i] = 0.f;

  // fragments of k-step ks+1 are read while the MFMAs of ks run (two
  // register sets, static indices after unrolling). 32x32x16: lane l reads
  // row l & 31, 8-element chunk 2 ks + (l >> 5); 16x16x32: row l & 15, chunk
  // 4 ks + (l >> 4)
  const int frow = MF == 32 ? lr : (lane & 15);
  const int fchunk = MF == 32 ? lh : (lane >> 4);
  auto frag = [&](const char* As, const char* Bs, int ks, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
    const int c = ks * (KS / 8) + fchunk;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int row = wm * WTM + t * MF + frow;
      af[t] = *(const bf16x8*)(As + row * ROWB + ((c ^ pipe_sw<BK>(row)) << 4));
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int row = wn * WTN + t * MF + frow;
      bfr[t] = *(const bf16x8*)(Bs + row * ROWB + ((c ^ pipe_sw<BK>(row)) << 4));
    }
  };
  // mid(ks) runs after k-step ks's next fragment reads are issued, before its
  // MFMAs (SPREAD: a piece of the next K-tile's DMA)
  auto compute_mid = [&](int stage, auto&& mid) {
    const char* As = smem + stage * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
    bf16x8 fa[2][TM], fb[2][TN];
    frag(As, Bs, 0, fa[0], fb[0]);
    static_for<0, BK / KS>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      if constexpr (ks + 1 < BK / KS) frag(As, Bs, ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
      mid(ksc);
      if constexpr (SPREAD >= 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          if constexpr (MF == 16)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks & 1][b], fa[ks & 1][a], acc[a][b], 0, 0, 0);
          else if constexpr (EPI != 0)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[ks & 1][b], fa[ks & 1][a], acc[a][b], 0, 0, 0);
          else
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks & 1][a], fb[ks & 1][b], acc[a][b], 0, 0, 0);
        }
      if constexpr (SPREAD >= 2) __builtin_amdgcn_s_setprio(0);
    });
  };
  auto compute = [&](int stage) { compute_mid(stage, [](auto) {}); };

  // residual rows for the direct epilogue, in flight under the K loop
  typedef typename std::conditional<MF == 32, bf16x4[TM][TN][4], bf16x4[TM][TN]>::type rpreT;
  rpreT rpre;
  const T* Rg0 = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  char* Rs = smem + (SMEM - R_BYTES);
  if constexpr (EPI == 1) {
    if (Rg0) {
      if constexpr (MF == 32) prefetch_r_direct<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);
      else prefetch_r_direct16<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);
    }
  } else if constexpr (EPI == 2) {
    // whole 16-B chunks of R rows into a [BM][BN] image, chunk slot XOR
    // pipe_rswz(row) on the source side (lane-linear DMA destination)
    if (Rg0) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int q = i * NT + tid;
        const int row = q / (BN / 8);
        const int col = ((q % (BN / 8)) ^ pipe_rswz<BN>(row)) * 8;
        const bool ok = m0 + row < M && n0 + col < N;
        const T* src = ok ? Rg0 + (long long)(m0 + row) * p.ldr + n0 + col : zero;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(Rs + (i * NT + wave * 64) * 16),
                                         16, 0, 0);
      }
    }
  }

  // ---- main loop: STAGES - 1 K-tiles in flight across each barrier ------
  constexpr int PER_STAGE = NA + NB;  // DMA instructions per thread per stage
  static_assert(STAGES < 2 || (STAGES - 2) * PER_STAGE < 64, "vmcnt holds at most 63 loads in flight");
  if constexpr (STAGES == 1) {
    // short reductions (the 1x1 convs with K = 64: one K-tile): one stage,
    // a small LDS footprint, several blocks per CU overlap each other's
    // load / MFMA / epilogue phases
    for (int t = 0; t < nk; ++t) {
      if (t > 0) __builtin_amdgcn_s_barrier();  // everyone's fragment reads of tile t-1 done
      issue(t, 0);
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      compute(0);
    }
  } else {
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < nk) issue(i, i);
  for (int t = 0; t < nk; ++t) {
    // tile t landed (this thread's part): the tiles issued after it may stay in flight
    const int ahead = min(nk - 1 - t, STAGES - 2);
    if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
    else if (STAGES > 4 && ahead == 3) wait_vmcnt<(STAGES > 4 ? 3 : 0) * PER_STAGE>();
    else if (STAGES > 3 && ahead == 2) wait_vmcnt<(STAGES > 3 ? 2 : 0) * PER_STAGE>();
    else if (ahead == 1) wait_vmcnt<PER_STAGE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // ... everyone's part; stage (t-1) % STAGES is free
    if constexpr (SPREAD == 1 || SPREAD == 2) {
      // the pieces of tile t + STAGES - 1 between the k-steps (a tile with
      // nothing to issue takes the same path: uniform per block)
      const bool more = t + STAGES - 1 < nk;
      const TileSrc ts = tile_src(t + STAGES - 1);
      const int st = (t + STAGES - 1) % STAGES;
      compute_mid(t % STAGES, [&](auto ksc) {
        constexpr int ks = decltype(ksc)::value, NKS = BK / KS, PS = NA + NB;
        if (more)
          issue_range(ts, st, std::integral_constant<int, ks * PS / NKS>{},
                      std::integral_constant<int, (ks + 1) * PS / NKS>{});
      });
    } else {
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      compute(t % STAGES);
    }
  }
  }
  if constexpr (EPI != 1) __syncthreads();  // all DMA retired (vmcnt 0 above) and all fragment reads done: reuse LDS
  if constexpr (EPI == 2) {
    if (Rg0) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int rl = wm * WTM + a * 32 + lr;
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int ch = (wn * WTN + b * 32) / 8 + g;
            rpre[a][b][g] = *(const bf16x4*)(Rs + rl * (BN * 2) + ((ch ^ pipe_rswz<BN>(rl)) << 4) + lh * 8);
          }
      }
    }
  }

  char* Cg = (char*)Cp0;
  const long long c_off = zo * p.c_so + zi * p.c_si + (long long)blockIdx.y * p.c_split;
  if constexpr (MF == 16) {
    epilogue_direct16<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg0 != nullptr, rpre);
  } else if constexpr (EPI) {
    epilogue_direct<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg0 != nullptr, rpre);
  } else {
    epilogue_rows<T, TM, TN, WTN>(p, acc, (float*)smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off,
                                  Rg0, true);
  }
}

// ---------------------------------------------------------------------------
// Loader-wave form of gemm_pipe_kernel (round 6; tools/gemm_lw.h and
// tools/fwd_bench.hip -DFB_LW measured it): WM x WN MFMA waves that only read
// LDS fragments and issue v_mfma_f32_16x16x32_bf16, plus NLW loader waves that
// own every LDS-DMA of the STAGES-deep K-tile ring and its im2col address
// arithmetic — in the 8-wave kernel each K-tile's DMA issue (60-185 cycles per
// wave-instruction, MI355X_MICROARCH.md) sat in the MFMA waves' own streams.
// One raw s_barrier per K-tile over all waves: loaders wait (counted vmcnt)
// for K-tile t, barrier, then issue K-tile t + STAGES - 1 into the slot of
// t - 1; consumers pass the barrier and read / multiply K-tile t (each of
// their fragment reads feeds an MFMA of the same tile, so all have returned
// before the next barrier). The consumers issue no DMA, so their residual
// rows are plain loads into registers before the loop (no ring drain).
// Same LDS image, K order and epilogue (epilogue_direct16) as the MF = 16
// pipe kernel: the results are bitwise those of gemm_pipe_kernel<..., MF 16>.
// Grouped launches, batch (grid.z) and split-K (grid.y) as gemm_pipe_kernel.
// MS < BM (the M step): a tile covers MS output rows while the LDS image and
// the loader lanes keep BM rows (rows MS .. BM-1 DMA the zero chunk and are
// never read), so the tile count over M is cdiv(M, MS) — e.g. MS = 112 puts
// the C2 P3 conv (M = 25088) on 224 tiles instead of 196 of a 256-CU chip.
template <int BM, int BN, int WM, int WN, int AM, int NLW, int STAGES, int MS = BM>
__global__ __launch_bounds__(64 * (WM * WN + NLW)) void gemm_pipe_lw_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int BK = 64, CPR = 8, ROWB = 128, MF = 16, KS = 32;
  constexpr int NC = 64 * WM * WN, NL = 64 * NLW;
  constexpr int WTM = MS / WM, WTN = BN / WN, TM = WTM / MF, TN = WTN / MF;
  static_assert(TM >= 1 && TN >= 1 && TM * MF * WM == MS && TN * MF * WN == BN && MS <= BM,
                "whole 16x16 MFMA tiles per wave");
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * CPR / NL, NB = BN * CPR / NL;  // DMA chunks per loader lane per stage
  static_assert(NA * NL == BM * CPR && NB * NL == BN * CPR && NA >= 1, "loader lanes divide the tile's chunks");
  static_assert(AM == A_ROW || AM == A_IM2COL, "k-contiguous A only");
  constexpr int PER = NA + NB;
  static_assert(STAGES >= 2 && STAGES <= 5 && (STAGES - 2) * PER < 64, "vmcnt range");
  static_assert(STAGES * STAGE_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int ntile = p.tiles_m * p.tiles_n;
  const int bid = xcd_remap(blockIdx.x, ntile);
  int tmi = bid / p.tiles_n;
  const int tni = bid - tmi * p.tiles_n;
  const void* Ap = p.A;
  void* Cp0 = p.C;
  const void* Rp = p.R;
  int M = p.M;
  int gH = p.H, gW = p.W, gHo = p.Ho, gWo = p.Wo;
  FastDiv gfdHoWo = p.fd_HoWo, gfdWo = p.fd_Wo;
  if (p.ngroups > 0) {  // m-grouped launch (shared B); static indices only (see gemm_pipe_kernel)
    GemmGroup G = p.groups[0];
#pragma unroll
    for (int q = 1; q < MAX_GROUPS; ++q)
      if (q < p.ngroups && tmi >= p.groups[q].start) G = p.groups[q];
    tmi -= G.start;
    Ap = G.A; Cp0 = G.C; Rp = G.R;
    M = G.M;
    gH = G.H; gW = G.W; gHo = G.Ho; gWo = G.Wo;
    gfdHoWo = G.fd_HoWo; gfdWo = G.fd_Wo;
  }
  const int N = p.N, K = p.K;
  const int m0 = tmi * MS, n0 = tni * BN;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const int kt0 = (int)blockIdx.y * (p.k_per_split / BK);
  const int nk = max(0, min(K / BK - kt0, p.k_per_split / BK));
  typedef __attribute__((address_space(3))) void lds_void;

  if (wave >= WM * WN) {  // ---- loader waves -------------------------------
    const T* __restrict__ Ag = (const T*)Ap + zo * p.a_so + zi * p.a_si;
    const T* __restrict__ Bg = (const T*)p.B + zo * p.b_so + zi * p.b_si;
    const T* zero = (const T*)p.zero16;
    const int lt = tid - NC, lw = wave - WM * WN;
    int a_off[NA];
    unsigned long long a_vm[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = i * NL + lt;
      const int row = q / CPR;
      const int kc = ((q % CPR) ^ pipe_sw<BK>(row)) * 8;
      const int m = m0 + row;
      const bool live = row < MS && m < M;  // rows MS .. BM-1 of the image: the zero chunk
      if constexpr (AM == A_ROW) {
        a_off[i] = m * p.lda + kc;
        a_vm[i] = live ? 1ull : 0ull;
      } else {
        const uint32_t nimg = fdiv((uint32_t)min(m, M - 1), gfdHoWo);
        const int rem = min(m, M - 1) - (int)nimg * gHo * gWo;
        const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
        const int wo = rem - (int)ho * gWo;
        const int hi0 = (int)ho * p.sh - p.pt, wi0 = wo * p.sw - p.pl;
        a_off[i] = (((int)nimg * gH + hi0) * gW + wi0) * p.Cc + kc;
        unsigned long long vm = 0;
        if (live)
          for (int r = 0; r < p.Rk; ++r)
            for (int s2 = 0; s2 < p.Sk; ++s2)
              if (hi0 + r >= 0 && hi0 + r < gH && wi0 + s2 >= 0 && wi0 + s2 < gW) vm |= 1ull << (r * p.Sk + s2);
        a_vm[i] = vm;
      }
    }
    int b_off[NB];
    bool b_ok[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = i * NL + lt;
      const int row = q / CPR;
      const int kc = ((q % CPR) ^ pipe_sw<BK>(row)) * 8;
      b_ok[i] = n0 + row < N;
      b_off[i] = (n0 + row) * p.ldb + kc;
    }
    auto issue = [&](int kt, int stage) {
      const int k0 = (kt0 + kt) * BK;
      int tap = 0, tap_off = k0;
      if constexpr (AM == A_IM2COL) {  // the whole K-tile sits in one filter tap (Cc % 64 == 0)
        const uint32_t rs = fdiv((uint32_t)k0, p.fd_C);
        const int cb = k0 - (int)rs * p.Cc;
        const uint32_t r = fdiv(rs, p.fd_S);
        const int s2 = (int)rs - (int)r * p.Sk;
        tap = (int)rs;
        tap_off = ((int)r * gW + s2) * p.Cc + cb;
      }
      char* sb = smem + stage * STAGE_BYTES;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const T* src = ((a_vm[j] >> tap) & 1ull) ? Ag + (a_off[j] + tap_off) : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (j * NL + lw * 64) * 16), 16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const T* src = b_ok[j] ? Bg + (b_off[j] + k0) : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + A_BYTES + (j * NL + lw * 64) * 16), 16,
                                         0, 0);
      }
    };
#pragma unroll
    for (int i = 0; i < STAGES - 1; ++i)
      if (i < nk) issue(i, i);
    for (int t = 0; t < nk; ++t) {
      const int ahead = min(nk - 1 - t, STAGES - 2);
      if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER>();
      else if (STAGES > 3 && ahead == 2) wait_vmcnt<(STAGES > 3 ? 2 : 0) * PER>();
      else if (ahead == 1) wait_vmcnt<PER>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // K-tile t visible to every consumer; slot (t - 1) % STAGES free
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    }
    return;  // the consumers' epilogue has no barrier
  }

  // ---- MFMA waves ------------------------------------------------------
  const int wm = wave / WN, wn = wave % WN;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x4 rpre[TM][TN];
  const T* Rg0 = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  if (Rg0) prefetch_r_direct16<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);
  const int frow = lane & 15, fchunk = lane >> 4;
  auto frag = [&](const char* As, const char* Bs, int ks, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
    const int c = ks * (KS / 8) + fchunk;
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const int row = wm * WTM + t * MF + frow;
      af[t] = *(const bf16x8*)(As + row * ROWB + ((c ^ pipe_sw<BK>(row)) << 4));
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int row = wn * WTN + t * MF + frow;
      bfr[t] = *(const bf16x8*)(Bs + row * ROWB + ((c ^ pipe_sw<BK>(row)) << 4));
    }
  };
  for (int t = 0; t < nk; ++t) {
    __builtin_amdgcn_s_barrier();
    const char* As = smem + (t % STAGES) * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
    bf16x8 fa[2][TM], fb[2][TN];
    frag(As, Bs, 0, fa[0], fb[0]);
    static_for<0, BK / KS>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      if constexpr (ks + 1 < BK / KS) frag(As, Bs, ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks & 1][b], fa[ks & 1][a], acc[a][b], 0, 0, 0);
    });
  }
  const long long c_off = zo * p.c_so + zi * p.c_si + (long long)blockIdx.y * p.c_split;
  epilogue_direct16<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, (char*)Cp0, c_off, Rg0 != nullptr, rpre);
}


// ---------------------------------------------------------------------------
// Weight-gradient form: C[m][n] += sum_k A[k][m] * B[k][n] with both operands
// m/n-contiguous per reduction row k: A = im2col(x)^T (A_IM2COL_T; each 8-row
// chunk of the m range lies in one filter tap, Cc % 8 == 0) or x rows (A_COL),
// B = dz rows (B_KN). Operands move global -> LDS by LDS-DMA into [k][BM] /
// [k][BN] images (128- or 256-B rows, lane-linear as the DMA requires) whose 16-B
// chunk index is XOR-swizzled by (k & 3) << 2 on the SOURCE address; the MFMA
// fragments are read with ds_read_b64_tr_b16 (transposing read), for which
// that swizzle makes every 32-lane half touch 64 distinct banks. Same 3-stage
// / two-tiles-in-flight schedule as gemm_pipe_kernel; split-K over blockIdx.y
// (k-grouped launches as gemm_kernel), fp32 atomics into C.
// SPREAD as gemm_pipe_kernel: the next K-tile's DMA (and its im2col^T address
// arithmetic) issued in pieces between the k-steps' MFMAs; 2 = also MFMA priority.
// The LDS image swizzle of the weight-gradient kernel: 16-B chunk slot =
// chunk ^ wg_sw(k). (k & 3) << 2 spreads the four k-rows of one transposed
// read over the banks; the k-bit-3 term separates the two 16-lane groups of a
// 32-lane half that read rows k and k + 8 of the same columns (the 16x16x32
// operand, MF 16; the 32x32x16 halves differ in columns and keep it uniform).
__device__ __forceinline__ int wg_sw(int k) { return ((k & 3) << 2) ^ (((k >> 3) & 1) << 1); }
// 64-wide images (8 chunks = 128 B per k-row, MF 32 only): rows k and k + 1
// already sit in opposite bank halves; rows k and k + 2 are separated by
// flipping chunk bit 2 on (k & 2), so the four rows of a transposed read
// cover the 64 banks once.
template <int CH>
__device__ __forceinline__ int wg_swz(int k) {
  if constexpr (CH >= 16) return wg_sw(k);
  else return ((k >> 1) & 1) << 2;
}

// MF = 16: v_mfma_f32_16x16x32_bf16 with the operands swapped (lane: four
// consecutive columns n of one row m -> 16-B slab stores), 2 k-steps per
// K-tile; MF = 32: 32x32x16 as before.
// NLW > 0 (round 6, the loader-wave form; tools/wg_bench.hip -DWB_LW,
// profiles/r06/wg_lw.txt): NLW extra waves own the ring's LDS-DMA (and the
// im2col^T address arithmetic), the WM x WN MFMA waves only do the transposing
// fragment reads and MFMAs, one barrier per K-tile over all of them (see
// gemm_pipe_lw_kernel). Same images, K order and epilogue: bitwise the NLW 0
// kernel's results.
// the weight-gradient kernel's ring depth for a stage of `stage_bytes` (LDS
// 160 KB), and whether the folded bias column sums (one float per MFMA thread
// and 32-column tile, MF 32) fit beside that same ring
constexpr int wg_stages(int stage_bytes) {
  return 4 * stage_bytes <= 160 * 1024 ? 4 : 3 * stage_bytes <= 160 * 1024 ? 3 : 2;
}
template <int BM, int BN, int WM, int WN, int MF>
constexpr bool wg_cs_ok() {
  return MF == 32 && wg_stages(64 * (BM + BN) * 2) * 64 * (BM + BN) * 2 + 64 * WM * WN * (BN / WN / 32) * 4 <= 160 * 1024;
}

template <int BM, int BN, int WM, int WN, int AM, int SPREAD = 0, int MF = 32, int NLW = 0>
__global__ __launch_bounds__(64 * (WM * WN + NLW)) void gemm_pipe_wg_kernel(const GemmParams p) {
  typedef bf16 T;
  static_assert(NLW == 0 || SPREAD == 0, "the loader waves issue the whole tile");
  constexpr int NC = 64 * WM * WN;             // MFMA threads
  constexpr int NT = NLW ? 64 * NLW : NC;      // DMA-issuing threads
  constexpr int BK = 64;
  static_assert(AM == A_IM2COL_T || AM == A_COL, "m-contiguous A only");
  static_assert(MF == 32 || MF == 16, "");
  static_assert(BM % 64 == 0 && BN % 64 == 0, ">= 8 chunks per LDS row (wg_swz)");
  static_assert(MF == 32 || (BM % 128 == 0 && BN % 128 == 0), "MF 16 reads need 16-chunk rows (wg_sw's k-bit-3 term)");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / MF, TN = WTN / MF;
  typedef typename std::conditional<MF == 32, f32x16, f32x4>::type accT;
  constexpr int NACC = MF == 32 ? 16 : 4, KS = MF == 32 ? 16 : 32;
  constexpr int ROWA = BM * 2, ROWBB = BN * 2;       // bytes per k-row of the A / B images
  constexpr int A_BYTES = BK * ROWA, B_BYTES = BK * ROWBB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int CA = BM / 8, CB = BN / 8;            // 16-B chunks per row
  constexpr int NA = BK * (BM / 8) / NT, NB = BK * (BN / 8) / NT;  // DMA chunks per thread per stage
  static_assert(NA * NT == BK * (BM / 8) && NB * NT == BK * (BN / 8), "");
  // 256x256 (64 KB per stage): a 2-stage ring
  constexpr int STAGES = wg_stages(STAGE_BYTES);
  // the folded bias column sums (p.cs_part) per MFMA thread in LDS behind the
  // ring (registers are at the limit in the 16-wave form), where they fit
  // beside the same ring (wg_cs_ok; the host folds only there)
  constexpr int CS_BYTES = wg_cs_ok<BM, BN, WM, WN, MF>() ? NC * TN * 4 : 0;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES + CS_BYTES];

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const bool loader = NLW == 0 || wave >= WM * WN;  // issues DMA
  const int tid = NLW == 0 ? (int)threadIdx.x : (loader ? (int)threadIdx.x - NC : 0);  // DMA chunk owner index
  const int dwave = NLW == 0 ? wave : (loader ? wave - WM * WN : 0);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  // 1-D grid over (split, tile), XCD-aware: each XCD gets a contiguous run of
  // work items, i.e. all tiles of (about) one split, so the split's slices of
  // x and dz are fetched into that XCD's L2 once and re-read from there
  const int ntile = p.tiles_m * p.tiles_n;
  const int w = xcd_remap(blockIdx.x, ntile * p.split_k);
  const int split = w / ntile;
  const int bid = w - split * ntile;
  const int tmi = bid / p.tiles_n;
  const int tni = bid - tmi * p.tiles_n;
  // k-grouped launches (the FPN levels of one shared conv): the groups' K
  // ranges are laid end to end in whole K-tiles (groups[g].start = first
  // K-tile of group g), and the splits cut that sequence evenly, so a split
  // may run over several groups; every K-tile belongs to exactly one group.
  const int M = p.M, N = p.N;
  const int m0 = tmi * BM, n0 = tni * BN;
  const T* zero = (const T*)p.zero16;
  int tot_kt;
  if (p.ngroups > 0) {
    tot_kt = 0;
#pragma unroll
    for (int q = 0; q < MAX_GROUPS; ++q)
      if (q < p.ngroups) tot_kt = p.groups[q].start + (p.groups[q].K + BK - 1) / BK;
  } else {
    tot_kt = (p.K + BK - 1) / BK;
  }
  const int kt_per = p.k_per_split / BK;
  const int kt0 = split * kt_per;
  const int nk = max(0, min(kt_per, tot_kt - kt0));
  if (nk <= 0 && !p.c_split && !p.cs_part) return;  // empty split adds nothing (a slab gets its zeros below)
  // ---- per-thread DMA chunks: row (k within the tile) and logical chunk ----
  // chunk q = i*NT + tid lands at LDS byte q*16 of the image: row q>>4, slot
  // q&15, holding logical 8-element chunk (slot ^ ((row & 3) << 2)).
  int a_row[NA], a_col[NA];
  int b_row[NB], b_col[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    a_row[i] = q / CA;
    a_col[i] = (((q % CA) ^ wg_swz<CA>(a_row[i])) << 3);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    b_row[i] = q / CB;
    b_col[i] = (((q % CB) ^ wg_swz<CB>(b_row[i])) << 3);
  }
  // im2col^T: each A chunk's filter tap (r, s) and channel, fixed for the
  // block (a chunk's 8 rows m never straddle a tap: Cc % 8 == 0), so a tile
  // may span taps (the 64-channel convs' 128-row tiles)
  int tap_r[AM == A_IM2COL_T ? NA : 1], tap_s[AM == A_IM2COL_T ? NA : 1];
  if constexpr (AM == A_IM2COL_T) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + a_col[i];
      const uint32_t rs = fdiv((uint32_t)m, p.fd_C);
      const uint32_t r = fdiv(rs, p.fd_S);
      tap_r[i] = (int)r;
      tap_s[i] = (int)rs - (int)r * p.Sk;
      a_col[i] = m - (int)rs * p.Cc;  // from here on: the chunk's channel
    }
  }

  typedef __attribute__((address_space(3))) void lds_void;
  struct WgSrc {
    const T* Ag;
    const T* Bg;
    int K, k0, gH, gW, gHo, gWo;
    FastDiv fdHoWo, fdWo;
  };
  auto tile_src = [&](int kt) {
    // this K-tile's group (uniform: scalar selects over the kernarg groups)
    const int vkt = kt0 + kt;
    WgSrc ws{(const T*)p.A, (const T*)p.B, p.K, 0, p.H, p.W, p.Ho, p.Wo, p.fd_HoWo, p.fd_Wo};
    int t0 = 0;
    if (p.ngroups > 0) {
      GemmGroup G = p.groups[0];
#pragma unroll
      for (int q = 1; q < MAX_GROUPS; ++q)
        if (q < p.ngroups && vkt >= p.groups[q].start) G = p.groups[q];
      ws.Ag = (const T*)G.A; ws.Bg = (const T*)G.B;
      ws.K = G.K; t0 = G.start;
      ws.gH = G.H; ws.gW = G.W; ws.gHo = G.Ho; ws.gWo = G.Wo;
      ws.fdHoWo = G.fd_HoWo; ws.fdWo = G.fd_Wo;
    }
    ws.k0 = (vkt - t0) * BK;  // first reduction row of the tile within its group
    return ws;
  };
  // DMA instruction j of a stage: j < NA the A chunks, then the B chunks
  auto issue_range = [&](const WgSrc& ws, int stage, auto lo_c, auto hi_c) {
    constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
    char* sb = smem + stage * STAGE_BYTES;
    static_for<LO, HI>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j < NA) {
        const int k = ws.k0 + a_row[j];
        const T* src = zero;
        if constexpr (AM == A_IM2COL_T) {
          const uint32_t n = fdiv((uint32_t)k, ws.fdHoWo);
          const int rem = k - (int)n * ws.gHo * ws.gWo;
          const uint32_t ho = fdiv((uint32_t)rem, ws.fdWo);
          const int wo = rem - (int)ho * ws.gWo;
          const int hi = (int)ho * p.sh - p.pt + tap_r[j], wi = wo * p.sw - p.pl + tap_s[j];
          const bool ok = k < ws.K && tap_r[j] < p.Rk && hi >= 0 && hi < ws.gH && wi >= 0 && wi < ws.gW;
          if (ok) src = ws.Ag + ((long long)((int)n * ws.gH + hi) * ws.gW + wi) * p.Cc + a_col[j];
        } else {
          const bool ok = k < ws.K && m0 + a_col[j] < M;
          if (ok) src = ws.Ag + (long long)k * p.lda + m0 + a_col[j];
        }
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (j * NT + dwave * 64) * 16), 16, 0, 0);
      } else {
        constexpr int i = j - NA;
        const int k = ws.k0 + b_row[i];
        const bool ok = k < ws.K && n0 + b_col[i] < N;
        const T* src = ok ? ws.Bg + (long long)k * p.ldb + n0 + b_col[i] : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + A_BYTES + (i * NT + dwave * 64) * 16),
                                         16, 0, 0);
      }
    });
  };
  auto issue = [&](int kt, int stage) {
    issue_range(tile_src(kt), stage, std::integral_constant<int, 0>{}, std::integral_constant<int, NA + NB>{});
  };

  accT acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[a][b][i] = 0.f;
  // folded bias-gradient column sums (p.cs_part, MF 32): the k-steps of the
  // split are dealt round-robin over the (m-tile, wave row) pairs (k-steps
  // cs_r, cs_r + cs_R, ...), so every dz element of the split is summed once;
  // a wave sums its k-steps' B fragments with v_dot2c_f32_bf16 against (1, 1)
  // (lane l holds column cb + (l & 31), k rows 8 (l >> 5) .. +7 of the
  // k-step), fixed order; a wave-uniform counter, no per-step division
  float* const csum = (float*)(smem + STAGES * STAGE_BYTES) + (CS_BYTES ? (int)threadIdx.x : 0);  // [b * NC]
  const bool cs_on = CS_BYTES > 0 && p.cs_part != nullptr && wave < WM * WN;  // MFMA waves
  if (cs_on)
#pragma unroll
    for (int b = 0; b < TN; ++b) csum[b * NC] = 0.f;
  const int cs_R = p.tiles_m * WM;
  // the next k-step this wave sums, relative to the current K-tile's first
  // (never reached when the fold is off)
  int cs_rel = cs_on ? tmi * WM + wm : 1 << 30;

  // transposed fragment reads: lane (g16, tq, tp) supplies logical (row k =
  // ks*16 + 8*lh + tq [+4], cols cb + 16*g16 + 4*tp .. +3); lane i of each
  // 16-lane group receives column i of the 4 rows. MF 16: lane (q = l >> 4,
  // tq, tp) supplies row k = 32 ks + 8 q + tq [+4], cols cb + 4 tp .. +3, so
  // lane l receives column cb + (l & 15), k = 32 ks + 8 (l >> 4) .. +7
  const int g16 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  auto tr_addr_a = [&](const char* img, int k, int col) -> const char* {
    return img + k * ROWA + ((((col >> 3) ^ wg_swz<CA>(k)) << 4) | ((col & 7) << 1));
  };
  auto tr_addr_b = [&](const char* img, int k, int col) -> const char* {
    return img + k * ROWBB + ((((col >> 3) ^ wg_swz<CB>(k)) << 4) | ((col & 7) << 1));
  };
  const int kl = MF == 32 ? 8 * lh + tq : 8 * (lane >> 4) + tq;  // this lane's k row within a k-step
  const int cofs = MF == 32 ? 16 * g16 + 4 * tp : 4 * tp;        // and its column offset within a tile
  auto compute_mid = [&](int stage, auto&& mid) {
    const char* As = smem + stage * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
    static_for<0, BK / KS>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      const int k = ks * KS + kl;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const char* a = tr_addr_a(As, k, wm * WTM + t * MF + cofs);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a + 4 * ROWA));
        __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[t] = __builtin_bit_cast(bf16x8, w8);
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const char* b = tr_addr_b(Bs, k, wn * WTN + t * MF + cofs);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b + 4 * ROWBB));
        __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[t] = __builtin_bit_cast(bf16x8, w8);
      }
      if constexpr (CS_BYTES > 0) {
        if (ks == cs_rel) {
          typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
          const bf16x2_t one2 = {(__bf16)1.f, (__bf16)1.f};
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            float v = csum[b * NC];
#pragma unroll
            for (int e = 0; e < 8; e += 2)
              v = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{bfr[b][e], bfr[b][e + 1]}, one2, v, false);
            csum[b * NC] = v;
          }
          cs_rel += cs_R;
        }
        if constexpr (ks + 1 == BK / KS) cs_rel -= BK / KS;  // the next K-tile's k-steps
      }
      mid(ksc);
      if constexpr (SPREAD == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          if constexpr (MF == 16)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
          else
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
        }
      if constexpr (SPREAD == 2) __builtin_amdgcn_s_setprio(0);
    });
  };
  auto compute = [&](int stage) { compute_mid(stage, [](auto) {}); };

  // STAGES - 1 K-tiles in flight: a weight-gradient K-tile is little MFMA
  // work per block (8 per wave), so the DMA latency needs a deeper queue
  constexpr int PER_STAGE = NA + NB;
  if constexpr (NLW > 0) {
    // the two roles in separate loops (a shared loop keeps the DMA state live
    // in the MFMA waves and spills them at 16 waves per block)
    if (loader) {
#pragma unroll
      for (int i = 0; i < STAGES - 1; ++i)
        if (i < nk) issue(i, i);
      for (int t = 0; t < nk; ++t) {
        const int ahead = nk - 1 - t;
        if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
        else if (STAGES > 3 && ahead == 1) wait_vmcnt<PER_STAGE>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // K-tile t visible; stage (t-1)%STAGES is free
        if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      }
      return;  // the epilogue has no barrier
    }
    for (int t = 0; t < nk; ++t) {
      __builtin_amdgcn_s_barrier();
      compute(t % STAGES);
    }
  } else {
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < nk) issue(i, i);
  for (int t = 0; t < nk; ++t) {
    const int ahead = nk - 1 - t;  // tiles issued after tile t (capped below)
    if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
    else if (STAGES > 3 && ahead == 1) wait_vmcnt<PER_STAGE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // everyone's part landed; stage (t-1)%STAGES is free
    if constexpr (SPREAD != 0) {
      const bool more = t + STAGES - 1 < nk;
      const WgSrc ws = tile_src(t + STAGES - 1);
      const int st = (t + STAGES - 1) % STAGES;
      compute_mid(t % STAGES, [&](auto ksc) {
        constexpr int ks = decltype(ksc)::value, NKS = BK / KS, PS = NA + NB;
        if (more)
          issue_range(ws, st, std::integral_constant<int, ks * PS / NKS>{},
                      std::integral_constant<int, (ks + 1) * PS / NKS>{});
      });
    } else {
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      compute(t % STAGES);
    }
  }
  }

  if constexpr (CS_BYTES > 0) {
    if (cs_on) {  // lanes l and l ^ 32 hold the two 8-row halves of each k-step
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const float c = csum[b * NC];
        const float v = c + __shfl_xor(c, 32);
        const int col = n0 + wn * WTN + b * 32 + lane;
        if (lane < 32 && col < N) p.cs_part[((long long)(split * p.tiles_m + tmi) * WM + wm) * N + col] = v;
      }
    }
  }
  float* Cg = (float*)p.C;
  if constexpr (MF == 16) {
    // lane: row m0 + wm WTM + 16 a + (l & 15), columns n0 + wn WTN + 16 b +
    // 4 (l >> 4) .. +3
    const bool vec = (N & 3) == 0 && (p.ldc & 3) == 0;
    float* slab = p.c_split ? Cg + (long long)split * p.c_split : nullptr;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int row = m0 + wm * WTM + a * 16 + (lane & 15);
      if (row >= M) continue;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n0 + wn * WTN + b * 16 + 4 * (lane >> 4);
        if (col >= N) continue;
        if (slab) {  // deterministic split-K: raw partials, summed in split order later
          float* dst = slab + (long long)row * p.ldc + col;
          if (vec) *(f32x4*)dst = acc[a][b];
          else
            for (int j = 0; j < 4 && col + j < N; ++j) dst[j] = acc[a][b][j];
        } else {  // one split: a single fp32 atomic per element (one adder, any order)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (col + j < N)
              atomicAdd(Cg + (long long)row * p.ldc + col + j,
                        acc[a][b][j] * (p.col_scale ? p.col_scale[col + j] : 1.f) * p.alpha);
        }
      }
    }
  } else {
  if (p.c_split) {
    // deterministic split-K: raw partials into this split's slab (plain
    // stores), summed in split order by wgrad_reduce_kernel
    float* slab = Cg + (long long)split * p.c_split;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n0 + wn * WTN + b * 32 + lr;
        if (col >= N) continue;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
          if (row < M) slab[(long long)row * p.ldc + col] = acc[a][b][i];
        }
      }
    return;
  }
  // one split: a single fp32 atomic per element (one adder, any order)
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + wn * WTN + b * 32 + lr;
      if (col >= N) continue;
      const float cs = (p.col_scale ? p.col_scale[col] : 1.f) * p.alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        if (row < M) atomicAdd(Cg + (long long)row * p.ldc + col, acc[a][b][i] * cs);
      }
    }
  }
  }
}


// ---------------------------------------------------------------------------
// Grouped weight-gradient GEMMs (the deferred Dense wgrads of a backward,
// deferred.hip): block -> (job, 128 x 128 tile) by the jobs' block prefix;
// each block runs its tile's WHOLE reduction (no split: one writer per C
// element, C += alpha * acc by read-modify-write) with the LDS-DMA pipeline
// and transposing fragment reads of gemm_pipe_wg_kernel (A_COL / B_KN).
struct GemmJobs {
  DefGemmJob j[GEMM_JOBS_PER_LAUNCH];
  const void* zero;  // 256 B of zeros (out-of-range rows / columns)
  int n;
};

template <int BM, int BN, int WM, int WN, int NSTAGE>
__global__ __launch_bounds__(64 * WM * WN) void gemm_wg_jobs_kernel(const GemmJobs J) {
  typedef bf16 T;
  constexpr int NT = 64 * WM * WN;
  constexpr int BK = 64;
  static_assert(BM % 128 == 0 && BN % 128 == 0, ">= 16 chunks per LDS row (the swizzle flips chunk bits 2-3)");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  constexpr int ROWA = BM * 2, ROWBB = BN * 2;
  constexpr int A_BYTES = BK * ROWA, B_BYTES = BK * ROWBB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int CA = BM / 8, CB = BN / 8;
  constexpr int NA = BK * (BM / 8) / NT, NB = BK * (BN / 8) / NT;
  static_assert(NA * NT == BK * (BM / 8) && NB * NT == BK * (BN / 8), "");
  constexpr int STAGES = NSTAGE;
  static_assert(STAGES >= 2 && STAGES * STAGE_BYTES <= 160 * 1024, "");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  // this block's job: static selects over the kernarg table (no dynamic
  // index into the kernarg struct)
  DefGemmJob G = J.j[0];
#pragma unroll
  for (int q = 1; q < GEMM_JOBS_PER_LAUNCH; ++q)
    if (q < J.n && (int)blockIdx.x >= J.j[q].blk0) G = J.j[q];
  const int local = (int)blockIdx.x - G.blk0;
  const int tmi = local / G.tiles_n, tni = local - tmi * G.tiles_n;
  const int M = G.M, N = G.N, K = G.K;
  const int m0 = tmi * BM, n0 = tni * BN;
  const T* Ag = (const T*)G.A;
  const T* Bg = (const T*)G.B;
  const T* zero = (const T*)J.zero;
  const int nk = (K + BK - 1) / BK;

  int a_row[NA], a_col[NA];
  int b_row[NB], b_col[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    a_row[i] = q / CA;
    a_col[i] = (((q % CA) ^ ((a_row[i] & 3) << 2)) << 3);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    b_row[i] = q / CB;
    b_col[i] = (((q % CB) ^ ((b_row[i] & 3) << 2)) << 3);
  }
  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](int kt, int stage) {
    const int k0 = kt * BK;
    char* sb = smem + stage * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int k = k0 + a_row[i];
      const bool ok = k < K && m0 + a_col[i] < M;
      const T* src = ok ? Ag + (long long)k * G.lda + m0 + a_col[i] : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (i * NT + wave * 64) * 16), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int k = k0 + b_row[i];
      const bool ok = k < K && n0 + b_col[i] < N;
      const T* src = ok ? Bg + (long long)k * G.ldb + n0 + b_col[i] : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + A_BYTES + (i * NT + wave * 64) * 16), 16,
                                       0, 0);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
  const int g16 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  auto tr_addr = [&](const char* img, int rowb, int k, int col) -> const char* {
    return img + k * rowb + ((((col >> 3) ^ ((k & 3) << 2)) << 4) | ((col & 7) << 1));
  };
  auto compute_mid = [&](int stage, auto&& mid) {
    const char* As = smem + stage * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
    static_for<0, BK / 16>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      const int k = ks * 16 + 8 * lh + tq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const char* a = tr_addr(As, ROWA, k, wm * WTM + t * 32 + 16 * g16 + 4 * tp);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a + 4 * ROWA));
        __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[t] = __builtin_bit_cast(bf16x8, w8);
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const char* b = tr_addr(Bs, ROWBB, k, wn * WTN + t * 32 + 16 * g16 + 4 * tp);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b + 4 * ROWBB));
        __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[t] = __builtin_bit_cast(bf16x8, w8);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    });
  };
  auto compute = [&](int stage) { compute_mid(stage, [](auto) {}); };
  constexpr int PER_STAGE = NA + NB;
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < nk) issue(i, i);
  for (int t = 0; t < nk; ++t) {
    const int ahead = nk - 1 - t;
    if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
    else if (STAGES > 3 && ahead == 1) wait_vmcnt<PER_STAGE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    compute(t % STAGES);
  }
  // one writer per element in this launch: C += alpha * acc
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + wn * WTN + b * 32 + lr;
      if (col >= N) continue;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        if (row < M) {
          float* cp = G.C + (long long)row * G.ldc + col;
          *cp = *cp + acc[a][b][i] * G.alpha;
        }
      }
    }
  }
}

}  // namespace fpnmt
