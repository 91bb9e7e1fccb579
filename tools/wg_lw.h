// Loader-wave form of gemm_pipe_wg_kernel (round 6 probe; tools/wg_bench.hip
// -DWB_LW): NLW loader waves own the LDS-DMA of the ring, the WM x WN MFMA
// waves only do the transposing fragment reads and MFMAs. Same LDS images,
// K order and slab / atomic epilogue as gemm_pipe_wg_kernel<..., MF>.
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"

namespace fpnmt {

template <int BM, int BN, int WM, int WN, int AM, int NLW, int MF = 32>
__global__ __launch_bounds__(64 * (WM * WN + NLW)) void gemm_pipe_wg_lw_kernel(const GemmParams p) {
  constexpr int SPREAD = 0;
  typedef bf16 T;
  constexpr int NC = 64 * WM * WN, NT = 64 * NLW;  // NT: the DMA-issuing (loader) threads
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
  constexpr int STAGES = 4 * STAGE_BYTES <= 160 * 1024 ? 4 : 3 * STAGE_BYTES <= 160 * 1024 ? 3 : 2;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const bool loader = wave >= WM * WN;
  const int tid = loader ? (int)threadIdx.x - NC : 0;  // loader lane index (DMA chunk owner)
  const int dwave = loader ? wave - WM * WN : 0;
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
  if (nk <= 0 && !p.c_split) return;  // empty split adds nothing (a slab gets its zeros below)
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
  if (loader) {
#pragma unroll
    for (int i = 0; i < STAGES - 1; ++i)
      if (i < nk) issue(i, i);
    for (int t = 0; t < nk; ++t) {
      const int ahead = nk - 1 - t;  // tiles issued after tile t (capped below)
      if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
      else if (STAGES > 3 && ahead == 1) wait_vmcnt<PER_STAGE>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // K-tile t visible; stage (t-1)%STAGES is free
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    }
    return;
  }
  for (int t = 0; t < nk; ++t) {
    __builtin_amdgcn_s_barrier();
    compute(t % STAGES);
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



}  // namespace fpnmt
