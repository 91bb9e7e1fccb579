// One-wave-per-SIMD LDS-DMA MFMA GEMM for the wide k-contiguous problems
// (implicit-GEMM conv forward / stride-1 bwd-data with C % 64 == 0, and
// row-major Dense), B = (N, K) weights. Same operand images, zero page,
// grouping and split-K conventions as gemm_pipe_kernel (gemm_pipe.h); what
// differs is the schedule:
//
//   * 4 waves (one per SIMD), each owning a (BM/WM) x (BN/WN) output tile
//     (64 x 128 on the 128 x 256 block): 6 ds_read_b128 feed 8 MFMAs per
//     16-deep k-step (the 8-wave 64 x 64 form reads 4 per 4), and with 512
//     registers per lane the accumulators, two fragment sets and the
//     residual prefetch all stay in registers;
//   * fragments of k-step s+1 are read under the MFMAs of step s (two named
//     register sets, static indices);
//   * ONE barrier per K-tile, placed before the last k-step's MFMAs: before
//     it each wave retires its own DMA of tile t+1 (counted vmcnt, tiles
//     t+2.. stay in flight) and its LDS reads of tile t (lgkmcnt 0; the
//     last step's fragments are already in registers), so after it tile
//     t+1 is visible to every wave (its first fragments are read under the
//     last MFMAs of tile t) and tile t's stage is free: the DMA of tile
//     t+STAGES is issued into it right there, interleaved with those MFMAs.
//     The pipeline therefore never drains at a K-tile boundary, and a DMA
//     has STAGES-1 K-tiles of MFMA time to land.
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"

namespace fpnmt {

// ---------------------------------------------------------------------------
// The K loop shared by the wide kernels (3 LDS stages, tile k in stage k % 3).
// Per K-tile t: four 16-deep k-steps; before each, the next step's fragments
// are read (F0 / F1 alternate), and each step's MFMAs are spread with a share
// of the DMA chunks of a later tile. The barrier B_t sits before step 3:
//   * before it every thread retires its DMA of tile t+1 (tile t+2's PER
//     chunks stay in flight: vmcnt(PER)) and its LDS reads of tile t;
//   * after it tile t+1 is readable (its step-0 fragments are read under the
//     last MFMAs of t), and tile t's stage is free: the first quarter of the
//     DMA of tile t+3 goes there during step 3, the rest during steps 0-2 of
//     iteration t+1. A DMA thus has 1-2 K-tiles of MFMA time to land, the
//     address arithmetic of a chunk sits beside the MFMAs, and the pipeline
//     does not drain at K-tile boundaries.
// Tiles past the end are issued with out-of-range offsets (zeros into a free
// stage) so the wait counts never change; the last K-tile issues nothing.
//   tile_src(kt, stage, live) -> TS;  dma(ts, integral_constant<c>)
//   rd(stage_base, ks, Frag&);         mm1(const Frag&, integral_constant<j>)
template <int PER, int NMF, int STAGE_BYTES, class Frag, class FTS, class FDma, class FRd, class FMm>
__device__ __forceinline__ void wide_mainloop(int nk, char* smem, FTS tile_src, FDma dma, FRd rd, FMm mm1, Frag& F0,
                                              Frag& F1) {
  constexpr int CPS = (PER + 3) / 4;        // chunks per k-step
  constexpr int CPM = (CPS + NMF - 1) / NMF;  // chunks per MFMA
  // one k-step: MFMA j, then its chunks of issue order O (0 = the step after
  // the barrier, 1..3 = steps 0..2 of the next iteration)
  auto step = [&](const Frag& F, auto oc, const auto& ts, auto dmac) {
    constexpr int O = decltype(oc)::value;
    constexpr bool DMA = decltype(dmac)::value;
    static_for<0, NMF>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      mm1(F, jc);
      if constexpr (DMA) {
        constexpr int lo = O * CPS + j * CPM;
        constexpr int hi0 = O * CPS + (j + 1) * CPM, hi1 = (O + 1) * CPS;
        constexpr int hi = hi0 < hi1 ? (hi0 < PER ? hi0 : PER) : (hi1 < PER ? hi1 : PER);
        static_for<lo, (hi > lo ? hi : lo)>([&](auto cc) { dma(ts, cc); });
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  typedef std::integral_constant<bool, true> yes;
  typedef std::integral_constant<bool, false> no;
  // prologue: tiles 0 and 1 whole, the first quarter of tile 2
  {
    const auto t0 = tile_src(0, 0, true);
    const auto t1 = tile_src(1, 1, 1 < nk);
    const auto t2 = tile_src(2, 2, 2 < nk);
    static_for<0, PER>([&](auto cc) { dma(t0, cc); });
    static_for<0, PER>([&](auto cc) { dma(t1, cc); });
    static_for<0, (CPS < PER ? CPS : PER)>([&](auto cc) { dma(t2, cc); });
  }
  wait_vmcnt<PER + (CPS < PER ? CPS : PER)>();  // tile 0 landed
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  rd(smem, 0, F0);
  auto ts = tile_src(2, 2, 2 < nk);  // the tile whose remaining chunks steps 0-2 issue
  int st = 0;
  for (int t = 0; t < nk - 1; ++t) {
    const char* S = smem + st * STAGE_BYTES;
    const int st1 = st == 2 ? 0 : st + 1;
    rd(S, 1, F1);
    step(F0, std::integral_constant<int, 1>{}, ts, yes{});
    rd(S, 2, F0);
    step(F1, std::integral_constant<int, 2>{}, ts, yes{});
    rd(S, 3, F1);
    step(F0, std::integral_constant<int, 3>{}, ts, yes{});
    wait_vmcnt<PER>();                   // tile t+1 landed (tile t+2 in flight)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of tile t done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    rd(smem + st1 * STAGE_BYTES, 0, F0);
    ts = tile_src(t + 3, st, t + 3 < nk);  // into tile t's stage, free now
    step(F1, std::integral_constant<int, 0>{}, ts, yes{});
    st = st1;
  }
  {  // last K-tile: no barrier, no DMA
    const char* S = smem + st * STAGE_BYTES;
    rd(S, 1, F1);
    step(F0, std::integral_constant<int, 0>{}, ts, no{});
    rd(S, 2, F0);
    step(F1, std::integral_constant<int, 0>{}, ts, no{});
    rd(S, 3, F1);
    step(F0, std::integral_constant<int, 0>{}, ts, no{});
    step(F1, std::integral_constant<int, 0>{}, ts, no{});
  }
  wait_vmcnt<0>();  // every DMA (the dummies too) lands before the block's LDS is released
}

template <int BM, int BN, int WM, int WN, int AM, int STAGES>
__global__ __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_wide_kernel(const GemmParams p) {
  // the body only exists for the device: the buffer-resource type and its
  // builtins are not declared in the host pass, and a failed host-side
  // instantiation silently drops the launch stub
#if defined(__HIP_DEVICE_COMPILE__)

  typedef bf16 T;
  constexpr int NT = 64 * WM * WN;
  constexpr int BK = 64;
  static_assert(STAGES == 3, "the wide main loop runs 3 stages");
  static_assert(AM == A_ROW || AM == A_IM2COL, "k-contiguous A only");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;  // 16-B DMA chunks per thread per stage
  static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "");
  constexpr int SMEM = STAGES * STAGE_BYTES;
  static_assert(SMEM <= 160 * 1024, "LDS");
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
  if (p.ngroups > 0) {  // m-grouped launch (shared B); static kernarg indices only
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
  const int kt0 = (int)blockIdx.y * (p.k_per_split / BK);
  const int nk = max(0, min(K / BK - kt0, p.k_per_split / BK));

  // operands through buffer descriptors: 32-bit byte offsets, and a row / tap
  // outside the operand gets an offset past num_records, which the DMA turns
  // into zeros (no zero page, no 64-bit address arithmetic per chunk)
  constexpr unsigned OOB = 0x80000000u;
  long long a_bytes;
  if constexpr (AM == A_ROW) a_bytes = (long long)M * p.lda * 2;
  else a_bytes = (long long)(fdiv((uint32_t)(M - 1), gfdHoWo) + 1) * gH * gW * p.Cc * 2;
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)Ag, (short)0, (int)min(a_bytes, (long long)OOB), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)Bg, (short)0, (int)min((long long)N * p.ldb * 2, (long long)OOB), 0x00020000);

  // per-thread DMA sources, as gemm_pipe_kernel: chunk q = i*NT + tid lands
  // at LDS byte q*16 (row q>>3, slot q&7 holding logical chunk slot ^ sw(row));
  // im2col rows keep the byte offset of their (hi0, wi0) pixel (mod 2^32: a
  // padding row's base may be "negative") and a bit per in-image filter tap
  unsigned a_off[NA], a_vm[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    const int row = q >> 3;
    const int kc = ((q & 7) ^ ((row >> 1) & 7)) * 8;
    const int m = m0 + row;
    if constexpr (AM == A_ROW) {
      a_off[i] = (unsigned)(m * p.lda + kc) * 2u;
      a_vm[i] = m < M ? ~0u : 0u;
    } else {
      const uint32_t nimg = fdiv((uint32_t)min(m, M - 1), gfdHoWo);
      const int rem = min(m, M - 1) - (int)nimg * gHo * gWo;
      const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
      const int wo = rem - (int)ho * gWo;
      const int hi0 = (int)ho * p.sh - p.pt, wi0 = wo * p.sw - p.pl;
      a_off[i] = (unsigned)((((int)nimg * gH + hi0) * gW + wi0) * p.Cc + kc) * 2u;
      unsigned vm = 0;
      if (m < M)
        for (int r = 0; r < p.Rk; ++r)
          for (int s2 = 0; s2 < p.Sk; ++s2)
            if (hi0 + r >= 0 && hi0 + r < gH && wi0 + s2 >= 0 && wi0 + s2 < gW) vm |= 1u << (r * p.Sk + s2);
      a_vm[i] = vm;
    }
  }
  unsigned b_off[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    const int row = q >> 3;
    const int kc = ((q & 7) ^ ((row >> 1) & 7)) * 8;
    b_off[i] = n0 + row < N ? (unsigned)((n0 + row) * p.ldb + kc) * 2u : OOB;
  }

  typedef __attribute__((address_space(3))) void lds_void;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  // K-tile kt into `stage`; live == false issues the same DMA count with every
  // offset out of range (zeros into a free stage), so the wait counts below
  // stay the same in every iteration and the loop body has no branch.
  // tile_src: the tile's scalar part; dma<c>: the thread's chunk c (A chunks
  // first), so the issue can be spread over the MFMAs
  struct TileSrc {
    char* sb;
    int tap;
    unsigned tap_off, k0b, kill;
  };
  auto tile_src = [&](int kt, int stage, bool live) {
    TileSrc ts;
    const int k0 = (kt0 + kt) * BK;
    ts.sb = smem + stage * STAGE_BYTES + wave_u * 1024;
    ts.tap = 0;
    ts.tap_off = (unsigned)k0 * 2u;
    if constexpr (AM == A_IM2COL) {
      const uint32_t rs = fdiv((uint32_t)k0, p.fd_C);
      const int cb = k0 - (int)rs * p.Cc;
      const uint32_t r = fdiv(rs, p.fd_S);
      const int s2 = (int)rs - (int)r * p.Sk;
      ts.tap = (int)rs;
      ts.tap_off = (unsigned)(((int)r * gW + s2) * p.Cc + cb) * 2u;
    }
    ts.k0b = (unsigned)k0 * 2u;
    ts.kill = live ? 0u : OOB;
    return ts;
  };
  auto dma = [&](const TileSrc& ts, auto cc) {
    constexpr int c = decltype(cc)::value;
    if constexpr (c < NA) {
      const unsigned off = ((a_vm[c] >> ts.tap) & 1u) ? a_off[c] + ts.tap_off : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(ts.sb + c * NT * 16), 16, off | ts.kill, 0, 0, 0);
    } else if constexpr (c < NA + NB) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void*)(ts.sb + A_BYTES + (c - NA) * NT * 16), 16,
                                               (b_off[c - NA] + ts.k0b) | ts.kill, 0, 0, 0);
    }
  };
  auto issue = [&](int kt, int stage, bool live) {
    const TileSrc ts = tile_src(kt, stage, live);
    static_for<0, NA + NB>([&](auto cc) { dma(ts, cc); });
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  // fragment row offsets (bytes) within a stage; the chunk swizzle of a row
  // depends only on (row >> 1) & 7 = (lr >> 1) & 7 since every fragment row
  // base is a multiple of 32
  const int sw = (lr >> 1) & 7;
  const int a_row_b = (wm * WTM + lr) * 128;
  const int b_row_b = A_BYTES + (wn * WTN + lr) * 128;
  struct Frag {
    bf16x8 a[TM], b[TN];
  };
  auto rd = [&](const char* S, int ks, Frag& F) {
    const int cb = ((ks * 2 + lh) ^ sw) << 4;
#pragma unroll
    for (int t = 0; t < TM; ++t) F.a[t] = *(const bf16x8*)(S + a_row_b + t * 32 * 128 + cb);
#pragma unroll
    for (int t = 0; t < TN; ++t) F.b[t] = *(const bf16x8*)(S + b_row_b + t * 32 * 128 + cb);
  };
  auto mm = [&](const Frag& F) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.b[b], F.a[a], acc[a][b], 0, 0, 0);
  };
  constexpr int NMF = TM * TN, NRD = TM + TN;
  // one k-step's MFMAs with the next step's fragment reads between them
  auto sched_step = [&]() {
#pragma unroll
    for (int j = 0; j < NMF; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      if (j < NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
  };

  // residual / act-mask rows for the direct epilogue, in flight under the K loop
  bf16x4 rpre[TM][TN][4];
  const T* Rg0 = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  if (Rg0) prefetch_r_direct<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);

  if (nk > 0) {
    Frag F0, F1;
    auto mm1 = [&](const Frag& F, auto jc) {
      constexpr int j = decltype(jc)::value, a = j / TN, b = j % TN;
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.b[b], F.a[a], acc[a][b], 0, 0, 0);
    };
    wide_mainloop<NA + NB, TM * TN, STAGE_BYTES>(nk, smem, tile_src, dma, rd, mm1, F0, F1);
  }

  char* Cg = (char*)Cp0;
  const long long c_off = zo * p.c_so + zi * p.c_si + (long long)blockIdx.y * p.c_split;
  epilogue_direct<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg0 != nullptr, rpre);
#endif
}


// ---------------------------------------------------------------------------
// Weight-gradient form on the same main loop: C[m][n] (+)= sum_k A[k][m] B[k][n]
// with A = im2col(x)^T (A_IM2COL_T: the BM-wide m range of a tile lies in ONE
// filter tap, Cc % BM == 0) or x rows (A_COL), B = dz rows (B_KN); k = output
// pixels / rows. LDS images [k][BM] / [k][BN] (lane-linear 16-B chunks,
// chunk index XOR (k & 3) << 2 on the source side, as gemm_pipe_wg_kernel),
// fragments by ds_read_b64_tr_b16. 4 waves, one per SIMD, (BM/WM) x (BN/WN)
// per wave (128 x 64 on 256 x 128: 12 transposed reads per 8 MFMAs). Split-K
// over a 1-D (split, tile) grid (k-grouped launches: the groups' K-tiles end
// to end), raw fp32 partials into the split's slab (c_split) or one fp32
// atomic per element for a single split — the conventions of
// gemm_pipe_wg_kernel, so the dispatch's slab reduce applies unchanged.
template <int BM, int BN, int WM, int WN, int AM>
__global__ __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_wide_wg_kernel(
    const GemmParams p) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef bf16 T;
  constexpr int NT = 64 * WM * WN;
  constexpr int BK = 64;
  static_assert(AM == A_IM2COL_T || AM == A_COL, "m-contiguous A only");
  static_assert(BM % 128 == 0 && BN % 128 == 0, ">= 16 chunks per LDS row (the swizzle flips chunk bits 2-3)");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "");
  constexpr int ROWA = BM * 2, ROWB = BN * 2;
  constexpr int A_BYTES = BK * ROWA, B_BYTES = BK * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int CA = BM / 8, CB = BN / 8;
  constexpr int NA = BK * CA / NT, NB = BK * CB / NT;
  static_assert(NA * NT == BK * CA && NB * NT == BK * CB, "");
  static_assert(3 * STAGE_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[3 * STAGE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  const int ntile = p.tiles_m * p.tiles_n;
  const int w = xcd_remap(blockIdx.x, ntile * p.split_k);
  const int split = w / ntile;
  const int bid = w - split * ntile;
  const int tmi = bid / p.tiles_n;
  const int tni = bid - tmi * p.tiles_n;
  const int M = p.M, N = p.N;
  const int m0 = tmi * BM, n0 = tni * BN;
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

  constexpr unsigned OOB = 0x80000000u;  // >= num_records: the DMA returns zeros
  // per-thread chunks: row (k within the K-tile) and logical column chunk
  int a_row[NA], a_col[NA], b_row[NB], b_col[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    a_row[i] = q / CA;
    a_col[i] = ((q % CA) ^ ((a_row[i] & 3) << 2)) << 3;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    b_row[i] = q / CB;
    b_col[i] = ((q % CB) ^ ((b_row[i] & 3) << 2)) << 3;
  }
  int tap_r = 0, tap_s = 0, c_base = 0;
  if constexpr (AM == A_IM2COL_T) {
    const uint32_t rs = fdiv((uint32_t)m0, p.fd_C);
    c_base = m0 - (int)rs * p.Cc;
    const uint32_t r = fdiv(rs, p.fd_S);
    tap_r = (int)r;
    tap_s = (int)rs - (int)r * p.Sk;
  }

  typedef __attribute__((address_space(3))) void lds_void;
  struct TileSrc {
    __amdgpu_buffer_rsrc_t ra, rb;
    int k0, K, gH, gW, gHo, gWo;
    FastDiv fdHoWo, fdWo;
    char* sb;
    unsigned kill;
  };
  // K-tile kt (of this split) into `stage`: its group (uniform), descriptors
  // (2 GB records: every valid offset is below 2^31, host-checked)
  auto tile_src = [&](int kt, int stage, bool live) {
    TileSrc ts;
    const int vkt = kt0 + kt;
    const T* Ag = (const T*)p.A;
    const T* Bg = (const T*)p.B;
    int t0 = 0;
    ts.K = p.K; ts.gH = p.H; ts.gW = p.W; ts.gHo = p.Ho; ts.gWo = p.Wo;
    ts.fdHoWo = p.fd_HoWo; ts.fdWo = p.fd_Wo;
    if (p.ngroups > 0) {
      GemmGroup G = p.groups[0];
#pragma unroll
      for (int q = 1; q < MAX_GROUPS; ++q)
        if (q < p.ngroups && vkt >= p.groups[q].start) G = p.groups[q];
      Ag = (const T*)G.A; Bg = (const T*)G.B;
      ts.K = G.K; t0 = G.start;
      ts.gH = G.H; ts.gW = G.W; ts.gHo = G.Ho; ts.gWo = G.Wo;
      ts.fdHoWo = G.fd_HoWo; ts.fdWo = G.fd_Wo;
    }
    ts.k0 = (vkt - t0) * BK;
    ts.ra = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, (short)0, 0x7fffffff, 0x00020000);
    ts.rb = __builtin_amdgcn_make_buffer_rsrc((void*)Bg, (short)0, 0x7fffffff, 0x00020000);
    ts.sb = smem + stage * STAGE_BYTES + wave_u * 1024;
    ts.kill = live ? 0u : OOB;
    return ts;
  };
  auto dma = [&](const TileSrc& ts, auto cc) {
    constexpr int c = decltype(cc)::value;
    if constexpr (c < NA) {
      const int k = ts.k0 + a_row[c];
      unsigned off = OOB;
      if constexpr (AM == A_IM2COL_T) {
        const uint32_t n = fdiv((uint32_t)k, ts.fdHoWo);
        const int rem = k - (int)n * ts.gHo * ts.gWo;
        const uint32_t ho = fdiv((uint32_t)rem, ts.fdWo);
        const int wo = rem - (int)ho * ts.gWo;
        const int hi = (int)ho * p.sh - p.pt + tap_r, wi = wo * p.sw - p.pl + tap_s;
        const bool ok = k < ts.K && m0 + a_col[c] < M && hi >= 0 && hi < ts.gH && wi >= 0 && wi < ts.gW;
        if (ok) off = (unsigned)((((int)n * ts.gH + hi) * ts.gW + wi) * p.Cc + c_base + a_col[c]) * 2u;
      } else {
        if (k < ts.K && m0 + a_col[c] < M) off = (unsigned)(k * (int)p.lda + m0 + a_col[c]) * 2u;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ts.ra, (lds_void*)(ts.sb + c * NT * 16), 16, off | ts.kill, 0, 0, 0);
    } else if constexpr (c < NA + NB) {
      constexpr int i = c - NA;
      const int k = ts.k0 + b_row[i];
      const unsigned off =
          k < ts.K && n0 + b_col[i] < N ? (unsigned)(k * (int)p.ldb + n0 + b_col[i]) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ts.rb, (lds_void*)(ts.sb + A_BYTES + i * NT * 16), 16, off | ts.kill, 0,
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

  // transposed fragment reads: lane (g16, tq, tp) supplies logical (row k =
  // ks*16 + 8*lh + tq [+4], cols cb + 16*g16 + 4*tp .. +3)
  const int g16 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  struct Frag {
    bf16x8 a[TM], b[TN];
  };
  auto rd = [&](const char* S, int ks, Frag& F) {
    const int k = ks * 16 + 8 * lh + tq;
    auto tr = [&](const char* img, int rowb, int col) {
      const char* ad = img + k * rowb + ((((col >> 3) ^ ((k & 3) << 2)) << 4) | ((col & 7) << 1));
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(ad));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(ad + 4 * rowb));
      __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, w8);
    };
#pragma unroll
    for (int t = 0; t < TM; ++t) F.a[t] = tr(S, ROWA, wm * WTM + t * 32 + 16 * g16 + 4 * tp);
#pragma unroll
    for (int t = 0; t < TN; ++t) F.b[t] = tr(S + A_BYTES, ROWB, wn * WTN + t * 32 + 16 * g16 + 4 * tp);
  };
  auto mm1 = [&](const Frag& F, auto jc) {
    constexpr int j = decltype(jc)::value, a = j / TN, b = j % TN;
    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F.a[a], F.b[b], acc[a][b], 0, 0, 0);
  };
  if (nk <= 0 && !p.c_split) return;  // an empty split adds nothing (a slab gets its zeros below)
  if (nk > 0) {
    Frag F0, F1;
    wide_mainloop<NA + NB, TM * TN, STAGE_BYTES>(nk, smem, tile_src, dma, rd, mm1, F0, F1);
  }

  float* Cg = (float*)p.C;
  if (p.c_split) {  // raw partials into this split's slab, summed in split order by the reduce
    float* slab = Cg + (long long)split * p.c_split;
    static_for<0, TM>([&](auto ac) {
      constexpr int a = decltype(ac)::value;
      static_for<0, TN>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        const int col = n0 + wn * WTN + b * 32 + lr;
        if (col < N) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
            if (row < M) slab[(long long)row * p.ldc + col] = acc[a][b][i];
          }
        }
      });
    });
    return;
  }
  static_for<0, TM>([&](auto ac) {  // one split: a single fp32 atomic per element
    constexpr int a = decltype(ac)::value;
    static_for<0, TN>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      const int col = n0 + wn * WTN + b * 32 + lr;
      if (col < N) {
        const float cs = (p.col_scale ? p.col_scale[col] : 1.f) * p.alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
          if (row < M) atomicAdd(Cg + (long long)row * p.ldc + col, acc[a][b][i] * cs);
        }
      }
    });
  });
#endif
}

}  // namespace fpnmt
