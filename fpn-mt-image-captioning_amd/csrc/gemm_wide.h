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
#include "gemm_pipe.h"

namespace fpnmt {

template <int BM, int BN, int WM, int WN, int AM, int STAGES>
__global__ __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_wide_kernel(const GemmParams p) {
  // the body only exists for the device: the buffer-resource type and its
  // builtins are not declared in the host pass, and a failed host-side
  // instantiation silently drops the launch stub
#if defined(__HIP_DEVICE_COMPILE__)

  typedef bf16 T;
  constexpr int NT = 64 * WM * WN;
  constexpr int BK = 64;
  static_assert(STAGES >= 2 && STAGES <= 4, "stages");
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

  constexpr int PER_STAGE = NA + NB;  // DMA instructions per thread per K-tile
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < STAGES - 1; ++i) issue(i, i, i < nk);
    wait_vmcnt<(STAGES - 2) * PER_STAGE>();  // tile 0 (the STAGES-2 younger tiles stay in flight)
    __builtin_amdgcn_s_barrier();
    Frag F0, F1;
    rd(smem, 0, F0);
    int st = 0;  // stage of tile t
    for (int t = 0; t < nk - 1; ++t) {
      const char* S = smem + st * STAGE_BYTES;
      const int st1 = st + 1 == STAGES ? 0 : st + 1;
      rd(S, 1, F1);
      mm(F0);
      sched_step();
      __builtin_amdgcn_sched_barrier(0);
      rd(S, 2, F0);
      mm(F1);
      sched_step();
      __builtin_amdgcn_sched_barrier(0);
      rd(S, 3, F1);
      mm(F0);
      sched_step();
      __builtin_amdgcn_sched_barrier(0);
      // tile t+1 landed for this thread (tiles t+2 .. t+STAGES-1 in flight),
      // this wave's reads of tile t done; then for every wave
      wait_vmcnt<(STAGES - 2) * PER_STAGE>();
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      rd(smem + st1 * STAGE_BYTES, 0, F0);
      {
        // the last k-step's MFMAs, each followed by two DMA chunks of tile
        // t+STAGES (source order pinned by the fences)
        const TileSrc ts = tile_src(t + STAGES, st, t + STAGES < nk);
        __builtin_amdgcn_sched_barrier(0);
        static_for<0, NMF>([&](auto jc) {
          constexpr int j = decltype(jc)::value, a = j / TN, b = j % TN;
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F1.b[b], F1.a[a], acc[a][b], 0, 0, 0);
          constexpr int per = (NA + NB + NMF - 1) / NMF;
          static_for<j * per, (j + 1) * per>([&](auto cc) { dma(ts, cc); });
          __builtin_amdgcn_sched_barrier(0);
        });
      }
      st = st1;
    }
    {  // last K-tile: no barrier, no DMA
      const char* S = smem + st * STAGE_BYTES;
      rd(S, 1, F1);
      mm(F0);
      rd(S, 2, F0);
      mm(F1);
      rd(S, 3, F1);
      mm(F0);
      mm(F1);
    }
    wait_vmcnt<0>();  // the dummy DMAs land before the block's LDS is released
  }

  char* Cg = (char*)Cp0;
  const long long c_off = zo * p.c_so + zi * p.c_si + (long long)blockIdx.y * p.c_split;
  epilogue_direct<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg0 != nullptr, rpre);
#endif
}

}  // namespace fpnmt
