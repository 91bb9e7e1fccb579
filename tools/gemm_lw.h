// Loader-wave form of the 8-wave 128x256 implicit-GEMM conv tile (the
// dominant conv, csrc/gemm_pipe.h gemm_pipe_kernel<128, 256, 2, 4, ..., MF 16>):
// WM x WN MFMA ("consumer") waves that only read LDS fragments and issue
// v_mfma_f32_16x16x32_bf16, plus NLW loader waves that own every LDS-DMA
// (global_load_lds_dwordx4) of the STAGES-deep K-tile ring and its im2col
// address arithmetic. VERDICT r05 item 3: the 8-wave kernel carries each
// K-tile's DMA issue (60-185 cycles per wave-instruction, MI355X_MICROARCH.md)
// in the MFMA waves' own instruction streams.
//
// Synchronisation: the pipe kernel's one raw s_barrier per K-tile, now over
// all WM*WN + NLW waves. Loaders: wait (counted vmcnt) until K-tile t landed,
// barrier, issue K-tile t + STAGES - 1 into the slot tile t - 1 used.
// Consumers: barrier, then the fragment reads and MFMAs of K-tile t (all of a
// consumer's reads of a slot have returned before it reaches the next
// barrier: each fragment feeds an MFMA of the same tile). Same LDS image,
// swizzle and epilogue (epilogue_direct16) as the pipe kernel, so results are
// bit for bit the pipe kernel's.
// PRIO: 0 none, 1 consumers at s_setprio 1 around their MFMAs, 2 loaders at
// s_setprio 1 (issue their DMA first).
// Not part of the library (tools/fwd_bench.hip -DFB_LW measures it).
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"

namespace fpnmt {

template <int BM, int BN, int WM, int WN, int AM, int NLW, int STAGES, int PRIO>
__global__ __launch_bounds__(64 * (WM * WN + NLW)) void gemm_lw_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int BK = 64, CPR = 8, ROWB = 128, MF = 16, KS = 32;
  constexpr int NC = 64 * WM * WN, NL = 64 * NLW;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / MF, TN = WTN / MF;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * CPR / NL, NB = BN * CPR / NL;  // DMA chunks per loader lane per stage
  static_assert(NA * NL == BM * CPR && NB * NL == BN * CPR, "loader lanes divide the tile's chunks");
  constexpr int PER = NA + NB;
  static_assert(STAGES >= 2 && (STAGES - 2) * PER < 64, "vmcnt range");
  static_assert(STAGES * STAGE_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = wave >= WM * WN;

  const int ntile = p.tiles_m * p.tiles_n;
  const int bid = xcd_remap(blockIdx.x, ntile);
  const int tmi = bid / p.tiles_n, tni = bid - tmi * p.tiles_n;
  const int M = p.M, N = p.N, K = p.K;
  const int m0 = tmi * BM, n0 = tni * BN;
  const T* __restrict__ Ag = (const T*)p.A;
  const T* __restrict__ Bg = (const T*)p.B;
  const T* zero = (const T*)p.zero16;
  const int nk = K / BK;
  typedef __attribute__((address_space(3))) void lds_void;

  if (loader) {
    const int lt = tid - NC, lw = wave - WM * WN;
    int a_off[NA];
    unsigned long long a_vm[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = i * NL + lt;
      const int row = q / CPR;
      const int kc = ((q % CPR) ^ pipe_sw<BK>(row)) * 8;
      const int m = m0 + row;
      if constexpr (AM == A_ROW) {
        a_off[i] = m * p.lda + kc;
        a_vm[i] = m < M ? 1ull : 0ull;
      } else {
        const uint32_t nimg = fdiv((uint32_t)min(m, M - 1), p.fd_HoWo);
        const int rem = min(m, M - 1) - (int)nimg * p.Ho * p.Wo;
        const uint32_t ho = fdiv((uint32_t)rem, p.fd_Wo);
        const int wo = rem - (int)ho * p.Wo;
        const int hi0 = (int)ho * p.sh - p.pt, wi0 = wo * p.sw - p.pl;
        a_off[i] = (((int)nimg * p.H + hi0) * p.W + wi0) * p.Cc + kc;
        unsigned long long vm = 0;
        if (m < M)
          for (int r = 0; r < p.Rk; ++r)
            for (int s2 = 0; s2 < p.Sk; ++s2)
              if (hi0 + r >= 0 && hi0 + r < p.H && wi0 + s2 >= 0 && wi0 + s2 < p.W) vm |= 1ull << (r * p.Sk + s2);
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
      const int k0 = kt * BK;
      int tap = 0, tap_off = k0;
      if constexpr (AM == A_IM2COL) {
        const uint32_t rs = fdiv((uint32_t)k0, p.fd_C);
        const int cb = k0 - (int)rs * p.Cc;
        const uint32_t r = fdiv(rs, p.fd_S);
        const int s2 = (int)rs - (int)r * p.Sk;
        tap = (int)rs;
        tap_off = ((int)r * p.W + s2) * p.Cc + cb;
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
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < STAGES - 1; ++i)
      if (i < nk) issue(i, i);
    for (int t = 0; t < nk; ++t) {
      const int ahead = min(nk - 1 - t, STAGES - 2);
      if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER>();
      else if (STAGES > 3 && ahead == 2) wait_vmcnt<(STAGES > 3 ? 2 : 0) * PER>();
      else if (ahead == 1) wait_vmcnt<PER>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // K-tile t visible to every consumer; slot (t-1) % STAGES free
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    }
    return;  // the consumers' epilogue has no barrier
  }

  const int wm = wave / WN, wn = wave % WN;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // residual rows straight into registers before the K loop: the consumer
  // waves issue no LDS-DMA, so these plain loads drain nothing
  bf16x4 rpre[TM][TN];
  const T* Rg = (const T*)p.R;
  if (Rg) prefetch_r_direct16<TM, TN>(p, Rg, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);
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
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ks & 1][b], fa[ks & 1][a], acc[a][b], 0, 0, 0);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    });
  }
  epilogue_direct16<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, (char*)p.C, 0, Rg != nullptr, rpre);
}

}  // namespace fpnmt
