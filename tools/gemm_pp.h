// ROUND-5 NEGATIVE RESULT (not in the library; tools/fwd_bench.hip -DFB_PP,
// profiles/r05/pp_bench_r5b.txt: C2 P3 3x3 65.0 us (32x32x16) / 56.7 us
// (16x16x32) against 54.5 for the shipped spread+prio tile).
// Ping-pong LDS-DMA MFMA GEMM for the wide k-contiguous problems (implicit-
// GEMM conv forward / stride-1 bwd-data, row-major Dense): the operand
// geometry, swizzle, im2col sources and epilogue of gemm_pipe_kernel
// (gemm_pipe.h), with a different schedule.
//
// Why: in gemm_pipe_kernel both waves of a SIMD issue their LDS-DMA and
// fragment reads in the same stretch and then their MFMAs in the same
// stretch (one barrier per K-tile keeps them in step), so the DMA issue cost
// (≈70-85 SIMD cycles per 1 KiB wave-instruction, MI355X_MICROARCH.md; 12 per
// SIMD per 128x256 K-tile) ADDS to the K-tile's 1024 MFMA cycles per SIMD
// (profiles/r04/lds_feed.txt: a synthetic K loop of this tile at 53 % of the
// MFMA pipe). Here the 8 waves form two groups of four, one wave of each
// group per SIMD (waves w and w+4 share a SIMD), and every K-tile is cut into
// two phases of two 16-deep k-steps; a phase is a READ segment (the phase's
// fragment reads + half of a later K-tile's DMA, then lgkmcnt(0)) and an
// MFMA segment (8 MFMAs at raised priority), each ended by a barrier. Group 1
// runs one barrier behind group 0, so on every SIMD one wave's MFMAs run
// while the other wave reads and issues DMA (cdna_hip_programming.md, "The
// 256^2 8-phase template": staggered wave groups).
//
// Hazards (3 LDS stages, K-tile t in stage t % 3; b(t,p,0/1) = the barriers
// ending group 0's READ / MFMA segment of phase p of K-tile t):
//   RAW  K-tile t+1 is waited for (counted vmcnt, its 6 DMA instructions per
//        thread) by group 0 in its MFMA segment (t,1) and by group 1 in its
//        READ segment (t,1), both before b(t,1,1); its first reads follow
//        b(t,1,1);
//   WAR  K-tile t+2 goes into stage (t-1) % 3, whose last reads (group 1's
//        READ segment (t-1,1)) were retired by that segment's lgkmcnt(0)
//        before b(t-1,1,1); the first DMA of t+2 is issued after it.
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"

namespace fpnmt {

__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int BM, int BN, int WM, int WN, int AM, int MF = 32>
__global__ __launch_bounds__(512) void gemm_pp_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int NT = 512, BK = 64, STAGES = 3;
  constexpr int CPR = BK / 8, ROWB = BK * 2;
  static_assert(WM * WN == 8, "two groups of four waves");
  static_assert(AM == A_ROW || AM == A_IM2COL, "k-contiguous A only");
  static_assert(MF == 32 || MF == 16, "MFMA shape: 32x32x16 or 16x16x32");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / MF, TN = WTN / MF;
  static_assert(TM >= 1 && TN >= 1, "");
  typedef typename std::conditional<MF == 32, f32x16, f32x4>::type accT;
  constexpr int NACC = MF == 32 ? 16 : 4;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * CPR / NT, NB = BN * CPR / NT;
  static_assert((BM * CPR) % NT == 0 && (BN * CPR) % NT == 0 && NA >= 1 && NB >= 1, "");
  constexpr int PER_STAGE = NA + NB;          // DMA instructions per thread per K-tile
  constexpr int HALF = PER_STAGE / 2;         // issued in phase 0; the rest in phase 1
  static_assert(STAGES * STAGE_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int grp = wave >> 2;
  const int wm = wave / WN, wn = wave % WN;
  const int lh = lane >> 5, lr = lane & 31;

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
  const T* zero = (const T*)p.zero16;
  const int nk = K / BK;

  // per-thread DMA sources (as gemm_pipe_kernel)
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
    ts.k0 = kt * BK;
    ts.tap = 0;
    ts.tap_off = ts.k0;
    if constexpr (AM == A_IM2COL) {
      const uint32_t rs = fdiv((uint32_t)ts.k0, p.fd_C);
      const int cb = ts.k0 - (int)rs * p.Cc;
      const uint32_t r = fdiv(rs, p.fd_S);
      const int s2 = (int)rs - (int)r * p.Sk;
      ts.tap = (int)rs;
      ts.tap_off = ((int)r * gW + s2) * p.Cc + cb;
    }
    return ts;
  };
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

  accT acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[a][b][i] = 0.f;

  // fragment reads of k-slice ks: 16 deep (32x32x16: lanes 32-63 the upper 8)
  // or 32 deep (16x16x32: lane l reads row l & 15, 8-element chunk l >> 4)
  const int frow = MF == 32 ? lr : (lane & 15);
  const int fchunk = MF == 32 ? lh : (lane >> 4);
  auto frag = [&](const char* As, const char* Bs, int ks, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
    const int c = ks * (MF == 32 ? 2 : 4) + fchunk;
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
  auto mfma = [&](const bf16x8 (&af)[TM], const bf16x8 (&bfr)[TN]) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        if constexpr (MF == 32)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
        else
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
      }
  };

  // residual / act-mask rows of the direct epilogue, in flight under the K loop
  typedef typename std::conditional<MF == 32, bf16x4[TM][TN][4], bf16x4[TM][TN]>::type rpreT;
  rpreT rpre;
  const T* Rg0 = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  if (Rg0) {
    if constexpr (MF == 32) prefetch_r_direct<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);
    else prefetch_r_direct16<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);
  }

  // ---- prologue: K-tiles 0 and 1 in flight, tile 0 landed -----------------
  if (nk > 0) issue_range(tile_src(0), 0, std::integral_constant<int, 0>{}, std::integral_constant<int, PER_STAGE>{});
  if (nk > 1) {
    issue_range(tile_src(1), 1, std::integral_constant<int, 0>{}, std::integral_constant<int, PER_STAGE>{});
    wait_vmcnt<PER_STAGE>();
  } else {
    wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (grp) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  for (int t = 0; t < nk; ++t) {
    const char* As = smem + (t % STAGES) * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
    const bool more = t + 2 < nk;
    const TileSrc ts2 = tile_src(t + 2);
    const int st2 = (t + 2) % STAGES;
    bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
    // ---- phase 0: READ (the DMA first: hipcc waits lgkmcnt(0) before each
    // M0 write of an LDS-DMA, which would serialise it behind the reads) ----
    if (more) issue_range(ts2, st2, std::integral_constant<int, 0>{}, std::integral_constant<int, HALF>{});
    if constexpr (MF == 32) {
      frag(As, Bs, 0, fa0, fb0);
      frag(As, Bs, 1, fa1, fb1);
    } else {
      frag(As, Bs, 0, fa0, fb0);
    }
    wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 0: MFMA ----
    __builtin_amdgcn_s_setprio(1);
    mfma(fa0, fb0);
    if constexpr (MF == 32) mfma(fa1, fb1);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 1: READ ----
    if (more) issue_range(ts2, st2, std::integral_constant<int, HALF>{}, std::integral_constant<int, PER_STAGE>{});
    if constexpr (MF == 32) {
      frag(As, Bs, 2, fa0, fb0);
      frag(As, Bs, 3, fa1, fb1);
    } else {
      frag(As, Bs, 1, fa1, fb1);
    }
    wait_lgkm0();
    if (grp) {  // K-tile t+1 landed (this thread's part) before the barrier that precedes its reads
      if (more) wait_vmcnt<PER_STAGE>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 1: MFMA ----
    __builtin_amdgcn_s_setprio(1);
    if constexpr (MF == 32) mfma(fa0, fb0);
    mfma(fa1, fb1);
    __builtin_amdgcn_s_setprio(0);
    if (!grp) {
      if (more) wait_vmcnt<PER_STAGE>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (!grp) __builtin_amdgcn_s_barrier();  // equal barrier counts in both groups

  char* Cg = (char*)Cp0;
  const long long c_off = zo * p.c_so + zi * p.c_si;
  if constexpr (MF == 32)
    epilogue_direct<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg0 != nullptr, rpre);
  else
    epilogue_direct16<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg0 != nullptr, rpre);
}

}  // namespace fpnmt
