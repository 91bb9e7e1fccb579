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
//     requires) with the 16-B chunk index XOR-swizzled by (row & 7) on the
//     SOURCE address, so the ds_read_b128 fragment reads are conflict-free;
//   * out-of-range rows / conv padding taps read a 16-B zero page;
//   * the shared staged row epilogue (bias, residual, act, dropout, 16-B stores).
#pragma once
#include "gemm_impl.h"

namespace fpnmt {

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  // gfx9 s_waitcnt encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14], expcnt[6:4]=7, lgkmcnt[11:8]=15
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int BM, int BN, int WM, int WN, int AM, int NT = 512>
__global__ __launch_bounds__(NT) void gemm_pipe_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int BK = 64, STAGES = 3;
  static_assert(WM * WN * 64 == NT, "one wave per 64 threads");
  static_assert(AM == A_ROW || AM == A_IM2COL, "k-contiguous A only");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * 8 / NT, NB = BN * 8 / NT;  // 16-B DMA chunks per thread per stage
  static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "");
  constexpr int EPI_BYTES = (NT / 64) * 32 * (WTN + 4) * 4;
  constexpr int SMEM = STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES;
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
  const int nk = K / BK;

  // ---- per-thread DMA sources (rows fixed across K-tiles) ---------------
  // chunk q = i*NT + tid lands at LDS byte q*16: row q>>3, slot q&7, holding
  // logical k-chunk (slot ^ (row & 7)).
  long long a_base[NA];
  int a_hi0[NA], a_wi0[NA], a_kc[NA];
  bool a_ok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int q = i * NT + tid;
    const int row = q >> 3;
    a_kc[i] = ((q & 7) ^ (row & 7)) * 8;
    const int m = m0 + row;
    a_ok[i] = m < M;
    if constexpr (AM == A_ROW) {
      a_base[i] = (long long)m * p.lda + a_kc[i];
      a_hi0[i] = a_wi0[i] = 0;
    } else {
      const uint32_t nimg = fdiv((uint32_t)m, gfdHoWo);
      const int rem = m - (int)nimg * gHo * gWo;
      const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
      const int wo = rem - (int)ho * gWo;
      a_base[i] = (long long)nimg * gH;  // first input row of this image
      a_hi0[i] = (int)ho * p.sh - p.pt;
      a_wi0[i] = wo * p.sw - p.pl;
    }
  }
  long long b_base[NB];
  bool b_ok[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    const int row = q >> 3;
    const int kc = ((q & 7) ^ (row & 7)) * 8;
    b_ok[i] = n0 + row < N;
    b_base[i] = (long long)(n0 + row) * p.ldb + kc;
  }

  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](int kt, int stage) {
    const int k0 = kt * BK;
    char* sb = smem + stage * STAGE_BYTES;
    if constexpr (AM == A_ROW) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const T* src = a_ok[i] ? Ag + a_base[i] + k0 : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (i * NT + wave * 64) * 16), 16, 0, 0);
      }
    } else {
      // the whole 64-deep K-tile sits in one filter tap (Cc % 64 == 0)
      const uint32_t rs = fdiv((uint32_t)k0, p.fd_C);
      const int cb = k0 - (int)rs * p.Cc;
      const uint32_t r = fdiv(rs, p.fd_S);
      const int s = (int)rs - (int)r * p.Sk;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int hi = a_hi0[i] + (int)r, wi = a_wi0[i] + s;
        const bool ok = a_ok[i] && hi >= 0 && hi < gH && wi >= 0 && wi < gW;
        const T* src = ok ? Ag + ((a_base[i] + hi) * gW + wi) * (long long)p.Cc + cb + a_kc[i] : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (i * NT + wave * 64) * 16), 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const T* src = b_ok[i] ? Bg + b_base[i] + k0 : zero;
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

  auto compute = [&](int stage) {
    const char* As = smem + stage * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks * 2 + lh;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int row = wm * WTM + t * 32 + lr;
        af[t] = *(const bf16x8*)(As + row * 128 + ((c ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int row = wn * WTN + t * 32 + lr;
        bfr[t] = *(const bf16x8*)(Bs + row * 128 + ((c ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
  };

  // ---- main loop: 3 stages, two K-tiles in flight across each barrier ----
  constexpr int PER_STAGE = NA + NB;  // DMA instructions per thread per stage
  if (nk > 0) issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) wait_vmcnt<PER_STAGE>();  // tile t landed (this thread's part)
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // ... everyone's part; stage (t+2)%3 is free (read in t-1)
    if (t + 2 < nk) issue(t + 2, (t + 2) % STAGES);
    compute(t % STAGES);
  }
  __syncthreads();  // all DMA retired (vmcnt 0 above) and all fragment reads done: reuse LDS

  char* Cg = (char*)Cp0;
  const long long c_off = zo * p.c_so + zi * p.c_si;
  const T* Rg = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  epilogue_rows<T, TM, TN, WTN>(p, acc, (float*)smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg,
                                true);
}

}  // namespace fpnmt
