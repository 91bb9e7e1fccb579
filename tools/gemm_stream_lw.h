// Streaming loader-wave kernel for the short-K 1x1 convs with a residual
// operand (round 6 negative result; see the note above launch_stream below).
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_dispatch.h"

namespace fpnmt {

// ---------------------------------------------------------------------------
// Streaming form for the short-K, HBM-bound GEMMs: the 1x1 stride-1 convs with
// K = 64 / 128 / 256 input channels (keras-resnet bottleneck 2c + shortcut,
// and the identity blocks' 2a bwd-data with the residual gradient R and the
// previous block's ReLU' mask M2), M = the pixel rows (round 6).
// The round-4 weight-stationary attempt (tools/gemm_stream.h) lost because
// each tile's stores and the next tile's loads serialised behind one
// vmcnt(0); here the roles are split by wave: NLW loader waves own every
// LDS-DMA (the block's resident B slice once, then per 32-row tile the A rows
// and the R / M2 rows into a STAGES-deep ring), 4 MFMA waves multiply and run
// the epilogue from LDS and issue only stores (their vmcnt never gates a load).
// Persistent blocks: block b owns the N-slice b % (N / BN) and walks its
// m-tiles; one raw s_barrier per tile over all waves (see gemm_pipe_lw_kernel).
// MFMA v_mfma_f32_16x16x32_bf16, K in 64-deep tiles in order: the K order of
// the MF 16 pipe kernels. LDS images: A / B [rows][64] per 64-column K-tile
// (pipe_sw swizzle), R / M2 [32][BN] with the 16-B chunk slot XOR (row & 15)
// (the epilogue's 16-row 8-B reads of one chunk hit 64 distinct banks).
template <int K, int BN, bool HAS_R, bool HAS_M2, int STAGES, int NLW, int BM = 32>
__global__ __launch_bounds__(64 * (4 + NLW)) void gemm_stream_lw_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int NC = 256, NL = 64 * NLW, MF = 16;
  static_assert(BM == 16 || BM == 32, "tile rows");
  constexpr int KT = K / 64;                          // 64-deep K-tiles
  constexpr int WTN = BN / 4, TM = BM / MF, TN = WTN / MF;
  static_assert(K % 64 == 0 && BN % 128 == 0 && TN % 2 == 0, "");
  constexpr int B_BYTES = BN * K * 2;                 // resident
  constexpr int A_BYTES = BM * K * 2, RB = BM * BN * 2;
  constexpr int SLOT = A_BYTES + (HAS_R ? RB : 0) + (HAS_M2 ? RB : 0);
  static_assert(B_BYTES + STAGES * SLOT <= 160 * 1024, "LDS");
  constexpr int CA = BM * 8 * KT, CR = BM * BN / 8;   // 16-B chunks per slot part
  constexpr int NA = CA / NL, NR = CR / NL, NBB = BN * 8 * KT / NL;
  static_assert(NA * NL == CA && NR * NL == CR && NBB * NL == BN * 8 * KT, "loader lanes divide the chunks");
  constexpr int PER = NA + (HAS_R ? NR : 0) + (HAS_M2 ? NR : 0);
  static_assert((STAGES - 2) * PER < 64, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) char smem[B_BYTES + STAGES * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = p.M, N = p.N;
  const int nch = N / BN;
  const int nc = (int)blockIdx.x % nch;
  const int n0 = nc * BN;
  const int tiles = (M + BM - 1) / BM;
  const int t_first = (int)blockIdx.x / nch, t_step = (int)gridDim.x / nch;
  const int my = t_first < tiles ? (tiles - t_first + t_step - 1) / t_step : 0;
  const T* __restrict__ Ag = (const T*)p.A;
  const T* __restrict__ Bg = (const T*)p.B;
  const T* __restrict__ Rg = (const T*)p.R;
  const T* __restrict__ M2g = (const T*)p.M2;
  const T* zero = (const T*)p.zero16;
  typedef __attribute__((address_space(3))) void lds_void;

  if (wave >= 4) {  // ---- loader waves ---------------------------------------
    const int lt = tid - NC, lw = wave - 4;
    // resident B slice: K-tile kt of row n at B_img + kt * BN * 128 + n * 128
#pragma unroll
    for (int i = 0; i < NBB; ++i) {
      const int q = i * NL + lt;
      const int kt = q / (BN * 8), r = q - kt * BN * 8;
      const int row = r / 8, kc = ((r % 8) ^ pipe_sw<64>(row)) * 8;
      const T* src = Bg + (long long)(n0 + row) * p.ldb + kt * 64 + kc;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(smem + (i * NL + lw * 64) * 16), 16, 0, 0);
    }
    auto issue = [&](int i, int slot) {
      const int m0 = (t_first + i * t_step) * BM;
      char* sb = smem + B_BYTES + slot * SLOT;
#pragma unroll
      for (int j = 0; j < NA; ++j) {  // A: K-tile kt of row r at kt * BM * 128 + r * 128
        const int q = j * NL + lt;
        const int kt = q / (BM * 8), r = q - kt * BM * 8;
        const int row = r / 8, kc = ((r % 8) ^ pipe_sw<64>(row)) * 8;
        const T* src = m0 + row < M ? Ag + (long long)(m0 + row) * p.lda + kt * 64 + kc : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (j * NL + lw * 64) * 16), 16, 0, 0);
      }
      if constexpr (HAS_R || HAS_M2) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const int q = j * NL + lt;
          const int row = q / (BN / 8), col = ((q % (BN / 8)) ^ (row & 15)) * 8;
          const long long off = (long long)(m0 + row) * p.ldr + n0 + col;
          const bool ok = m0 + row < M;
          if constexpr (HAS_R)
            __builtin_amdgcn_global_load_lds((const void*)(ok ? Rg + off : zero),
                                             (lds_void*)(sb + A_BYTES + (j * NL + lw * 64) * 16), 16, 0, 0);
          if constexpr (HAS_M2)
            __builtin_amdgcn_global_load_lds((const void*)(ok ? M2g + off : zero),
                                             (lds_void*)(sb + A_BYTES + (HAS_R ? RB : 0) + (j * NL + lw * 64) * 16),
                                             16, 0, 0);
        }
      }
    };
#pragma unroll
    for (int i = 0; i < STAGES - 1; ++i)
      if (i < my) issue(i, i);
    for (int i = 0; i < my; ++i) {
      const int ahead = min(my - 1 - i, STAGES - 2);
      if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER>();
      else if (STAGES > 3 && ahead == 2) wait_vmcnt<(STAGES > 3 ? 2 : 0) * PER>();
      else if (ahead == 1) wait_vmcnt<PER>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // tile i (and B) visible; slot (i - 1) % STAGES free
      if (i + STAGES - 1 < my) issue(i + STAGES - 1, (i + STAGES - 1) % STAGES);
    }
    return;
  }

  // ---- MFMA waves: rows 0..31 of the tile, columns wave * WTN .. + WTN ------
  const int frow = lane & 15, fchunk = lane >> 4, q4 = lane >> 4;
  const bool bias_vec = p.bias && ((uintptr_t)p.bias & 15) == 0;
  const bool scaled = p.alpha != 1.f || p.col_scale;
  const bool drop = p.drop_p > 0.f;
  const unsigned long long key = drop ? drop_key(p) : 0ull;
  const float dsc = drop ? 1.f / (1.f - p.drop_p) : 1.f;
  const int cw0 = wave * WTN;  // this wave's first column within the slice
  EpiCols ec[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) ec[b] = epi_cols(p, n0 + cw0 + 16 * b + 4 * q4, bias_vec, scaled);
  for (int i = 0; i < my; ++i) {
    __builtin_amdgcn_s_barrier();
    const int m0 = (t_first + i * t_step) * BM;
    const char* sb = smem + B_BYTES + (i % STAGES) * SLOT;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    static_for<0, KT * 2>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value, kt = ks / 2, kk = ks % 2;
      const int c = kk * 4 + fchunk;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int row = a * MF + frow;
        af[a] = *(const bf16x8*)(sb + kt * BM * 128 + row * 128 + ((c ^ pipe_sw<64>(row)) << 4));
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int row = cw0 + b * MF + frow;
        bfr[b] = *(const bf16x8*)(smem + kt * BN * 128 + row * 128 + ((c ^ pipe_sw<64>(row)) << 4));
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
    });
    // epilogue: lane holds rows a * 16 + (l & 15), columns 16 b + 4 (l >> 4) .. +3
    const char* Rs = sb + A_BYTES;
    const char* Ms = sb + A_BYTES + (HAS_R ? RB : 0);
    static_for<0, TN / 2>([&](auto pc) {
      constexpr int b0 = 2 * decltype(pc)::value;
      static_for<0, TM>([&](auto ac) {
        constexpr int a = decltype(ac)::value;
        const int rl = a * MF + frow;  // row within the tile
        const int row = m0 + rl;
        const int rowc = min(row, M - 1);
        float v0[4], v1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v0[j] = acc[a][b0][j];
          v1[j] = acc[a][b0 + 1][j];
        }
        const int cl0 = cw0 + b0 * 16 + 4 * q4, cl1 = cl0 + 16;  // columns within the slice
        auto lds4 = [&](const char* img, int cl) -> bf16x4 {
          return *(const bf16x4*)(img + rl * (BN * 2) + ((((cl >> 3) ^ (rl & 15)) << 4) | ((cl & 4) << 1)));
        };
        bf16x4 r0 = {}, r1 = {}, y0 = {}, y1 = {};
        if constexpr (HAS_R) { r0 = lds4(Rs, cl0); r1 = lds4(Rs, cl1); }
        if constexpr (HAS_M2) { y0 = lds4(Ms, cl0); y1 = lds4(Ms, cl1); }
        epi_values(p, v0, ec[b0], rowc, n0 + cl0, N, scaled, drop, key, dsc, HAS_R, r0, HAS_M2 ? &y0 : nullptr);
        epi_values(p, v1, ec[b0 + 1], rowc, n0 + cl1, N, scaled, drop, key, dsc, HAS_R, r1, HAS_M2 ? &y1 : nullptr);
        const bf16x4 o0 = {(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]};
        const bf16x4 o1 = {(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
        u32x2 x = __builtin_bit_cast(u32x2, o0), y = __builtin_bit_cast(u32x2, o1);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
        const u32x4 out = {s0[0], s1[0], s0[1], s1[1]};
        if (row < M)
          *(u32x4*)((bf16*)p.C + (long long)row * p.ldc + n0 + cw0 + b0 * 16 + 16 * (q4 & 1) + 8 * (q4 >> 1)) = out;
      });
    });
  }
}

// The short-K 1x1 convs with a residual operand R (the bottleneck 2c +
// shortcut forward, and the identity blocks' 2a bwd-data with the residual
// gradient, usually with the previous block's ReLU' mask M2) on the streaming
// loader-wave kernel (gemm_stream_lw_kernel): stride-1 1x1 (A = the pixel
// rows, lda = C), K = 64 / 128 / 256, plain bf16 store (no accumulate / split
// / batch / groups / scatter), N a multiple of the slice width.
// NEGATIVE (round 6, kept here, not in the library): tools/fwd_bench.hip
// -DFB_LW (profiles/r06/stream_1x1.txt, cold caches) at batch 32: the 2a
// bwd-data + R + M2 61.7 -> 55.8 us (res2), 38.4 -> 32.4 (res3), 26.7 -> 23.5
// (res4); 2c + R 44.3 -> 43.6, 29.8 -> 27.8, 21.8 -> 20.8; without R it lost
// (res2 shortcut 46.2 -> 66.0). In the C2 step (profiles/r06/stream_1x1_step.txt)
// the gain did not carry over: res2 class 43.2 -> 46.9 us per launch, res3
// 26.8 -> 27.1, res4 19.1 -> 20.3 (operands partly cache-resident there);
// C2 step 9.94 -> 9.97 ms, C3 15.7 -> 16.1 ms. Deeper rings (16-row tiles,
// 4-6 slots) and 4 loader waves measured equal: every form sits at ~3 TB/s.
static int stream_bn(int K) { return K == 64 ? 256 : 128; }
static bool stream_eligible(const GemmParams& p, int batch, int amode) {
  if (!p.R || batch != 1 || p.ngroups > 0 || p.accumulate != 0 || p.c_f32 || p.c_mode != C_ROW) return false;
  if (p.K != 64 && p.K != 128 && p.K != 256) return false;
  if (p.N % stream_bn(p.K) || p.M < 1024 || !g_split_ws.zero) return false;
  if (amode == A_IM2COL) {
    if (p.Rk != 1 || p.Sk != 1 || p.sh != 1 || p.sw != 1 || p.pt || p.pl || p.Cc != p.K || p.Ho != p.H || p.Wo != p.W)
      return false;
  } else if (amode != A_ROW || p.lda % 8) {
    return false;
  }
  if (p.ldb % 8 || p.ldc % 8 || ((p.R || p.M2) && p.ldr % 8)) return false;
  if (((uintptr_t)p.A | (uintptr_t)p.B | (uintptr_t)p.C | (uintptr_t)p.R | (uintptr_t)p.M2) & 15) return false;
  return true;
}

template <int K, bool HR, bool HM, int ST = 3, int NLW = 2, int BM = 32>
static int launch_stream_k(GemmParams& q, hipStream_t s) {
  constexpr int BN = K == 64 ? 256 : 128;
  const int nch = q.N / BN;
  const long long items = (long long)nch * cdiv(q.M, BM);
  long long grid = std::min<long long>(items, cu_count_dispatch());
  grid = std::max<long long>(nch, grid / nch * nch);
  hipLaunchKernelGGL((gemm_stream_lw_kernel<K, BN, HR, HM, ST, NLW, BM>), dim3((unsigned)grid), dim3(64 * (4 + NLW)), 0,
                     s, q);
  return check_launch("gemm_stream_lw_kernel");
}

template <int K>
static int launch_stream_hr(GemmParams& q, hipStream_t s) {
  if (q.R && q.M2) return launch_stream_k<K, true, true>(q, s);
  if (q.R) return launch_stream_k<K, true, false>(q, s);
  if (q.M2) return launch_stream_k<K, false, true>(q, s);
  return launch_stream_k<K, false, false>(q, s);
}

static int launch_stream(const GemmParams& p, int amode, hipStream_t s) {
  GemmParams q = p;
  if (amode == A_IM2COL) q.lda = p.Cc;
  q.zero16 = g_split_ws.zero;
  if (p.K == 64) return launch_stream_hr<64>(q, s);
  if (p.K == 128) return launch_stream_hr<128>(q, s);
  return launch_stream_hr<256>(q, s);
}

}  // namespace fpnmt
