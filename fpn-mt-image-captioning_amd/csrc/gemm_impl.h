// MFMA GEMM / implicit-GEMM convolution kernel family for gfx950.
//
// One kernel template covers every contraction on the hot path:
//   conv fwd        A = im2col(x) (k-contig),      B = w_ohwi        (k-contig)
//   conv bwd-data   A = im2col'(dz) or dz rows,    B = w_flip        (k-contig)
//   conv bwd-filter A = im2col(x)^T (m-contig),    B = dz            (n-contig)
//   Dense fwd/dgrad A = x rows,                    B = W^T / W       (k-contig)
//   Dense wgrad     A = x^T (m-contig),            B = dz            (n-contig)
//   attention       S = Q K^T, O = P V, dP, dQ, dK, dV (batched over b*h)
//
// LDS images: k-contiguous operands are stored [row][BK+pad] (80-byte rows,
// conflict-free ds_read_b128 fragment reads); m/n-contiguous operands are
// stored [k][rows+pad] straight from 16-byte global vectors and read as MFMA
// fragments with ds_read_b64_tr_b16 (bf16) — no transposing register pass.
// Tiles are 32x32 MFMA blocks (v_mfma_f32_32x32x16_bf16 / _32x32x2_f32),
// double-buffered LDS with register staging, one barrier per K-tile,
// XCD-aware block remap. Epilogue: alpha, per-column scale (frozen BN),
// bias, residual, ReLU/LeakyReLU, store / read-modify-write / fp32 atomics
// (split-K), optional stride-s scatter of output rows (1x1 strided dgrad).
#pragma once
#include "common.h"
#include <type_traits>

namespace fpnmt {

enum { A_ROW = 0, A_COL = 1, A_IM2COL = 2, A_IM2COL_T = 3 };
enum { B_NK = 0, B_KN = 1 };
enum { C_ROW = 0, C_SCATTER = 1 };

struct FastDiv {
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  if (d == 0) d = 1;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.s = l;
  f.m = (uint32_t)(((((uint64_t)1) << 32) * ((((uint64_t)1) << l) - d)) / d + 1);
  return f;
}
// exact for n < 2^31
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// Grouped launch: up to MAX_GROUPS independent problems sharing N and the
// filter geometry — the FPN levels pushed through ONE shared-weight conv.
// group_k == 0: groups split M (fwd / dgrad; per-group A, C, R; shared B);
// group_k == 1: groups split the reduction (wgrad; per-group A, B; shared C,
// fp32 atomics). `start` is the group's first m-tile / first split.
constexpr int MAX_GROUPS = 6;
struct GemmGroup {
  const void* A;
  const void* B;
  void* C;
  const void* R;
  int M, K, start;
  int H, W, Ho, Wo;
  FastDiv fd_HoWo, fd_Wo;
};

struct GemmParams {
  int M, N, K;
  const void* A;
  const void* B;
  void* C;
  const void* R;
  long long lda, ldb, ldc, ldr;
  int batch_inner;
  long long a_so, a_si, b_so, b_si, c_so, c_si, r_so, r_si;
  // implicit-GEMM geometry: input NHWC (., H, W, Cc); output grid (Ho, Wo)
  int H, W, Cc, Ho, Wo, Rk, Sk, sh, sw, pt, pl;
  FastDiv fd_HoWo, fd_Wo, fd_C, fd_S;
  // C_SCATTER: row m of grid (n, sHo, sWo) -> (n, ho*ss, wo*ss) of (Hd, Wd)
  int c_mode, scat_Hd, scat_Wd, scat_s;
  FastDiv fd_sHoWo, fd_sWo;
  // epilogue
  float alpha;
  const float* col_scale;
  const float* bias;
  int act;
  float act_alpha;
  int accumulate;  // 0 store, 1 RMW, 2 atomic
  int c_f32;
  // R operand role: 0 = residual added before the activation; FPNMT_ACT_RELU /
  // FPNMT_ACT_RELU6 = R is the activation output of the layer that produced
  // this GEMM's output grid (a bwd-data dx), and the result is multiplied by
  // that activation's 0/1 derivative (the producer's act_bwd, fused; C_ROW only)
  int r_mask;
  // optional second epilogue operand (bf16 pipe kernels; the dispatcher
  // applies it by a separate pass elsewhere): M2 is the activation output of
  // the layer that produced this GEMM's output grid (same ld / offsets as R),
  // and the result — after the residual add — is multiplied by that
  // activation's 0/1 derivative, m2_act (FPNMT_ACT_RELU / RELU6). With
  // accumulate 1 the mask multiplies this launch's contribution before the
  // add (or, on the separate pass, the sum: the same values when C already
  // carries the mask). C_SCATTER: M2 is indexed at the scattered C row.
  const void* M2;
  int m2_act;
  // grid
  int tiles_m, tiles_n, split_k, k_per_split;
  int ngroups, group_k;
  GemmGroup groups[MAX_GROUPS];
  // small-kernel split-K (deterministic): per-(tile, split) fp32 partial
  // tiles + per-tile arrival counters (zero between launches)
  float* ws_part;
  unsigned* ws_cnt;
  // gemm_kernel partial mode (split-K through the workspace): split y adds
  // y * c_split elements to C (0 otherwise)
  long long c_split;
  const void* zero16;  // >= 16 B of zeros in device memory (DMA source for padding)
  // fused dropout (see fpnmt_gemm_desc): out = R + dropout(act(...))
  float drop_p;
  unsigned long long drop_seed;
  const long long* drop_seed_dev;
  // weight gradients (B = dz rows): the bias gradient's column sums of B
  // folded into the launch. cs_db (host): db += sum over k of B[k][:]; a
  // launcher that folds them clears it (the caller runs the separate column
  // pass otherwise). cs_part (kernel): per-(split, m-tile, wave row) partial
  // rows of N floats, summed in row order into cs_db by colsum_launch.
  float* cs_db;
  float* cs_part;
};

__device__ __forceinline__ unsigned long long drop_key(const GemmParams& p) {
  return p.drop_seed + (p.drop_seed_dev ? (unsigned long long)(*p.drop_seed_dev) * 0x9E3779B97F4A7C15ull : 0ull);
}

// process-wide split-K workspace (fpnmt_set_workspace)
struct SplitWs {
  const void* zero;  // 256 B that stay zero
  float* part;
  unsigned* cnt;
  long long part_floats;
  int cnt_n;
};
extern SplitWs g_split_ws;

template <typename T> struct TT;
template <> struct TT<bf16> {
  static constexpr int VEC = 8;
  static constexpr int BK = 32;
  typedef bf16x8 Vec;
};
template <> struct TT<float> {
  static constexpr int VEC = 4;
  static constexpr int BK = 16;
  typedef f32x4 Vec;
};

typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  int q = nwg >> 3, r = nwg & 7;
  int xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Staged row epilogue shared by the GEMM kernels (accumulate != 2): see
// gemm_kernel. row0 / col0: first output row / column of this wave's tile.
//
// Each wave spills one 32-row slab of its accumulators to LDS (fp32), then
// re-reads it row-major so every lane applies the epilogue to 8 consecutive
// columns and issues 16-B row stores (the accumulator layout alone would
// store one element per lane per row). The residual rows (16-B bf16 loads)
// of EVERY slab are issued before the first staging barrier, so their
// latency overlaps the staging instead of serialising one dependent load per
// item (the 1x1 bottleneck convs are output/residual-stream bound).
template <typename T, int TM, int TN, int WTN>
__device__ __forceinline__ void epilogue_rows(const GemmParams& p, f32x16 (&acc)[TM][TN], float* stage_all,
                                              int wave, int lane, int row0, int col0, int M, int N, char* Cg,
                                              long long c_off, const T* Rg, bool first_split) {
  const int lr = lane & 31, lh = lane >> 5;
  constexpr int SLD = WTN + 4;
  constexpr int CPR = WTN / 8;
  constexpr int NIT = (32 * CPR + 63) / 64;  // items per lane per slab
  constexpr bool BF = sizeof(T) == 2;
  float* stage = stage_all + wave * (32 * SLD);
  const bool use_r = Rg && first_split;
  // residual prefetch (bf16, full 8-column items, 16-B aligned rows)
  bf16x8 rpre[TM][NIT];
  bool rok[TM][NIT];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = lane + 64 * it;
      const int r = e / CPR, cc = (e % CPR) * 8;
      const int row = row0 + a * 32 + r, col = col0 + cc;
      const T* rrow = Rg + (long long)row * p.ldr + col;
      rok[a][it] = BF && use_r && e < 32 * CPR && row < M && col + 8 <= N && ((uintptr_t)rrow & 15) == 0;
      if (rok[a][it]) rpre[a][it] = *(const bf16x8*)rrow;
    }
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) stage[((i & 3) + 8 * (i >> 2) + 4 * lh) * SLD + b * 32 + lr] = acc[a][b][i];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int e = lane + 64 * it;
      if (e >= 32 * CPR) break;
      const int r = e / CPR, cc = (e % CPR) * 8;
      const int row = row0 + a * 32 + r;
      const int col = col0 + cc;
      if (row >= M || col >= N) continue;
      float v[8];
      const f32x4 lo = *(const f32x4*)(stage + r * SLD + cc);
      const f32x4 hi = *(const f32x4*)(stage + r * SLD + cc + 4);
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
      long long orow = row;
      if (p.c_mode == C_SCATTER) {
        const uint32_t n = fdiv((uint32_t)row, p.fd_sHoWo);
        const int rem = row - (int)n * (int)p.fd_sHoWo.d;
        const uint32_t ho = fdiv((uint32_t)rem, p.fd_sWo);
        const int wo = rem - (int)ho * (int)p.fd_sWo.d;
        orow = ((long long)n * p.scat_Hd + (long long)ho * p.scat_s) * p.scat_Wd + (long long)wo * p.scat_s;
      }
      const long long idx = c_off + orow * p.ldc + col;
      const bool full = col + 8 <= N;
      if (full && p.alpha == 1.f && !p.col_scale) {
        if (p.bias && first_split && ((uintptr_t)(p.bias + col) & 15) == 0) {
          const f32x4 b0 = *(const f32x4*)(p.bias + col), b1 = *(const f32x4*)(p.bias + col + 4);
          v[0] += b0[0]; v[1] += b0[1]; v[2] += b0[2]; v[3] += b0[3];
          v[4] += b1[0]; v[5] += b1[1]; v[6] += b1[2]; v[7] += b1[3];
        } else if (p.bias && first_split) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += p.bias[col + j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (!full && col + j >= N) break;
          const float cs = p.col_scale ? p.col_scale[col + j] : 1.f;
          const float bi = (p.bias && first_split) ? p.bias[col + j] : 0.f;
          v[j] = v[j] * p.alpha * cs + bi;
        }
      }
      if (p.drop_p > 0.f) {  // R + dropout(act(v)): residual after the mask
        const unsigned long long key = drop_key(p);
        const float sc = 1.f / (1.f - p.drop_p);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a_ = act_apply(v[j], p.act, p.act_alpha);
          v[j] = uniform01(key, (uint64_t)row * (uint64_t)N + (uint64_t)(col + j)) >= p.drop_p ? a_ * sc : 0.f;
        }
      }
      float rv[8];
      if (use_r) {
        if (rok[a][it]) {
#pragma unroll
          for (int j = 0; j < 8; ++j) rv[j] = (float)rpre[a][it][j];
        } else {
          const T* rrow = Rg + (long long)row * p.ldr + col;
#pragma unroll
          for (int j = 0; j < 8; ++j) rv[j] = (full || col + j < N) ? to_f32(rrow[j]) : 0.f;
        }
        if (!p.r_mask) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += rv[j];
        }
      }
      if (!(p.drop_p > 0.f)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = act_apply(v[j], p.act, p.act_alpha);
      }
      if (use_r && p.r_mask) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= act_mask_from_y(rv[j], p.r_mask, p.act_alpha);
      }
      if (p.M2) {
        const T* yr = (const T*)p.M2 + orow * p.ldr + col;  // C's layout (scattered rows too)
        if (BF && full && ((uintptr_t)yr & 15) == 0) {  // one 16-B load (8 two-byte loads were
          const bf16x8 yv = *(const bf16x8*)yr;           // an identity block's 2a bwd-data tail)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= act_mask_from_y((float)yv[j], p.m2_act);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (full || col + j < N) v[j] *= act_mask_from_y(to_f32(yr[j]), p.m2_act);
        }
      }
      if (p.c_f32) {
        float* Cp = (float*)Cg + idx;
        if (full && ((uintptr_t)Cp & 15) == 0) {
          f32x4 o0 = {v[0], v[1], v[2], v[3]}, o1 = {v[4], v[5], v[6], v[7]};
          if (p.accumulate == 1) {
            o0 += *(const f32x4*)Cp;
            o1 += *(const f32x4*)(Cp + 4);
          }
          *(f32x4*)Cp = o0;
          *(f32x4*)(Cp + 4) = o1;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (full || col + j < N) Cp[j] = p.accumulate == 1 ? Cp[j] + v[j] : v[j];
        }
      } else {
        T* Cp = (T*)Cg + idx;
        if (full && ((uintptr_t)Cp & 15) == 0 && BF) {
          bf16x8 o;
          if (p.accumulate == 1) {
            const bf16x8 old = *(const bf16x8*)Cp;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (bf16)(v[j] + (float)old[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
          }
          *(bf16x8*)Cp = o;
        } else if (full && ((uintptr_t)Cp & 15) == 0) {
          f32x4 o0 = {v[0], v[1], v[2], v[3]}, o1 = {v[4], v[5], v[6], v[7]};
          if (p.accumulate == 1) {
            o0 += *(const f32x4*)Cp;
            o1 += *(const f32x4*)(Cp + 4);
          }
          *(f32x4*)Cp = o0;
          *(f32x4*)(Cp + 4) = o1;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (full || col + j < N) Cp[j] = from_f32<T>(p.accumulate == 1 ? to_f32(Cp[j]) + v[j] : v[j]);
        }
      }
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN, int AM, int BMODE, bool VEC, int BKT = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(const GemmParams p) {
  constexpr int NT = 64 * WM * WN;
  constexpr int V = TT<T>::VEC;
  constexpr int BK = BKT ? BKT : TT<T>::BK;
  typedef typename TT<T>::Vec VecT;
  constexpr bool A_KC = (AM == A_ROW || AM == A_IM2COL);
  constexpr bool B_KC = (BMODE == B_NK);
  constexpr int KS = BK + 16 / (int)sizeof(T);    // k-contig LDS row stride (elements)
  constexpr int AMS = BM + 64 / (int)sizeof(T);   // m-contig LDS row stride
  constexpr int BNS = BN + 64 / (int)sizeof(T);
  constexpr int A_ELEMS = A_KC ? BM * KS : BK * AMS;
  constexpr int B_ELEMS = B_KC ? BN * KS : BK * BNS;
  constexpr int NVA = (BM * BK / V + NT - 1) / NT;  // vectors per thread
  constexpr int NVB = (BN * BK / V + NT - 1) / NT;
  constexpr int WTM = BM / WM, WTN = BN / WN;        // wave tile
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  static_assert(NT % (BK / V) == 0, "");

  // one LDS array (staging double buffer, reused by the epilogue's fp32 slabs)
  constexpr int MAIN_BYTES = 2 * (A_ELEMS + B_ELEMS) * (int)sizeof(T);
  constexpr int EPI_BYTES = (NT / 64) * 32 * (WTN + 4) * 4;
  constexpr int SMEM_ELEMS = (MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES) / (int)sizeof(T);
  __shared__ __attribute__((aligned(16))) T smem[SMEM_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  const int ntile = p.tiles_m * p.tiles_n;
  const int bid = xcd_remap(blockIdx.x, ntile);
  int tmi = bid / p.tiles_n;
  const int tni = bid - tmi * p.tiles_n;
  int split = blockIdx.y;
  // problem of this block (a group of a grouped launch, or the one problem)
  const void* Ap = p.A;
  const void* Bp = p.B;
  void* Cp0 = p.C;
  const void* Rp = p.R;
  int M = p.M, K = p.K;
  int gH = p.H, gW = p.W, gHo = p.Ho, gWo = p.Wo;
  FastDiv gfdHoWo = p.fd_HoWo, gfdWo = p.fd_Wo;
  if (p.ngroups > 0) {
    const int key = p.group_k ? split : tmi;
    // static indices only (a dynamic index into the kernarg struct makes
    // the compiler copy the whole struct to scratch)
    GemmGroup G = p.groups[0];
#pragma unroll
    for (int q = 1; q < MAX_GROUPS; ++q)
      if (q < p.ngroups && key >= p.groups[q].start) G = p.groups[q];
    if (p.group_k) split -= G.start;
    else tmi -= G.start;
    Ap = G.A; Bp = G.B; Cp0 = G.C; Rp = G.R;
    M = G.M; K = G.K;
    gH = G.H; gW = G.W; gHo = G.Ho; gWo = G.Wo;
    gfdHoWo = G.fd_HoWo; gfdWo = G.fd_Wo;
  }
  const int N = p.N;
  const int m0 = tmi * BM, n0 = tni * BN;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const T* __restrict__ Ag = (const T*)Ap + zo * p.a_so + zi * p.a_si;
  const T* __restrict__ Bg = (const T*)Bp + zo * p.b_so + zi * p.b_si;
  const int kbeg = split * p.k_per_split;
  const int kend = min(K, kbeg + p.k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // ---- loop-invariant loader state ------------------------------------
  // k-contig A: rows fixed per vector, k offset fixed per thread
  int a_row[NVA];
  int a_pix[NVA], a_hi0[NVA], a_wi0[NVA];  // im2col (fwd)
  int a_fr = 0, a_fs = 0, a_fc = 0;        // im2col_T: fixed feature of this thread
  bool a_fok = false;
#pragma unroll
  for (int i = 0; i < NVA; ++i) {
    const int v = tid + i * NT;
    if constexpr (A_KC) {
      a_row[i] = v / (BK / V);
      if constexpr (AM == A_IM2COL) {
        const int m = m0 + a_row[i];
        const uint32_t n = fdiv((uint32_t)m, gfdHoWo);
        const int rem = m - (int)n * gHo * gWo;
        const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
        const int wo = rem - (int)ho * gWo;
        a_pix[i] = (m < M) ? (int)n * gH : -0x40000000;
        a_hi0[i] = (int)ho * p.sh - p.pt;
        a_wi0[i] = wo * p.sw - p.pl;
      }
    } else {
      a_row[i] = v / (BM / V);  // k row within tile
      if constexpr (AM == A_IM2COL_T) {
        if (i == 0) {
          const int f = m0 + (v % (BM / V)) * V;
          a_fok = f < M;
          const uint32_t rs = fdiv((uint32_t)f, p.fd_C);
          a_fc = f - (int)rs * p.Cc;
          const uint32_t r = fdiv(rs, p.fd_S);
          a_fs = (int)rs - (int)r * p.Sk;
          a_fr = (int)r;
        }
      }
    }
  }

  VecT ra[NVA], rb[NVB];

  // VEC loaders are branch-free: every 16-B vector is either wholly in range
  // or wholly out (the host only picks VEC when the vector extent divides the
  // contiguous dimension), is loaded unconditionally from a clamped in-bounds
  // address, and out-of-range vectors are zeroed with a bit mask afterwards.
  // A branch around a load (or a per-element "load or zero" fallback) made
  // hipcc wait vmcnt(0) behind every load and serialised the K loop on memory
  // latency; the scalar fallbacks below are compiled only for VEC = false.
  // The mask is applied in store_tiles (after compute), not here: masking
  // right after the load would make the K loop wait for the next tile's
  // loads before computing the current one.
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
  unsigned amk[NVA], bmk[NVB];
  auto vmask = [](VecT v, unsigned mk) -> VecT {
    return __builtin_bit_cast(VecT, __builtin_bit_cast(u32x4_t, v) & mk);
  };

  auto load_tiles = [&](int k0) {
    if constexpr (VEC) {
      // ---------------- A ----------------
      if constexpr (AM == A_ROW) {
        const int k = k0 + (tid % (BK / V)) * V;
#pragma unroll
        for (int i = 0; i < NVA; ++i) {
          const int m = m0 + a_row[i];
          const bool ok = m < M && k < K;
          ra[i] = *(const VecT*)(Ag + (ok ? (long long)m * p.lda + k : 0));
          amk[i] = ok ? ~0u : 0u;
        }
      } else if constexpr (AM == A_IM2COL) {
        const int k = k0 + (tid % (BK / V)) * V;
        const uint32_t rs = fdiv((uint32_t)k, p.fd_C);
        const int c = k - (int)rs * p.Cc;
        const uint32_t r = fdiv(rs, p.fd_S);
        const int s = (int)rs - (int)r * p.Sk;
#pragma unroll
        for (int i = 0; i < NVA; ++i) {
          const int hi = a_hi0[i] + (int)r, wi = a_wi0[i] + s;
          const bool ok = k < K && a_pix[i] >= 0 && hi >= 0 && hi < gH && wi >= 0 && wi < gW;
          const long long off = ok ? ((long long)(a_pix[i] + hi) * gW + wi) * p.Cc + c : 0;
          ra[i] = *(const VecT*)(Ag + off);
          amk[i] = ok ? ~0u : 0u;
        }
      } else if constexpr (AM == A_COL) {
        const int m = m0 + (tid % (BM / V)) * V;
#pragma unroll
        for (int i = 0; i < NVA; ++i) {
          const int k = k0 + a_row[i];
          const bool ok = k < K && m < M;
          ra[i] = *(const VecT*)(Ag + (ok ? (long long)k * p.lda + m : 0));
          amk[i] = ok ? ~0u : 0u;
        }
      } else {  // A_IM2COL_T
#pragma unroll
        for (int i = 0; i < NVA; ++i) {
          const int k = k0 + a_row[i];
          const uint32_t n = fdiv((uint32_t)k, gfdHoWo);
          const int rem = k - (int)n * gHo * gWo;
          const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
          const int wo = rem - (int)ho * gWo;
          const int hi = (int)ho * p.sh - p.pt + a_fr, wi = wo * p.sw - p.pl + a_fs;
          const bool ok = a_fok && k < K && hi >= 0 && hi < gH && wi >= 0 && wi < gW;
          const long long off = ok ? ((long long)((int)n * gH + hi) * gW + wi) * p.Cc + a_fc : 0;
          ra[i] = *(const VecT*)(Ag + off);
          amk[i] = ok ? ~0u : 0u;
        }
      }
      // ---------------- B ----------------
      if constexpr (BMODE == B_NK) {
        const int k = k0 + (tid % (BK / V)) * V;
#pragma unroll
        for (int i = 0; i < NVB; ++i) {
          const int n = n0 + (tid + i * NT) / (BK / V);
          const bool ok = n < N && k < K;
          rb[i] = *(const VecT*)(Bg + (ok ? (long long)n * p.ldb + k : 0));
          bmk[i] = ok ? ~0u : 0u;
        }
      } else {
        const int n = n0 + (tid % (BN / V)) * V;
#pragma unroll
        for (int i = 0; i < NVB; ++i) {
          const int k = k0 + (tid + i * NT) / (BN / V);
          const bool ok = k < K && n < N;
          rb[i] = *(const VecT*)(Bg + (ok ? (long long)k * p.ldb + n : 0));
          bmk[i] = ok ? ~0u : 0u;
        }
      }
      return;
    }
    // ---------------- A ----------------
    if constexpr (AM == A_ROW) {
      const int kv = (tid % (BK / V)) * V;
      const int k = k0 + kv;
#pragma unroll
      for (int i = 0; i < NVA; ++i) {
        const int m = m0 + a_row[i];
        VecT r;
        if (VEC && m < M && k + V <= K) {
          r = *(const VecT*)(Ag + (long long)m * p.lda + k);
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j)
            r[j] = (m < M && k + j < K) ? Ag[(long long)m * p.lda + k + j] : (T)0.f;
        }
        if (tid + i * NT < BM * BK / V) ra[i] = r;
      }
    } else if constexpr (AM == A_IM2COL) {
      const int kv = (tid % (BK / V)) * V;
      const int k = k0 + kv;
      if constexpr (VEC) {
        const uint32_t rs = fdiv((uint32_t)k, p.fd_C);
        const int c = k - (int)rs * p.Cc;
        const uint32_t r = fdiv(rs, p.fd_S);
        const int s = (int)rs - (int)r * p.Sk;
#pragma unroll
        for (int i = 0; i < NVA; ++i) {
          const int hi = a_hi0[i] + (int)r, wi = a_wi0[i] + s;
          VecT val;
          if (k < K && a_pix[i] >= 0 && hi >= 0 && hi < gH && wi >= 0 && wi < gW) {
            val = *(const VecT*)(Ag + ((long long)(a_pix[i] + hi) * gW + wi) * p.Cc + c);
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) val[j] = (T)0.f;
          }
          if (tid + i * NT < BM * BK / V) ra[i] = val;
        }
      } else {
#pragma unroll
        for (int i = 0; i < NVA; ++i) {
          VecT val;
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const int kk = k + j;
            T e = (T)0.f;
            if (kk < K && a_pix[i] >= 0) {
              const uint32_t rs = fdiv((uint32_t)kk, p.fd_C);
              const int c = kk - (int)rs * p.Cc;
              const uint32_t r = fdiv(rs, p.fd_S);
              const int s = (int)rs - (int)r * p.Sk;
              const int hi = a_hi0[i] + (int)r, wi = a_wi0[i] + s;
              if (hi >= 0 && hi < gH && wi >= 0 && wi < gW)
                e = Ag[((long long)(a_pix[i] + hi) * gW + wi) * p.Cc + c];
            }
            val[j] = e;
          }
          if (tid + i * NT < BM * BK / V) ra[i] = val;
        }
      }
    } else if constexpr (AM == A_COL) {
      const int mv = (tid % (BM / V)) * V;
      const int m = m0 + mv;
#pragma unroll
      for (int i = 0; i < NVA; ++i) {
        const int k = k0 + a_row[i];
        VecT r;
        if (VEC && k < K && m + V <= M) {
          r = *(const VecT*)(Ag + (long long)k * p.lda + m);
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j)
            r[j] = (k < K && m + j < M) ? Ag[(long long)k * p.lda + m + j] : (T)0.f;
        }
        if (tid + i * NT < BM * BK / V) ra[i] = r;
      }
    } else {  // A_IM2COL_T: element (feature m, pixel k)
#pragma unroll
      for (int i = 0; i < NVA; ++i) {
        const int k = k0 + a_row[i];
        VecT val;
        const uint32_t n = fdiv((uint32_t)k, gfdHoWo);
        const int rem = k - (int)n * gHo * gWo;
        const uint32_t ho = fdiv((uint32_t)rem, gfdWo);
        const int wo = rem - (int)ho * gWo;
        if constexpr (VEC) {
          const int hi = (int)ho * p.sh - p.pt + a_fr, wi = wo * p.sw - p.pl + a_fs;
          if (a_fok && k < K && hi >= 0 && hi < gH && wi >= 0 && wi < gW) {
            val = *(const VecT*)(Ag + ((long long)((int)n * gH + hi) * gW + wi) * p.Cc + a_fc);
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) val[j] = (T)0.f;
          }
        } else {
          const int f0 = m0 + (tid % (BM / V)) * V;
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const int f = f0 + j;
            T e = (T)0.f;
            if (f < M && k < K) {
              const uint32_t rs = fdiv((uint32_t)f, p.fd_C);
              const int c = f - (int)rs * p.Cc;
              const uint32_t r = fdiv(rs, p.fd_S);
              const int s = (int)rs - (int)r * p.Sk;
              const int hi = (int)ho * p.sh - p.pt + (int)r, wi = wo * p.sw - p.pl + s;
              if (hi >= 0 && hi < gH && wi >= 0 && wi < gW)
                e = Ag[((long long)((int)n * gH + hi) * gW + wi) * p.Cc + c];
            }
            val[j] = e;
          }
        }
        if (tid + i * NT < BM * BK / V) ra[i] = val;
      }
    }
    // ---------------- B ----------------
    if constexpr (BMODE == B_NK) {
      const int kv = (tid % (BK / V)) * V;
      const int k = k0 + kv;
#pragma unroll
      for (int i = 0; i < NVB; ++i) {
        const int row = (tid + i * NT) / (BK / V);
        const int n = n0 + row;
        VecT r;
        if (VEC && n < N && k + V <= K) {
          r = *(const VecT*)(Bg + (long long)n * p.ldb + k);
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j)
            r[j] = (n < N && k + j < K) ? Bg[(long long)n * p.ldb + k + j] : (T)0.f;
        }
        if (tid + i * NT < BN * BK / V) rb[i] = r;
      }
    } else {
      const int nv = (tid % (BN / V)) * V;
      const int n = n0 + nv;
#pragma unroll
      for (int i = 0; i < NVB; ++i) {
        const int k = k0 + (tid + i * NT) / (BN / V);
        VecT r;
        if (VEC && k < K && n + V <= N) {
          r = *(const VecT*)(Bg + (long long)k * p.ldb + n);
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j)
            r[j] = (k < K && n + j < N) ? Bg[(long long)k * p.ldb + n + j] : (T)0.f;
        }
        if (tid + i * NT < BN * BK / V) rb[i] = r;
      }
    }
  };

  auto store_tiles = [&](int buf) {
    T* As = smem + buf * (A_ELEMS + B_ELEMS);
    T* Bs = As + A_ELEMS;
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < NVA; ++i) ra[i] = vmask(ra[i], amk[i]);
#pragma unroll
      for (int i = 0; i < NVB; ++i) rb[i] = vmask(rb[i], bmk[i]);
    }
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int v = tid + i * NT;
      if (v < BM * BK / V) {
        if constexpr (A_KC) {
          *(VecT*)(As + (v / (BK / V)) * KS + (v % (BK / V)) * V) = ra[i];
        } else {
          *(VecT*)(As + (v / (BM / V)) * AMS + (v % (BM / V)) * V) = ra[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int v = tid + i * NT;
      if (v < BN * BK / V) {
        if constexpr (B_KC) {
          *(VecT*)(Bs + (v / (BK / V)) * KS + (v % (BK / V)) * V) = rb[i];
        } else {
          *(VecT*)(Bs + (v / (BN / V)) * BNS + (v % (BN / V)) * V) = rb[i];
        }
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  // fragment readers ------------------------------------------------------
  const int g16 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;

  auto compute = [&](int buf) {
    const T* As = smem + buf * (A_ELEMS + B_ELEMS);
    const T* Bs = As + A_ELEMS;
    if constexpr (std::is_same<T, bf16>::value) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          const int rb0 = wm * WTM + t * 32;
          if constexpr (A_KC) {
            af[t] = *(const bf16x8*)(As + (rb0 + lr) * KS + ks * 16 + 8 * lh);
          } else {
            const T* base = As + (ks * 16 + 8 * lh + tq) * AMS + rb0 + 16 * g16 + 4 * tp;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(base));
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(base + 4 * AMS));
            __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3],
                                                            hi[0], hi[1], hi[2], hi[3]};
            af[t] = __builtin_bit_cast(bf16x8, w8);
          }
        }
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          const int cb0 = wn * WTN + t * 32;
          if constexpr (B_KC) {
            bfr[t] = *(const bf16x8*)(Bs + (cb0 + lr) * KS + ks * 16 + 8 * lh);
          } else {
            const T* base = Bs + (ks * 16 + 8 * lh + tq) * BNS + cb0 + 16 * g16 + 4 * tp;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(base));
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(base + 4 * BNS));
            __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3],
                                                            hi[0], hi[1], hi[2], hi[3]};
            bfr[t] = __builtin_bit_cast(bf16x8, w8);
          }
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
      }
    } else {
      // f32: one 16-deep chunk per tile; lane (r,h) supplies k = 8h + j
      float af[TM][8], bfr[TN][8];
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int rb0 = wm * WTM + t * 32;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          af[t][j] = A_KC ? As[(rb0 + lr) * KS + 8 * lh + j] : As[(8 * lh + j) * AMS + rb0 + lr];
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int cb0 = wn * WTN + t * 32;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          bfr[t][j] = B_KC ? Bs[(cb0 + lr) * KS + 8 * lh + j] : Bs[(8 * lh + j) * BNS + cb0 + lr];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][j], bfr[b][j], acc[a][b], 0, 0, 0);
    }
  };

  // ---- main loop: register-staged double buffer, one barrier per tile ----
  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const bool more = (t + 1) < nk;
      if (more) load_tiles(kbeg + (t + 1) * BK);
      compute(t & 1);
      if (more) store_tiles((t + 1) & 1);
      __syncthreads();
    }
  } else if (split > 0 && p.c_split == 0) {
    return;  // empty split: nothing to add (a partial slab is still written: zeros)
  }

  // ---- epilogue --------------------------------------------------------
  char* Cg = (char*)Cp0;
  // partial-slab mode: slab index = the launch's split (blockIdx.y), also in
  // k-grouped launches where `split` was made local to the group
  const long long c_off = zo * p.c_so + zi * p.c_si + (long long)blockIdx.y * p.c_split;
  const T* Rg = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  const bool first_split = split == 0;
  if (p.accumulate != 2) {
    epilogue_rows<T, TM, TN, WTN>(p, acc, (float*)smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off,
                                  Rg, first_split);
    return;
  }
  // fp32 atomic accumulation (split-K / shared-weight gradients): one
  // atomic per element straight from the accumulator layout (two 128-B row
  // segments per wave instruction: the full-rate atomic shape on gfx950)
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = n0 + wn * WTN + b * 32 + lr;
      if (col >= N) continue;
      const float cs = p.col_scale ? p.col_scale[col] : 1.f;
      const float bi = (p.bias && first_split) ? p.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = m0 + wm * WTM + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * lh;
        if (row >= M) continue;
        float v = acc[a][b][i] * p.alpha * cs + bi;
        const float rv = (Rg && first_split) ? to_f32(Rg[(long long)row * p.ldr + col]) : 0.f;
        if (!p.r_mask) v += rv;
        v = act_apply(v, p.act, p.act_alpha);
        if (Rg && first_split && p.r_mask) v *= act_mask_from_y(rv, p.r_mask, p.act_alpha);
        long long orow = row;
        if (p.c_mode == C_SCATTER) {
          const uint32_t n = fdiv((uint32_t)row, p.fd_sHoWo);
          const int rem = row - (int)n * (int)p.fd_sHoWo.d;
          const uint32_t ho = fdiv((uint32_t)rem, p.fd_sWo);
          const int wo = rem - (int)ho * (int)p.fd_sWo.d;
          orow = ((long long)n * p.scat_Hd + (long long)ho * p.scat_s) * p.scat_Wd + (long long)wo * p.scat_s;
        }
        const long long idx = c_off + orow * p.ldc + col;
        if (p.c_f32) {
          float* Cp = (float*)Cg + idx;
          if (p.accumulate == 2) atomicAdd(Cp, v);
          else if (p.accumulate == 1) *Cp = *Cp + v;
          else *Cp = v;
        } else {
          T* Cp = (T*)Cg + idx;
          if (p.accumulate == 1) v += to_f32(*Cp);
          *Cp = from_f32<T>(v);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Small-M GEMM (few output tiles, both operands k-contiguous: A_ROW x B_NK):
// latency-bound for the tiled kernel (one wave walking K serially through
// LDS). Here MFMA fragments are loaded straight from global memory (16 B per
// lane, a register double buffer of U k-steps in flight), K is split over the
// block's KW waves and the partial 32x64 tiles are summed through LDS. No LDS
// staging of operands, no barriers in the K loop.
// Cross-block split-K (gridDim.y = S > 1): every block stores its reduced
// partial tile (fp32, accumulator order) to the process workspace with plain
// stores and gemm_small_reduce_kernel sums the S partials in split order and
// runs the epilogue: the kernel boundary is the publish. (An in-launch
// last-arriver combine needs an agent-scope release per block, i.e. an L2
// writeback per block on the 8-XCD part: measured ~28 us per split level at
// M = 992.)
constexpr int SMALL_TN = 2;
constexpr int SMALL_TILE_FLOATS = SMALL_TN * 16 * 64;

// epilogue of one output element (small kernel and the split-K reduces), with
// explicit output / residual bases (a group's, in grouped launches)
template <typename T>
__device__ __forceinline__ void small_epilogue_at(const GemmParams& p, float v, int row, int col, void* Cbase,
                                                  const void* Rbase, long long zo, long long zi) {
  const float cs = p.col_scale ? p.col_scale[col] : 1.f;
  const float bi = p.bias ? p.bias[col] : 0.f;
  const T* Rg = Rbase ? (const T*)Rbase + zo * p.r_so + zi * p.r_si : nullptr;
  v = v * p.alpha * cs + bi;
  if (p.drop_p > 0.f) {
    v = act_apply(v, p.act, p.act_alpha);
    v = uniform01(drop_key(p), (uint64_t)row * (uint64_t)p.N + (uint64_t)col) >= p.drop_p ? v / (1.f - p.drop_p) : 0.f;
    if (Rg) v += to_f32(Rg[(long long)row * p.ldr + col]);
  } else if (Rg && p.r_mask) {
    v = act_apply(v, p.act, p.act_alpha) * act_mask_from_y(to_f32(Rg[(long long)row * p.ldr + col]), p.r_mask, p.act_alpha);
  } else {
    if (Rg) v += to_f32(Rg[(long long)row * p.ldr + col]);
    v = act_apply(v, p.act, p.act_alpha);
  }
  const long long idx = zo * p.c_so + zi * p.c_si + (long long)row * p.ldc + col;
  if (p.c_f32) {
    float* Cp = (float*)Cbase + idx;
    if (p.accumulate == 2) atomicAdd(Cp, v);
    else if (p.accumulate == 1) *Cp = *Cp + v;
    else *Cp = v;
  } else {
    T* Cp = (T*)Cbase + idx;
    if (p.accumulate == 1) v += to_f32(*Cp);
    *Cp = from_f32<T>(v);
  }
}
template <typename T>
__device__ __forceinline__ void small_epilogue(const GemmParams& p, float v, int row, int col, long long zo,
                                               long long zi) {
  small_epilogue_at<T>(p, v, row, col, p.C, p.R, zo, zi);
}

// NE elements per thread: every global read of the epilogue (scale, bias,
// residual, the old C of a read-modify-write) is issued for all NE elements
// before the first store. Element by element, each store could alias the next
// element's residual / bias and the compiler serialised the reads behind it:
// one memory latency per element (~8 of the ~10 us of an M = 32 GEMM).
template <typename T, int NE>
__device__ __forceinline__ void small_epilogue_n(const GemmParams& p, const float (&v)[NE], const int (&row)[NE],
                                                 const int (&col)[NE], const bool (&ok)[NE], void* Cb,
                                                 const void* Rb, long long zo, long long zi) {
  const T* Rg = Rb ? (const T*)Rb + zo * p.r_so + zi * p.r_si : nullptr;
  const long long cbase = zo * p.c_so + zi * p.c_si;
  float cs[NE], bi[NE], rv[NE], old[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int c = ok[e] ? col[e] : 0;
    const long long rr = ok[e] ? (long long)row[e] : 0;
    cs[e] = p.col_scale ? p.col_scale[c] : 1.f;
    bi[e] = p.bias ? p.bias[c] : 0.f;
    rv[e] = Rg ? to_f32(Rg[rr * p.ldr + c]) : 0.f;
    old[e] = 0.f;
    if (p.accumulate == 1) {
      const long long idx = cbase + rr * p.ldc + c;
      old[e] = p.c_f32 ? ((const float*)Cb)[idx] : to_f32(((const T*)Cb)[idx]);
    }
  }
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    if (!ok[e]) continue;
    float x = v[e] * p.alpha * cs[e] + bi[e];
    if (p.drop_p > 0.f) {
      x = act_apply(x, p.act, p.act_alpha);
      x = uniform01(drop_key(p), (uint64_t)row[e] * (uint64_t)p.N + (uint64_t)col[e]) >= p.drop_p
              ? x / (1.f - p.drop_p) : 0.f;
      x += rv[e];
    } else if (p.r_mask) {
      x = Rg ? act_apply(x, p.act, p.act_alpha) * act_mask_from_y(rv[e], p.r_mask, p.act_alpha) : act_apply(x, p.act, p.act_alpha);
    } else {
      x = act_apply(x + rv[e], p.act, p.act_alpha);
    }
    const long long idx = cbase + (long long)row[e] * p.ldc + col[e];
    if (p.c_f32) {
      float* Cp = (float*)Cb + idx;
      if (p.accumulate == 2) atomicAdd(Cp, x);
      else *Cp = p.accumulate == 1 ? old[e] + x : x;
    } else {
      ((T*)Cb)[idx] = from_f32<T>(p.accumulate == 1 ? old[e] + x : x);
    }
  }
}

template <typename T, int KW>
__global__ __launch_bounds__(64 * KW) void gemm_small_kernel(const GemmParams p) {
  constexpr int TN = SMALL_TN;  // 32 x 64 output tile
  constexpr int U = 4;          // k-steps of 16 per register buffer
  __shared__ float red[4][TN][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int tiles_n = (p.N + 63) / 64;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * 32, n0 = tn * 64;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const T* __restrict__ Ag = (const T*)p.A + zo * p.a_so + zi * p.a_si;
  const T* __restrict__ Bg = (const T*)p.B + zo * p.b_so + zi * p.b_si;
  const int M = p.M, N = p.N, K = p.K;
  // split-K over blockIdx.y (k-range multiple of 16), then over the KW waves
  const int S = p.split_k > 1 ? p.split_k : 1, split = blockIdx.y;
  const int kb = S > 1 ? split * p.k_per_split : 0;
  const int ke = S > 1 ? min(K, kb + p.k_per_split) : K;
  const int nks = ke > kb ? (ke - kb + 15) / 16 : 0;
  const int per = (nks + KW - 1) / KW;
  // wave-uniform: readfirstlane keeps the K-loop control in SGPRs (scalar
  // branches instead of exec-mask regions around the loads)
  const int ks0 = __builtin_amdgcn_readfirstlane(kb / 16 + wave * per);
  const int ks1 = __builtin_amdgcn_readfirstlane(kb / 16 + min(nks, wave * per + per));
  const int arow = m0 + lr;
  f32x16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  const bool a_ok = arow < M;
  const T* arp = Ag + (long long)arow * p.lda;
  const T* brp[TN];
  bool b_ok[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int bcol = n0 + t * 32 + lr;
    b_ok[t] = bcol < N;
    brp[t] = Bg + (long long)bcol * p.ldb;
  }
  typedef typename TT<T>::Vec VecT;
  constexpr int V = TT<T>::VEC;
  constexpr int NV = 8 / V;  // 16-B vectors per 8-element fragment
  auto mfma_round = [&](VecT (&av)[U][NV], VecT (&bv)[U][TN][NV]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (std::is_same<T, bf16>::value) {
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[u][0], bv[u][t][0], acc[t], 0, 0, 0);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int t = 0; t < TN; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u][j / 4][j % 4], bv[u][t][j / 4][j % 4], acc[t], 0, 0, 0);
      }
    }
  };
  // Block-uniform choice of the load path. The vector path issues every
  // 16-B fragment load unconditionally from a clamped in-bounds address and
  // zeroes out-of-range values with a select afterwards: no branch around a
  // load, so all U x (1 + TN) x NV loads of a round are in flight together
  // (a per-element "load or zero" branch makes hipcc wait vmcnt(0) after
  // every load and serialises the K loop on memory latency).
  const bool vec_ok = ((p.lda | p.ldb) % V) == 0 && (K % V) == 0 && (((uintptr_t)Ag | (uintptr_t)Bg) & 15) == 0;
  if (vec_ok) {
    // rows >= M / columns >= N read row 0 / column 0 instead (their outputs
    // are never stored); k beyond the wave's range zeroes the A fragment only
    const T* ar = a_ok ? arp : Ag;
    const T* br[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) br[t] = b_ok[t] ? brp[t] : Bg;
    auto load_round = [&](int ks, VecT (&av)[U][NV], VecT (&bv)[U][TN][NV]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          const int kq = (ks + u) * 16 + 8 * lh + q * V;
          const int kc = ((ks + u) < ks1 && kq < K) ? kq : 0;
          av[u][q] = *(const VecT*)(ar + kc);
#pragma unroll
          for (int t = 0; t < TN; ++t) bv[u][t][q] = *(const VecT*)(br[t] + kc);
        }
      }
    };
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    auto mask_round = [&](int ks, VecT (&av)[U][NV]) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          const int kq = (ks + u) * 16 + 8 * lh + q * V;
          const unsigned keep = ((ks + u) < ks1 && kq < K) ? ~0u : 0u;
          av[u][q] = __builtin_bit_cast(VecT, __builtin_bit_cast(u32x4, av[u][q]) & keep);
        }
    };
    // register double buffer (two named sets, no copies): the next round's
    // loads are in flight while this round's MFMAs run
    VecT aA[U][NV], bA[U][TN][NV], aB[U][NV], bB[U][TN][NV];
    int ks = ks0;
    if (ks < ks1) load_round(ks, aA, bA);
    while (ks < ks1) {
      if (ks + U < ks1) load_round(ks + U, aB, bB);
      mask_round(ks, aA);
      mfma_round(aA, bA);
      ks += U;
      if (ks >= ks1) break;
      if (ks + U < ks1) load_round(ks + U, aA, bA);
      mask_round(ks, aB);
      mfma_round(aB, bB);
      ks += U;
    }
  } else {
    for (int ks = ks0; ks < ks1; ks += U) {
      VecT av[U][NV], bv[U][TN][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = (ks + u) * 16 + 8 * lh;
        const bool kin = (ks + u) < ks1;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          const int kq = k + q * V;
#pragma unroll
          for (int j = 0; j < V; ++j) av[u][q][j] = (kin && a_ok && kq + j < K) ? arp[kq + j] : (T)0.f;
#pragma unroll
          for (int t = 0; t < TN; ++t)
#pragma unroll
            for (int j = 0; j < V; ++j) bv[u][t][q][j] = (kin && b_ok[t] && kq + j < K) ? brp[t][kq + j] : (T)0.f;
        }
      }
      mfma_round(av, bv);
    }
  }
  // in-block reduction over the KW waves: waves 0..3 store, the others add
  // in groups of 4 (one LDS image of 4 partial tiles)
#pragma unroll
  for (int g = 0; g < KW / 4; ++g) {
    if ((wave >> 2) == g) {
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (g == 0) red[wave & 3][t][i][lane] = acc[t][i];
          else red[wave & 3][t][i][lane] += acc[t][i];
        }
    }
    __syncthreads();
  }
  const int tile_id = blockIdx.z * gridDim.x + blockIdx.x;
  if (S > 1) {
    // publish this split's partial tile; gemm_small_reduce_kernel combines
    float* mine = p.ws_part + ((long long)tile_id * S + blockIdx.y) * SMALL_TILE_FLOATS;
    for (int e = threadIdx.x; e < SMALL_TILE_FLOATS; e += 64 * KW) {
      const int t = e >> 10, i = (e >> 6) & 15, l = e & 63;
      mine[e] = red[0][t][i][l] + red[1][t][i][l] + red[2][t][i][l] + red[3][t][i][l];
    }
    return;
  }
  constexpr int NE = SMALL_TILE_FLOATS / (64 * KW);
  float ev[NE];
  int erow[NE], ecol[NE];
  bool eok[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int e = threadIdx.x + 64 * KW * j;
    const int t = e >> 10, i = (e >> 6) & 15, l = e & 63;
    ecol[j] = n0 + t * 32 + (l & 31);
    erow[j] = m0 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    eok[j] = ecol[j] < N && erow[j] < M;
    ev[j] = red[0][t][i][l] + red[1][t][i][l] + red[2][t][i][l] + red[3][t][i][l];
  }
  small_epilogue_n<T, NE>(p, ev, erow, ecol, eok, p.C, p.R, zo, zi);
}

// sums the S partial tiles of a split small GEMM in split order
// (deterministic) and runs the epilogue; grid (tiles, 8, batch): one element
// per thread, coalesced partial reads
template <typename T>
__global__ __launch_bounds__(256) void gemm_small_reduce_kernel(const GemmParams p, int S) {
  const int tiles_n = (p.N + 63) / 64;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * 32, n0 = tn * 64;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const int tile_id = blockIdx.z * gridDim.x + blockIdx.x;
  const float* parts = p.ws_part + (long long)tile_id * S * SMALL_TILE_FLOATS;
  const int e = blockIdx.y * 256 + threadIdx.x;
  const int t = e >> 10, i = (e >> 6) & 15, l = e & 63;
  const int col = n0 + t * 32 + (l & 31);
  const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
  if (col >= p.N || row >= p.M) return;
  float v = 0.f;
  for (int q = 0; q < S; ++q) v += parts[(long long)q * SMALL_TILE_FLOATS + e];
  small_epilogue<T>(p, v, row, col, zo, zi);
}

// Deterministic split-K for accumulating fp32 outputs (weight gradients):
// the S splits of a launch stored raw fp32 partials ws[split][z][row][col]
// (plain stores, no epilogue); this adds alpha * col_scale * (their sum) to
// C with one writer per element. Per-split fp32 atomics into C would sum in
// block-scheduling order, i.e. differently on every run. A block is G split
// lanes x (256 / G) four-column items: lane g sums splits g, g + G, ... and
// the G partials are combined in lane order through LDS — a fixed order, with
// G > 1 spreading the long split loops of small weight tensors (S ~ 100) over
// enough blocks to fill the chip.
// sum_{k = k0, k0 + G, ... < S} src[k * slab .. +3], added in k order (the
// deterministic order of every split-K reduction) with 8 loads in flight per
// thread: a plain loop keeps one 16-B load outstanding and the reduction runs
// at the load latency, not at HBM / L2 bandwidth. The last round (fewer than
// 8 splits left: every round of the common S / G <= 4 jobs) loads clamped
// addresses unconditionally and adds only the live ones, so its loads are in
// flight together too (the same adds in the same order as a plain loop).
__device__ __forceinline__ f32x4 ordered_slab_sum4(const float* src, long long slab, int k0, int S, int G) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  for (int k = k0; k < S; k += 8 * G) {
    f32x4 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = *(const f32x4*)(src + (long long)min(k + u * G, S - 1) * slab);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k + u * G < S) v += a[u];
  }
  return v;
}

template <int G>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const GemmParams p, const float* __restrict__ ws, int S,
                                                           int batch) {
  constexpr int IT = 256 / G;
  __shared__ f32x4 red[G][IT];
  const int c4 = (p.N + 3) / 4;
  const int it = threadIdx.x % IT, g = threadIdx.x / IT;
  const long long q = (long long)blockIdx.x * IT + it;
  const bool live = q < (long long)p.M * c4;
  const int z = blockIdx.y;
  const int row = live ? (int)(q / c4) : 0, col = live ? (int)(q - (long long)row * c4) * 4 : 0;
  const long long per = (long long)p.M * p.N, slab = per * batch;
  const float* src = ws + z * per + (long long)row * p.N + col;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    if ((p.N & 3) == 0) {
      v = ordered_slab_sum4(src, slab, g, S, G);
    } else {
      for (int k = g; k < S; k += G)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (col + j < p.N) v[j] += src[k * slab + j];
    }
  }
  if constexpr (G > 1) {
    red[g][it] = v;
    __syncthreads();
    if (g != 0) return;
#pragma unroll
    for (int k = 1; k < G; ++k) v += red[k][it];
  }
  if (!live) return;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  float* C = (float*)p.C + zo * p.c_so + zi * p.c_si + (long long)row * p.ldc + col;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (col + j < p.N) C[j] += v[j] * p.alpha * (p.col_scale ? p.col_scale[col + j] : 1.f);
}

// Split-K of gemm_kernel through the workspace: the S splits of an (M x N)
// problem wrote fp32 partial slabs ws[split][row][col] with no epilogue; this
// sums them in split order (deterministic) and runs the problem's epilogue.
// M-grouped launches: the slab rows are the groups' rows back to back
// (row_off), each group's output / residual its own. 4 consecutive columns
// per thread (16-B partial loads).
struct RowOffsets {
  int off[MAX_GROUPS + 1];
};
template <typename T>
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const GemmParams p, const float* __restrict__ ws,
                                                                 int S, RowOffsets ro) {
  const int Mt = p.ngroups > 0 ? ro.off[p.ngroups] : p.M;
  const int c4 = (p.N + 3) / 4;
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long long)Mt * c4) return;
  const int row = (int)(q / c4), col = (int)(q - (long long)row * c4) * 4;
  void* Cb = p.C;
  const void* Rb = p.R;
  int r0 = 0;
  if (p.ngroups > 0) {  // static indices only (no scratch copy of the kernarg struct)
    Cb = p.groups[0].C;
    Rb = p.groups[0].R;
#pragma unroll
    for (int g = 1; g < MAX_GROUPS; ++g)
      if (g < p.ngroups && row >= ro.off[g]) {
        Cb = p.groups[g].C;
        Rb = p.groups[g].R;
        r0 = ro.off[g];
      }
  }
  const long long slab = (long long)Mt * p.N;
  const float* src = ws + (long long)row * p.N + col;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (col + 4 <= p.N && (p.N & 3) == 0) {
    const f32x4 x = ordered_slab_sum4(src, slab, 0, S, 1);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  } else {
    for (int k = 0; k < S; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (col + j < p.N) v[j] += src[k * slab + j];
  }
  int er[4], ec[4];
  bool eok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    er[j] = row - r0;
    ec[j] = col + j;
    eok[j] = col + j < p.N;
  }
  small_epilogue_n<T, 4>(p, v, er, ec, eok, Cb, Rb, 0, 0);
}

template <typename T> int dispatch_gemm(GemmParams& p, int amode, int bmode, hipStream_t stream);

// deferred.hip: queue the ordered split reduction of slabs ws (written by an
// accumulating split-K launch of p) into p.C, split lanes G
int defer_wgrad(const GemmParams& p, const float* ws, int batch, int G, hipStream_t s);

// Deferred weight-gradient GEMMs: C (fp32, M x N, ldc) += alpha * A^T B with A
// (K x M, lda) and B (K x N, ldb) bf16 rows (a Dense layer's x and dz). Inside
// fpnmt_defer_begin / _flush these are queued (deferred.hip) and run at the
// flush as a few grouped launches (gemm_bf16.hip: launch_gemm_jobs), one
// writer per C element per launch.
struct DefGemmJob {
  const void* A;
  const void* B;
  float* C;
  int M, N, K;
  int lda, ldb, ldc;
  float alpha;
  int tiles_n, blk0;
};
constexpr int GEMM_JOBS_PER_LAUNCH = 32;
int defer_gemm_job(const DefGemmJob& J, hipStream_t s);                     // deferred.hip (queues)
int launch_gemm_jobs(const DefGemmJob* jobs, int n, hipStream_t s);         // gemm_bf16.hip

}  // namespace fpnmt
