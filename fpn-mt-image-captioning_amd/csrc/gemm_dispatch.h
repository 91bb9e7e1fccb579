// Host-side tile-config selection and launch for gemm_kernel<T,...> and
// gemm_small_kernel<T>. Included once per element type (gemm_bf16.hip,
// gemm_f32.hip) so the two instantiation sets compile in parallel.
//
// Config policy (tools/gemm_bench.hip, MI355X, bf16, C2 shapes): the tiled
// kernel is occupancy/latency bound at these sizes, so 64x64 tiles win unless
// 128x128 still gives >= 1.5 blocks per CU; BK = 64 pays for deep K (>= 1024).
#pragma once
#include <cstdio>
#include <cstdlib>
#include "gemm_impl.h"
#include "gemm_pipe.h"
#include "gemm_skinny.h"

namespace fpnmt {

static int cu_count_dispatch() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

enum { CFG_128_128_64 = 0, CFG_64_64_32, CFG_64_64_64, CFG_128_128_32, CFG_32_32_32, CFG_SMALL };
struct TileCfg {
  int bm, bn, bk;
};
static const TileCfg kCfg[] = {{128, 128, 64}, {64, 64, 32}, {64, 64, 64}, {128, 128, 32}, {32, 32, 32}, {32, 64, 16}};

template <typename T, int BM, int BN, int WM, int WN, int AM, int BMODE, int BK>
static int launch_one(GemmParams& p, int batch, bool vec, hipStream_t s) {
  if (p.ngroups > 0 && !p.group_k) {  // m-grouped: groups own consecutive m-tile ranges
    int t = 0;
    for (int g = 0; g < p.ngroups; ++g) {
      p.groups[g].start = t;
      t += cdiv(p.groups[g].M, BM);
    }
    p.tiles_m = t;
  } else {
    p.tiles_m = cdiv(p.M, BM);
  }
  p.tiles_n = cdiv(p.N, BN);
  dim3 grid(p.tiles_m * p.tiles_n, p.split_k, batch);
  dim3 block(64 * WM * WN);
  if (vec)
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, AM, BMODE, true, BK>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, AM, BMODE, false, BK>), grid, block, 0, s, p);
  return check_launch("gemm_kernel");
}

// M <= 32 rows and K <= 1024 (the encoder's baseline-token GEMMs):
// gemm_skinny_kernel when the operands are 16-B vectors. tools/small_bench.hip
// (MI355X, graph replay, us per launch, warm weights): 32x512x512 6.47
// (small<8>) -> 5.10 (skinny<4,32>); in the C2 step (cold weights) 8.7 -> 7.5
// (N = 512) and 6.8 (N = 2048). K = 2048 stays on the split small kernel:
// skinny<16,32> (16 blocks) took 17 us there against 9.4 warm in the bench.
static bool skinny_eligible(const GemmParams& p) {
  if (p.M > 32 || p.K > 1024 || p.ngroups > 0 || p.accumulate == 2 || p.c_mode != C_ROW) return false;
  if ((p.lda | p.ldb) % 8 || p.K % 8 || (p.a_so | p.a_si | p.b_so | p.b_si) % 8) return false;
  return (((uintptr_t)p.A | (uintptr_t)p.B) & 15) == 0;
}

static int launch_skinny(GemmParams& p, int batch, hipStream_t s) {
  p.split_k = 1;
  p.k_per_split = p.K;
  p.ws_part = nullptr;
  p.ws_cnt = nullptr;
  hipLaunchKernelGGL((gemm_skinny_kernel<4, 32>), dim3(cdiv(p.N, 32), 1, batch), dim3(256), 0, s, p);
  return check_launch("gemm_skinny_kernel");
}

template <typename T>
static int launch_small(GemmParams& p, int batch, hipStream_t s) {
  if constexpr (std::is_same<T, bf16>::value) {
    if (skinny_eligible(p)) return launch_skinny(p, batch, s);
  }
  // KW = 8 waves split K inside a block when each still gets >= 4 k-steps;
  // blocks split K further (partials + a reduce launch) only when the tile
  // count leaves most CUs idle, keeping >= 64 k per wave
  const long long tiles = (long long)cdiv(p.M, 32) * cdiv(p.N, 64) * batch;
  const int KW = p.K >= 8 * 64 ? 8 : 4;
  int S = 1;
  if (g_split_ws.part && p.accumulate != 2 && tiles < 128) {
    S = (int)std::min<long long>(16, (256 + tiles - 1) / tiles);
    S = std::min(S, p.K / (KW * 64));
    if (S < 2 || tiles * S * SMALL_TILE_FLOATS > g_split_ws.part_floats) S = 1;
  } else if (g_split_ws.part && p.accumulate != 2 && p.K > KW * 16 * 32) {
    // long reductions on enough tiles (the decoder's vocabulary-wide dgrad,
    // M = 992, K = 10000: 78 serial k-steps per wave, 85 us): ~16 k-steps
    // per wave, the rest across blocks
    S = (int)std::min<long long>(16, cdiv(p.K, KW * 16 * 16));
    if (tiles * S * SMALL_TILE_FLOATS > g_split_ws.part_floats) S = 1;
  }
  p.k_per_split = S > 1 ? cdiv(cdiv(p.K, S), 16) * 16 : p.K;
  if (S > 1) S = cdiv(p.K, p.k_per_split);
  p.split_k = S;
  p.ws_part = g_split_ws.part;
  // (the tile's last arriving split combining in this launch, through the
  // workspace's arrival counters, measured slower: 18.8 us against 7.5 + 4.9
  // for the two launches — the device-scope release before each arrival
  // writes back the XCD's L2)
  p.ws_cnt = nullptr;
  dim3 grid(cdiv(p.M, 32) * cdiv(p.N, 64), S, batch);
  if (KW == 8)
    hipLaunchKernelGGL((gemm_small_kernel<T, 8>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_small_kernel<T, 4>), grid, dim3(256), 0, s, p);
  if (S > 1) {
    const int st = check_launch("gemm_small_kernel");
    if (st) return st;
    hipLaunchKernelGGL((gemm_small_reduce_kernel<T>), dim3(grid.x, SMALL_TILE_FLOATS / 256, batch), dim3(256), 0, s, p, S);
  }
  return check_launch("gemm_small_kernel");
}

// bf16 gets the BK=64 variants; f32 (parity mode) keeps BK=16 everywhere.
template <typename T> constexpr int bk_of(int bk) { return std::is_same<T, float>::value ? 16 : bk; }

template <typename T, int AM, int BMODE>
static int launch_cfg(int cfg, GemmParams& p, int batch, bool vec, hipStream_t s) {
  constexpr bool F32 = std::is_same<T, float>::value;
  switch (cfg) {
    case CFG_128_128_64:
      if constexpr (!F32 && (AM == A_IM2COL || AM == A_ROW || AM == A_IM2COL_T || AM == A_COL))
        return launch_one<T, 128, 128, 2, 2, AM, BMODE, 64>(p, batch, vec, s);
      return launch_one<T, 128, 128, 2, 2, AM, BMODE, 0>(p, batch, vec, s);
    case CFG_64_64_64:
      if constexpr (!F32 && (AM == A_IM2COL || AM == A_ROW || AM == A_IM2COL_T))
        return launch_one<T, 64, 64, 2, 2, AM, BMODE, 64>(p, batch, vec, s);
      return launch_one<T, 64, 64, 2, 2, AM, BMODE, 0>(p, batch, vec, s);
    case CFG_128_128_32: return launch_one<T, 128, 128, 2, 2, AM, BMODE, 0>(p, batch, vec, s);
    case CFG_32_32_32: return launch_one<T, 32, 32, 1, 1, AM, BMODE, 0>(p, batch, vec, s);
    default: return launch_one<T, 64, 64, 2, 2, AM, BMODE, 0>(p, batch, vec, s);
  }
}

static long long blocks_for(int M, int N, long long batch, int cfg) {
  return (long long)cdiv(M, kCfg[cfg].bm) * cdiv(N, kCfg[cfg].bn) * batch;
}

static int choose_cfg(int amode, int bmode, int M, int N, int K, long long batch, int accumulate, int c_mode) {
  // long-K row GEMMs over a few hundred to a few thousand rows (the decoder's
  // vocabulary-wide dgrad, M = 992, K = 10 000; the views' grouped K/V
  // projection dgrads, K = 6144): 128x128 tiles split over K through the
  // workspace (ws_split_for) — the small kernel's 32x64 tiles re-read the
  // operands from L2 ~4x as often (C2 step, with the reduce: M = 992 84 ->
  // 48 us, M = 1568 80 -> 32; M = 288 went 29 -> 36 on its 12 tiles: small)
  if (c_mode == C_ROW && amode == A_ROW && bmode == B_NK && accumulate != 2 && batch == 1 && K >= 4096 &&
      M >= 512 && M <= 4096 && N >= 256)
    return CFG_128_128_64;
  // row-major x weight GEMMs that would leave the chip under-filled with 64x64
  // tiles go to the small kernel (4 waves split K inside a 32x64 tile)
  if (c_mode == C_ROW && amode == A_ROW && bmode == B_NK && K >= 64 &&
      (M <= 64 || blocks_for(M, N, batch, CFG_64_64_32) < 256) && blocks_for(M, N, batch, CFG_SMALL) <= 4096)
    return CFG_SMALL;
  if (M <= 32 && N <= 32) return CFG_32_32_32;
  const bool deep = K >= 1024;
  if (amode == A_IM2COL_T || amode == A_COL) {
    // weight gradients: K = pixels / rows (split-K over blocks); 128x128
    // tiles halve the operand traffic per FLOP where both sides are wide.
    // A rank-32 update (the encoder's M = 32 rows: 512 x 512 fp32 C read and
    // written once, 64 blocks of 64x64) is all C traffic: 32x32 tiles put 4x
    // the blocks on it
    if (K <= 64 && blocks_for(M, N, batch, CFG_64_64_32) < 256) return CFG_32_32_32;
    return deep ? CFG_64_64_64 : CFG_64_64_32;
  }
  // shallow (K <= 256) GEMMs over many rows are HBM-bound (the bottlenecks'
  // 1x1 convs, e.g. res2 64->256 + residual: 8 FLOP per byte moved):
  // 64x64 tiles at occupancy 4-6 keep more bytes in flight than 128x128 at 2
  // (tools/gemm_bench.hip, b64 res2 1x1 +R: 51.6 vs 80 us; res3: 34.6 vs 54.5)
  // (scattered rows too: the strided 1x1 bwd-data of a projection block's 2a)
  if (K <= 256 && blocks_for(M, N, batch, CFG_64_64_32) >= 1024)
    return K >= 256 ? CFG_64_64_64 : CFG_64_64_32;
  if (M > 64 && N > 64 && blocks_for(M, N, batch, CFG_128_128_64) >= 384) return deep ? CFG_128_128_64 : CFG_128_128_32;
  if (M <= 32 || N <= 32) return blocks_for(M, N, batch, CFG_32_32_32) >= 128 && (M <= 32) ? CFG_32_32_32 : CFG_64_64_32;
  return deep ? CFG_64_64_64 : CFG_64_64_32;
}

// FPNMT_GEMM_LOG=<file>: one line per launch (shape, modes, tile config),
// joined with a rocprofv3 kernel trace by tools/gemm_shapes.py
static FILE* gemm_log() {
  static FILE* f = [] {
    const char* path = std::getenv("FPNMT_GEMM_LOG");
    return path ? std::fopen(path, "a") : nullptr;
  }();
  return f;
}

template <typename T>
static void log_gemm(const GemmParams& p, int batch, int amode, int bmode, int cfg) {
  if (FILE* f = gemm_log()) {
    std::fprintf(f, "%s a=%d b=%d c=%d M=%d N=%d K=%d batch=%d acc=%d split=%d cfg=%d\n",
                 std::is_same<T, float>::value ? "f32" : "bf16", amode, bmode, p.c_mode, p.M, p.N, p.K, batch,
                 p.accumulate, p.split_k, cfg);
    std::fflush(f);
  }
}

// the batch entries' C tiles (M rows of ldc, N columns) do not overlap:
// batch_inner == 1 and c_so >= (M - 1) * ldc + N (each entry its own slice)
static bool c_batches_disjoint(const GemmParams& p, int batch) {
  if (p.batch_inner != 1 || p.c_mode != C_ROW) return false;
  return p.c_so >= (long long)(p.M - 1) * p.ldc + p.N && p.c_so > 0;
}

// ---- deterministic split-K for accumulating fp32 C (weight gradients) ---
// Splits write raw fp32 partial slabs ws[split][z][m][n] (q = the launch's
// params redirected there), wgrad_reduce_kernel adds their split-ordered sum
// into C. The slabs go to the deferred-reduction arena while one is active
// (fpnmt_defer_begin: the reduce is queued and batched at the flush), else
// to the process workspace (reduced right after the launch).
// slab_fits: the slabs of `splits` splits fit one of the two.
static bool slab_fits(const GemmParams& p, int batch, long long splits) {
  const long long need = splits * batch * (long long)p.M * p.N;
  return need <= defer_room() || (g_split_ws.part && need <= g_split_ws.part_floats);
}

static float* slab_alloc(const GemmParams& p, int batch, long long splits) {
  float* d = defer_alloc(splits * batch * (long long)p.M * p.N);
  return d ? d : g_split_ws.part;
}

static GemmParams slab_params(const GemmParams& p, int batch, float* base) {
  GemmParams q = p;
  const long long per = (long long)p.M * p.N;
  q.C = base;
  for (int g = 0; g < p.ngroups; ++g) q.groups[g].C = base;  // k-grouped: one shared C
  q.accumulate = 0;
  q.c_f32 = 1;
  q.alpha = 1.f;
  q.col_scale = nullptr;
  q.ldc = p.N;
  q.c_si = per;
  q.c_so = per * p.batch_inner;
  q.c_split = per * batch;
  return q;
}

// an immediate accumulation into C (atomics / read-modify-write) is about to
// be issued: queued reductions into the same gradient run first (their order)
static int touch_c(const GemmParams& p, int batch, hipStream_t s) {
  if (!defer_active()) return 0;
  long long hi = 0;
  for (int z = 0; z < batch; ++z) {
    const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
    hi = std::max(hi, zo * p.c_so + zi * p.c_si);
  }
  const float* c = (const float*)p.C;
  return defer_touch(c, c + hi + (long long)(p.M - 1) * p.ldc + p.N, s);
}

template <int G>
static void wgrad_reduce_g(const GemmParams& p, int batch, const float* base, hipStream_t s) {
  const long long items = (long long)p.M * cdiv(p.N, 4);
  constexpr int IT = 256 / G;
  hipLaunchKernelGGL((wgrad_reduce_kernel<G>), dim3((unsigned)((items + IT - 1) / IT), batch), dim3(256), 0, s, p,
                     base, p.split_k, batch);
}

static int launch_wgrad_reduce(const GemmParams& p, int batch, const float* base, hipStream_t s) {
  // split lanes per item: enough blocks for the chip on small weight tensors;
  // one lane per item on large ones (>= 65536 items: >= 256 blocks), so a
  // block sweeps 4 KB of every slab instead of 256 B - 1 KB runs of G of them
  const long long items = (long long)p.M * cdiv(p.N, 4) * batch;
  const int G = items >= 256 * 256 ? 1 : (p.split_k >= 8 ? 16 : p.split_k >= 4 ? 4 : 1);
  if (defer_owns(base)) return defer_wgrad(p, base, batch, G, s);
  {
    const int st = touch_c(p, batch, s);
    if (st) return st;
  }
  if (G == 16) wgrad_reduce_g<16>(p, batch, base, s);
  else if (G == 4) wgrad_reduce_g<4>(p, batch, base, s);
  else wgrad_reduce_g<1>(p, batch, base, s);
  return check_launch("wgrad_reduce_kernel");
}

// ---- pipelined LDS-DMA kernel (bf16, k-contiguous A and B) -------------
static bool pipe_row_short(const GemmParams& p, int batch) {
  return batch == 1 && p.M >= 256 && p.M <= 4096 && p.N >= 256 && p.K >= 256 && p.K <= 2048;
}

template <typename T>
static bool pipe_eligible(const GemmParams& p, int batch, int amode, int bmode, bool vec) {
  if constexpr (!std::is_same<T, bf16>::value) return false;
  if (!g_split_ws.zero || !vec || bmode != B_NK || p.accumulate == 2 || p.c_mode != C_ROW)
    return false;
  if (p.ngroups > 0 && p.group_k) return false;
  if (p.K % 64 || p.ldb % 8 || (p.b_so | p.b_si) % 8) return false;
  // 32-bit element offsets inside the kernel (A / B per batch entry)
  if ((long long)p.N * p.ldb >= (1LL << 31)) return false;
  if (amode == A_ROW && (long long)p.M * p.lda >= (1LL << 31)) return false;
  if (amode == A_IM2COL && ((long long)p.M * p.sh * p.sw + (long long)p.H * p.W) * p.Cc * 2 >= (1LL << 31)) return false;
  if (amode == A_IM2COL && p.Rk * p.Sk > 64) return false;
  // the direct epilogue's 4-column groups (N % 8 also keeps 16-B R rows)
  if (p.N % 8 || p.ldc % 4 || (p.R && p.ldr % 8) || (p.c_so | p.c_si | p.r_so | p.r_si) % 4) return false;
  if (((uintptr_t)p.C | (uintptr_t)p.R) & 7) return false;
  for (int g = 0; g < p.ngroups; ++g)
    if (((uintptr_t)p.groups[g].C | (uintptr_t)p.groups[g].R) & 7) return false;
  if (amode == A_IM2COL) {
    // every implicit-GEMM conv with 64-channel K-tiles (tools/fwd_bench.hip:
    // the LDS-DMA kernel beat the register-staged one on every R50-FPN
    // forward shape at batch 64)
    return p.Cc % 64 == 0;
  }
  if (amode == A_ROW) {
    if (p.lda % 8 || (p.a_so | p.a_si) % 8) return false;
    // row-major Dense: the wide problems (128x256 tiles), and the short-row
    // blocks of the decoder (M = B*T = 992 at C2, 2048 rows per C5 decode
    // step) on 64x64 tiles with a 4-stage ring (pipe_row_short); the
    // encoder's M = 32 rows stay on the skinny / small kernels
    if (p.N >= 256 && p.K >= 512 && (long long)cdiv(p.M, 128) * cdiv(p.N, 256) * batch >= 128) return true;
    return pipe_row_short(p, batch);
  }
  return false;
}

// splits > 1: split-K over grid.y; p is then the partial-slab form (see
// launch_pipe_split) and k_per_split K-tiles * 64 per split
template <int BM, int BN, int WM, int WN, int AM, int NT, int STAGES, int EPI, int SPREAD = 0, int MF = 32>
static int launch_pipe(GemmParams& p, int batch, int splits, hipStream_t s) {
  if (p.ngroups > 0) {
    int t = 0;
    for (int g = 0; g < p.ngroups; ++g) {
      p.groups[g].start = t;
      t += cdiv(p.groups[g].M, BM);
    }
    p.tiles_m = t;
  } else {
    p.tiles_m = cdiv(p.M, BM);
  }
  p.tiles_n = cdiv(p.N, BN);
  p.split_k = splits;
  if (splits <= 1) p.k_per_split = p.K;
  p.zero16 = g_split_ws.zero;
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, WM, WN, AM, NT, STAGES, EPI, 64, SPREAD, MF>),
                     dim3(p.tiles_m * p.tiles_n, splits, batch), dim3(NT), 0, s, p);
  return check_launch("gemm_pipe_kernel");
}

// the loader-wave form (gemm_pipe_lw_kernel): same grid / split / group
// conventions as launch_pipe, WM * WN + NLW waves per block
template <int BM, int BN, int WM, int WN, int AM, int NLW, int STAGES, int MS = BM>
static int launch_pipe_lw(GemmParams& p, int batch, int splits, hipStream_t s) {
  if (p.ngroups > 0) {
    int t = 0;
    for (int g = 0; g < p.ngroups; ++g) {
      p.groups[g].start = t;
      t += cdiv(p.groups[g].M, MS);
    }
    p.tiles_m = t;
  } else {
    p.tiles_m = cdiv(p.M, MS);
  }
  p.tiles_n = cdiv(p.N, BN);
  p.split_k = splits;
  if (splits <= 1) p.k_per_split = p.K;
  p.zero16 = g_split_ws.zero;
  hipLaunchKernelGGL((gemm_pipe_lw_kernel<BM, BN, WM, WN, AM, NLW, STAGES, MS>), dim3(p.tiles_m * p.tiles_n, splits, batch),
                     dim3(64 * (WM * WN + NLW)), 0, s, p);
  return check_launch("gemm_pipe_lw_kernel");
}

// Tile / stage choice (tools/fwd_bench.hip on MI355X: the R50-FPN forward
// convs at batch 64 with cold caches (512 MB written between launches, the
// input re-touched), us per launch):
//   * small tiles at high occupancy: 64x64 (4 waves, direct epilogue) with
//     one stage when the tiles fill the chip several times over (res2 1x1
//     64->256 47.7; res3 3x3 37.5), deeper rings as the tile count drops, since
//     a block then waits out each K-tile's DMA latency alone: two stages at
//     512-1023 tiles (res4 1x1 1024->256 21.9, res4 3x3 37.1), four below 512
//     (res5 3x3 42.6 against 70.3 with one stage, P5 23.4 against 38.4);
//   * a residual / act-mask operand: 128x64 with the LDS-staged row epilogue
//     (16-B residual rows; the direct epilogue's 8-B gathers were slower):
//     res2 1x1 + R 74.6;
//   * the wide compute-bound convs (N >= 256, K >= 2048, >= 192 tiles of
//     128x256): 128x256 with 8 waves, two stages (C2 P3 3x3, P3 at batch 64);
//   * fewer than 128 tiles (P7): split-K (fp32 slabs + ordered reduce).
//   * with a residual / act-mask operand the staged row epilogue pays only
//     on short reductions (nk < 8, where the epilogue is most of the time);
//     deeper ones (the bwd-data of the r4 / r5 / head 3x3 convs with the
//     producer's act' fused) take the same multi-stage tiles as without R,
//     the R rows prefetched into registers under the K loop (EPI 1): the
//     single-stage 128x64 form left 104-196 blocks waiting out every
//     K-tile's load (r5 bwd-data, 72 K-tiles: 61.8 us per launch).
//   * round 5 (tools/fwd_bench.hip -DFB_PP, profiles/r05/mf16_bench.txt): the
//     128x256 and 64x64 two-stage tiles on v_mfma_f32_16x16x32_bf16 (MF 16)
//     instead of 32x32x16: C2 P3 3x3 52.2 -> 48.2 us, P3 at batch 64 100.2 ->
//     89.4, res2 1x1 + R on 64x64 s2 96.1 -> 80.7; the one-stage 64x64 and
//     the 4-stage spread ring measured equal or slower on MF 16 and stay on
//     32x32x16; the staged-epilogue 128x64 form (EPI 0) has no MF 16 form.
//   * (measured and not taken: 64x128 tiles, 4 waves, one stage for
//     these: faster in tools/fwd_bench.hip with cold caches (52.7 / 91.1 us
//     against 56.7 / 100.2), 8 % slower on the warm P3 probe of bench.py
//     (58 against 53.5 us) and 0.06 ms per C2 step faster — within reach of
//     noise, so the 8-wave 128x256 form stays.)
//   * round 6 (tools/fwd_bench.hip -DFB_LW, profiles/r06/lw_sweep.txt): the
//     loader-wave kernel (gemm_pipe_lw_kernel: 4 waves own the LDS-DMA, the
//     MFMA waves only read fragments) in place of the 8-wave 128x256 tile
//     (C2 P3 3x3 48.7 -> 43.6 us, P3 at batch 64 91.3 -> 77.2), of the
//     4-stage 64x64 ring below 512 tiles (res5 3x3 43.2 -> 36.7, P5 22.4 ->
//     18.2, b32 res4 3x3 26.7 -> 22.7, b32 res5 36.8 -> 27.9) and, as a
//     128x128 tile, of the 2-stage 64x64 one on the 3x3 convs with N >= 256
//     (res4 3x3 / P4 37.0 -> 35.0, b32 FE output conv 37.6 -> 35.7); the
//     one-stage 64x64 and the staged-epilogue 128x64 classes stay (the loader
//     form lost 10-55 % there: short reductions, many tiles).
//     With the loader waves the 128x256 tile also takes the K >= 1024 1x1
//     convs once they fill the chip (C3's res4 1x1 1024->256 at 32^2 62.8 ->
//     52.9 us, res5 1x1 2048->512 at 16^2 49.0 -> 42.0; profiles/r06/c3_shapes.txt).
// M tiles of the launch at M step ms (grouped launches: per group)
static long long m_tiles(const GemmParams& p, int ms) {
  if (p.ngroups <= 0) return cdiv(p.M, ms);
  long long t = 0;
  for (int g = 0; g < p.ngroups; ++g) t += cdiv(p.groups[g].M, ms);
  return t;
}

//   * round 6, the wide class's tile count: 128x256 tiles leave CUs idle when
//     the launch's tiles fill a wave of blocks unevenly (C2 P3, M = 25 088: 196
//     tiles on 256 CUs). An M step of 112 rows (cfg 10: the same 128x256 LDS
//     image and 4 loaders, 1 x 8 MFMA waves of 112 x 32, rows 112-127 fed the
//     zero chunk) puts it on 224 tiles; taken where it leaves fewer output
//     rows per CU over the launch's waves of blocks (112 x ceil(t112 / CUs)
//     against 128 x ceil(t128 / CUs)). Measured against cfg 6 on one box
//     (bench.py --roofline-only, FPNMT_WIDE_CFG; profiles/r06/wide_tiles.txt):
//     42.1-42.6 -> 41.2-41.9 us by HIP events, 40.98 -> 40.37 us rocprofv3
//     average; headline forward 1.918 -> 1.905 ms. Lost: 224x128 (4 loaders, 2
//     x 4 waves of 112 x 32) 43.5-44.2 us, 208x128 (2 loaders, 1 x 8 of 208 x
//     16) 55.4-56.8 and 112x256 with 2 loaders (no zero rows) 47.8-48.4,
//     although the first two move fewer L2 -> LDS bytes per CU.
//     FPNMT_WIDE_CFG=6|10 forces one (A/B probes, the bitwise test).
static int wide_cfg(const GemmParams& p, int batch) {
  const char* e = std::getenv("FPNMT_WIDE_CFG");
  if (e && e[0]) {
    const int f = std::atoi(e);
    if (f == 6 || f == 10) return f;
  }
  const long long cus = cu_count_dispatch(), tn = (long long)cdiv(p.N, 256) * batch;
  const long long w128 = (m_tiles(p, 128) * tn + cus - 1) / cus, w112 = (m_tiles(p, 112) * tn + cus - 1) / cus;
  return 112 * w112 < 128 * w128 ? 10 : 6;
}

static int pipe_cfg(const GemmParams& p, int batch) {
  const long long tiles_big = (long long)cdiv(p.M, 128) * cdiv(p.N, 256) * batch;
  if (p.N >= 256 && p.K >= 1024 && tiles_big >= 192) return wide_cfg(p, batch);
  const long long tiles = (long long)cdiv(p.M, 64) * cdiv(p.N, 64) * batch;
  const int nk = p.K / 64;
  if (p.R && nk < 8) return 0;
  if (tiles < 512 && nk >= 8) return 8;
  if (tiles < 1024 && nk >= 32 && p.N >= 256) {
    // the 128x128 loader tile at the same 112-row M step (cfg 11: 1 x 4 MFMA
    // waves of 112 x 32) where it leaves fewer rows per CU (res4's 3x3: 196
    // tiles at batch 64, 98 at 32); FPNMT_WIDE_CFG=6 keeps the 128-row step
    const char* e = std::getenv("FPNMT_WIDE_CFG");
    const long long cus = cu_count_dispatch(), tn = (long long)cdiv(p.N, 128) * batch;
    const long long w128 = (m_tiles(p, 128) * tn + cus - 1) / cus, w112 = (m_tiles(p, 112) * tn + cus - 1) / cus;
    return !(e && e[0] == '6') && 112 * w112 < 128 * w128 ? 11 : 7;
  }
  if (tiles < 1024 && nk >= 8) return 2;
  return 1;
}

template <int AM>
static int launch_pipe_cfg(int cfg, GemmParams& p, int batch, int splits, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_pipe<128, 64, 4, 1, AM, 256, 1, 0>(p, batch, splits, s);
    case 2: return launch_pipe<64, 64, 2, 2, AM, 256, 2, 1, 0, 16>(p, batch, splits, s);
    case 3: return launch_pipe<128, 256, 2, 4, AM, 512, 3, 1, 2, 16>(p, batch, splits, s);
    case 4: return launch_pipe<64, 64, 2, 2, AM, 256, 4, 1, 1>(p, batch, splits, s);
    case 5: return launch_pipe<64, 32, 2, 2, AM, 256, 4, 1, 1, 16>(p, batch, splits, s);
    case 6: return launch_pipe_lw<128, 256, 2, 4, AM, 4, 3>(p, batch, splits, s);
    case 7: return launch_pipe_lw<128, 128, 2, 2, AM, 4, 3>(p, batch, splits, s);
    case 8: return launch_pipe_lw<64, 64, 2, 2, AM, 4, 4>(p, batch, splits, s);
    case 9: return launch_pipe_lw<64, 32, 2, 2, AM, 2, 4>(p, batch, splits, s);
    case 10: return launch_pipe_lw<128, 256, 1, 8, AM, 4, 3, 112>(p, batch, splits, s);
    case 11: return launch_pipe_lw<128, 128, 1, 4, AM, 4, 3, 112>(p, batch, splits, s);
    default: return launch_pipe<64, 64, 2, 2, AM, 256, 1, 1>(p, batch, splits, s);
  }
}

// Fewer than 128 tiles over a long K (P7 of the batch-64 forward): S partial
// fp32 slabs (no epilogue) in the workspace, summed in split order with the
// full epilogue by gemm_splitk_reduce_kernel.
// The decision counts 64x64 tiles whatever the launch's tile: a launch with
// a residual / act-mask operand (cfg 0) then splits exactly when the same
// launch without it does, so the fused act' epilogue stays bitwise equal to
// the unfused one (the same K order per output element).
static int pipe_split_for(const GemmParams& p, int batch) {
  if (!g_split_ws.part || batch != 1 || p.accumulate != 0) return 1;
  const int nkt = p.K / 64;
  long long tiles = 0;
  if (p.ngroups > 0)
    for (int g = 0; g < p.ngroups; ++g) tiles += cdiv(p.groups[g].M, 64);
  else
    tiles = cdiv(p.M, 64);
  tiles *= cdiv(p.N, 64);
  if (tiles >= 128 || nkt < 16) return 1;
  int S = (int)((256 + tiles - 1) / tiles);
  S = std::min(S, nkt / 8);
  S = std::min(S, 8);
  while (S > 1 && (long long)S * p.M * p.N > g_split_ws.part_floats) --S;
  return S < 2 ? 1 : S;
}

template <int AM>
static int launch_pipe_split(int cfg, int S, const GemmParams& p, hipStream_t s) {
  GemmParams q = p;
  const int nkt = p.K / 64;
  while (S > 1 && (long long)S * p.M * p.N > g_split_ws.part_floats) --S;  // the slabs fit the workspace
  if (S > nkt) S = nkt;
  const int kt_per = cdiv(nkt, std::max(S, 1));
  S = cdiv(nkt, kt_per);  // no empty split: every slab is written
  q.k_per_split = kt_per * 64;
  q.bias = nullptr;
  q.col_scale = nullptr;
  q.R = nullptr;
  q.r_mask = 0;
  q.act = FPNMT_ACT_NONE;
  q.drop_p = 0.f;
  q.drop_seed_dev = nullptr;
  q.alpha = 1.f;
  q.c_f32 = 1;
  q.accumulate = 0;
  q.C = g_split_ws.part;
  q.ldc = p.N;
  q.c_so = q.c_si = 0;
  q.c_split = (long long)p.M * p.N;  // p.M = the groups' rows in total
  RowOffsets ro{};
  for (int g = 0, r = 0; g < p.ngroups; ++g) {  // groups' slab rows back to back
    ro.off[g] = r;
    q.groups[g].C = g_split_ws.part + (long long)r * p.N;
    q.groups[g].R = nullptr;
    r += p.groups[g].M;
    ro.off[g + 1] = r;
  }
  const int st = launch_pipe_cfg<AM>(cfg, q, 1, S, s);
  if (st) return st;
  const long long items = (long long)p.M * cdiv(p.N, 4);
  hipLaunchKernelGGL((gemm_splitk_reduce_kernel<bf16>), dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, p,
                     (const float*)g_split_ws.part, S, ro);
  return check_launch("gemm_splitk_reduce_kernel");
}

// short rows (M = B * T = 992 decoder rows): round 6 loader-wave tiles
// (tools/small_bench.hip -DSB_LW, profiles/r06/small_lw.txt, graph replay):
// N <= 1024 on 64x32 with 2 loader waves (N 512 K 512 5.54 -> 5.12 us, K 2048
// 11.68 -> 9.59), N = 2048 on 64x64 with 4 (8.67 -> 7.84); N 1536 stays on
// the 64x32 16x16x32 ring (7.56; its loader forms 7.3-9.2)
// C5's decode steps (M = 2048 = 256 images x beam 8): 64x64 + 4 loaders on
// every N (profiles/r06/small_lw_c5.txt: N 512 K 512 6.37 -> 5.99 us, K 2048
// 13.16 -> 10.34, N 1536 12.94 -> 11.46)
static int row_short_cfg(const GemmParams& p) {
  if (p.M >= 1536) return 8;
  if (p.N <= 1024) return 9;
  if (p.N <= 1536) return 5;
  return 8;
}

template <int AM>
static int launch_pipe_auto(GemmParams& p, int batch, hipStream_t s) {
  // short rows: the 4-stage 64x64 ring (measured against 1 / 2 / 6 / 8
  // stages and a split-K of 2); up to N = 1536 on 64x32
  // tiles with 16x16x32 MFMA, twice the blocks on the same rows
  // (tools/small_bench.hip -DSB_PIPE, profiles/r05/small_pipe_r5h2.txt,
  // M = 992: N 512 K 512 6.73 -> 5.62 us, K 2048 14.22 -> 12.02, N 1536
  // 8.36 -> 7.55; N 2048 stays on 64x64: 8.64 against 10.76)
  const bool row_short = AM == A_ROW && pipe_row_short(p, batch);
  const int cfg = AM == A_ROW ? (row_short ? row_short_cfg(p) : 3) : pipe_cfg(p, batch);
  const int S = pipe_split_for(p, batch);
  if (S > 1) return launch_pipe_split<AM>(cfg, S, p, s);
  return launch_pipe_cfg<AM>(cfg, p, batch, 1, s);
}

// Weight gradients (fp32 atomics into the arena) of the wide convs / Dense
// layers: the LDS-DMA pipelined form (gemm_pipe_wg_kernel) when the operands
// are 16-B chunked, the m range of a 128-wide tile stays in one filter tap,
// and the reduction is long.
static bool pipe_wg_eligible(const GemmParams& p, int batch, int amode, int bmode, bool vec) {
  if (!g_split_ws.zero || !vec || batch != 1 || bmode != B_KN || p.accumulate != 2 ||
      !p.c_f32 || p.c_mode != C_ROW || p.act != FPNMT_ACT_NONE || p.bias || p.R)
    return false;
  if (p.ngroups > 0 && !p.group_k) return false;
  if (p.M < 64 || p.N < 64 || (p.M < 128 && p.N < 128) || p.N % 8 || p.ldb % 8 || p.ldc < p.N) return false;
  if (amode == A_IM2COL_T) {
    if (p.Cc % 8) return false;  // a 16-B A chunk inside one filter tap
    // 64-channel 3x3 (res2, M = 576, N = 64): the register-staged 64x64 kernel
    // measured faster than every LDS-DMA tile (tools/wg_bench.hip -DWB_W64,
    // profiles/r05/wg_w64.txt: 34.8 us against 38.5 for 128x128, 43.5 for 128x64)
    if (p.Cc < 128 && p.Rk * p.Sk > 1) return false;
  } else if (amode == A_COL) {
    if (p.M % 8 || p.lda % 8) return false;
  } else {
    return false;
  }
  long long kt = 0;
  if (p.ngroups > 0)
    for (int g = 0; g < p.ngroups; ++g) kt += (p.groups[g].K + 63) / 64;
  else
    kt = (p.K + 63) / 64;
  // >= 1024 reduction rows: the res5 weight gradients (K = 1568 at batch 32)
  // gain too (r5 3x3 on 256x128 24.7 us against 30.5; r5 1x1 on 128x128 12.1 /
  // 12.5 against 14.3 / 13.7)
  return kt >= 16;
}

template <int AM, int BM, int BN, int WM, int WN, int NLW = 0>
static int launch_pipe_wg_t(GemmParams& p, hipStream_t s) {
  constexpr int BK = 64;
  p.tiles_m = cdiv(p.M, BM);
  p.tiles_n = cdiv(p.N, BN);
  const long long tiles = (long long)p.tiles_m * p.tiles_n;
  // one block per CU (128 KB of LDS): at most one wave of blocks over the chip
  // (a few blocks past it would cost a whole second block time). k-grouped:
  // the groups' K-tiles end to end (groups[g].start = first K-tile), split
  // evenly across group boundaries (gemm_pipe_wg_kernel).
  const long long cus = cu_count_dispatch();
  const long long want = std::max<long long>(1, cus / tiles);
  long long tot_kt = 0;
  if (p.ngroups > 0) {
    for (int g = 0; g < p.ngroups; ++g) {
      p.groups[g].start = (int)tot_kt;
      tot_kt += cdiv(p.groups[g].K, BK);
    }
  } else {
    tot_kt = cdiv(p.K, BK);
  }
  long long kt_per = std::max<long long>(4, (tot_kt + want - 1) / want);
  // more than one split: partial slabs + ordered reduce (deterministic);
  // fewer, longer splits when the slabs would not fit the workspace
  while ((tot_kt + kt_per - 1) / kt_per > 1 && !slab_fits(p, 1, (tot_kt + kt_per - 1) / kt_per)) kt_per *= 2;
  p.k_per_split = (int)(kt_per * BK);
  p.split_k = (int)((tot_kt + kt_per - 1) / kt_per);
  p.zero16 = g_split_ws.zero;
  const dim3 grid((unsigned)(tiles * p.split_k), 1, 1);
  float* base = p.split_k > 1 ? slab_alloc(p, 1, p.split_k) : nullptr;
  // the folded bias column sums (p.cs_db): split_k x tiles_m x WM partial
  // rows in the deferred arena, else in the workspace after the slabs
  const long long cs_rows = (long long)p.split_k * p.tiles_m * WM;
  p.cs_part = nullptr;
  if (p.cs_db && wg_cs_ok<BM, BN, WM, WN, 32>()) {
    p.cs_part = defer_alloc(cs_rows * p.N);
    if (!p.cs_part && g_split_ws.part) {
      const long long off = base == g_split_ws.part ? (long long)p.split_k * p.M * p.N : 0;
      if (off + cs_rows * p.N <= g_split_ws.part_floats) p.cs_part = g_split_ws.part + off;
    }
  }
  auto fold_bias = [&]() -> int {  // db += the partial rows, in row order
    if (!p.cs_part) return 0;
    colsum_launch((int)cs_rows, p.N, p.cs_part, p.cs_db, s);
    p.cs_db = nullptr;  // consumed: the caller runs no separate column pass
    p.cs_part = nullptr;
    return check_launch("gemm_pipe_wg_kernel colsum");
  };
  if (p.split_k > 1) {
    const GemmParams q = slab_params(p, 1, base);
    hipLaunchKernelGGL((gemm_pipe_wg_kernel<BM, BN, WM, WN, AM, 0, 32, NLW>), grid, dim3(64 * (WM * WN + NLW)), 0, s,
                       q);
    int st = check_launch("gemm_pipe_wg_kernel");
    if (!st) st = launch_wgrad_reduce(p, 1, base, s);
    return st ? st : fold_bias();
  }
  {
    const int st = touch_c(p, 1, s);
    if (st) return st;
  }
  hipLaunchKernelGGL((gemm_pipe_wg_kernel<BM, BN, WM, WN, AM, 0, 32, NLW>), grid, dim3(64 * (WM * WN + NLW)), 0, s, p);
  const int st = check_launch("gemm_pipe_wg_kernel");
  return st ? st : fold_bias();
}

template <int AM>
static int launch_pipe_wg(GemmParams& p, hipStream_t s) {
  // 256x128 halves the dz re-reads on the long reductions (grouped P3-P7
  // head wgrad, M=2304 K=33248: 116 -> 103 us) but is slower on short ones
  // (K=6272: 32 -> 41 us) and on few m-tiles; 128x128 with 8 waves otherwise
  // (measured faster than 4 waves)
  long long kt = 0;
  if (p.ngroups > 0)
    for (int g = 0; g < p.ngroups; ++g) kt += (p.groups[g].K + 63) / 64;
  else
    kt = (p.K + 63) / 64;
  // 64-wide sides (8-chunk LDS rows, round 5, profiles/r05/wg_w64.txt): N = 64
  // (res2 1x1 256->64: 18.1 us against 20.5 on the 64x64 kernel) on 128x64,
  // M = 64 (res2 1x1 64->256: 18.6 against 20.6) on 64x256
  if (p.N < 128) return launch_pipe_wg_t<AM, 128, 64, 2, 2>(p, s);
  if (p.M < 128) return launch_pipe_wg_t<AM, 64, 256, 1, 4>(p, s);
  // conv weight gradients with N >= 256 over >= 1024 rows: 128x256 (half the
  // im2col^T rows per block, whose per-chunk tap gathers are the costly DMA
  // side) — tools/wg_bench.hip -DWB_HALO (profiles/r05/wg_halo.txt): P3 head
  // 60.3 -> 54.1 us, 256->512 at 14^2 34.9 -> 31.6, res5 3x3 24.5 -> 22.2,
  // res4 3x3 21.2 -> 20.6; the same split count. (256x256 on a 2-stage ring:
  // 46.5 us on the P3 head, but its 9 tiles double the ordered-slab bytes.)
  // Only where it keeps the split count (one wave of blocks: fewer tiles =
  // more splits = more ordered-slab bytes): in place of 256x128 (same tile
  // count), and at N >= 512, where the GEMM time saved exceeds the extra slab
  // traffic (256->512 at 14^2: 42.8 -> 31.6 us against ~19 MB more slabs);
  // at N = 256 over 128x128 (res4 3x3) the doubled slabs ate the gain (C2
  // step: wgrad + reduce 2379 -> 2351 us only with it there)
  // round 6 (tools/wg_bench.hip -DWB_LW, profiles/r06/wg_lw.txt): with 8
  // loader waves owning the LDS-DMA the 128x256 tile takes the P3 head 55.4 ->
  // 46.6 us, 256->512 at 14^2 31.8 -> 29.1; the 1x1 (A_COL) 128x128 tiles with
  // 4 loader waves 11.7 -> 11.3 us (r3 1x1 13.0 -> 11.9); the 3x3 128x128 and
  // the 256x128 tiles measured equal or slower with loaders and stay
  const bool wide = p.M >= 1024 && (kt >= 128 || p.M >= 4096) && (AM != A_IM2COL_T || p.Cc % 256 == 0);
  if (AM == A_IM2COL_T && p.N >= 256 && p.M >= 1024 && (wide || p.N >= 512))
    return launch_pipe_wg_t<AM, 128, 256, 2, 4, 8>(p, s);
  if (wide) return launch_pipe_wg_t<AM, 256, 128, 4, 2>(p, s);
  if (AM == A_COL) return launch_pipe_wg_t<AM, 128, 128, 2, 4, 4>(p, s);
  return launch_pipe_wg_t<AM, 128, 128, 2, 4>(p, s);
}

template <typename T>
static int launch_modes(int cfg, GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
#define FPNMT_L(AMv, BMv)                                                                   \
  if (amode == AMv && bmode == BMv) return launch_cfg<T, AMv, BMv>(cfg, p, batch, vec, s);
  FPNMT_L(A_ROW, B_NK)
  FPNMT_L(A_IM2COL, B_NK)
  FPNMT_L(A_ROW, B_KN)
  FPNMT_L(A_COL, B_KN)
  FPNMT_L(A_IM2COL_T, B_KN)
  FPNMT_L(A_COL, B_NK)
#undef FPNMT_L
  return fail(FPNMT_E_UNSUPPORTED, "gemm: operand mode pair not instantiated");
}

// Few blocks over a long K (res4 / res5 3x3 convs and the small FPN levels of
// the batch-32 step: 100-400 blocks x 36-72 K-tiles, every K-tile waiting out
// a load latency): split K into S partial fp32 slabs in the workspace, then
// sum them in split order and run the epilogue (gemm_splitk_reduce_kernel).
static int ws_split_for(const GemmParams& p, int batch, int cfg, int BK) {
  if (!g_split_ws.part || batch != 1 || (p.ngroups > 0 && p.group_k) || p.c_mode != C_ROW ||
      p.accumulate == 2)
    return 1;
  const int nkt = cdiv(p.K, BK);
  const long long blocks = blocks_for(p.M, p.N, batch, cfg);
  // measured (batch-32 step): M=1568 N=512 K=4608 (200 blocks) 69.5 -> 31.5 us;
  // M=6272 N=256 K=1024 (392 blocks, 16 K-tiles) 20.7 -> 28.3 us (slower)
  // M=6272 N=256 K=2304 (392 blocks, 36 K-tiles) 36.6 -> 33.1 us
  if (!((blocks < 320 && nkt >= 24) || (blocks < 512 && nkt >= 32))) return 1;
  int S = (int)((768 + blocks - 1) / blocks);
  S = std::min(S, nkt / 8);
  S = std::min(S, 8);
  while (S > 1 && (long long)S * p.M * p.N > g_split_ws.part_floats) --S;
  return S < 2 ? 1 : S;
}

// C *= act'(M2) in place (batch 1, C_ROW): the M2 operand for launches that
// do not take the pipe kernel's epilogue (bit for bit the same: a 0/1 factor;
// after an accumulating launch it masks the whole sum, which equals masking
// the contribution when the old C already carries the mask)
template <typename T>
__global__ __launch_bounds__(256) void mask_rows_kernel(const GemmParams p) {
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= (long long)p.M * p.N) return;
  const int row = (int)(i / p.N), col = (int)(i - (long long)row * p.N);
  T* c = (T*)p.C + (long long)row * p.ldc + col;
  *c = from_f32<T>(to_f32(*c) * act_mask_from_y(to_f32(((const T*)p.M2)[(long long)row * p.ldr + col]), p.m2_act));
}

template <typename T>
int dispatch_gemm_impl(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s);

template <typename T>
static int dispatch_with_m2(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  if (batch != 1 || p.accumulate == 2 || p.c_f32 || p.ngroups > 0)
    return fail(FPNMT_E_UNSUPPORTED, "gemm: the M2 mask needs batch 1, bf16 C, no atomics");
  // scattered rows (strided 1x1 bwd-data) only reach the register-staged
  // kernel, whose row epilogue applies M2 at the scattered row
  if (p.c_mode == C_SCATTER) return 1;
  if (pipe_eligible<T>(p, batch, amode, bmode, vec) && pipe_split_for(p, batch) == 1) return 1;  // the pipe epilogue applies M2
  GemmParams q = p;
  q.M2 = nullptr;
  const int st = dispatch_gemm_impl<T>(q, batch, amode, bmode, vec, s);
  if (st) return st;
  const long long n = (long long)p.M * p.N;
  hipLaunchKernelGGL((mask_rows_kernel<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
  return check_launch("mask_rows_kernel");
}

// Dense weight gradients (A = x rows, B = dz rows, fp32 C accumulated: every
// LinearFn / grouped-projection / view-projection wgrad of the transformer)
// inside a deferred-reduction region: queued per batch entry and run at the
// flush as grouped launches of whole-K 128x128 tiles (gemm_wg_jobs_kernel),
// instead of one under-filled launch each (64 tiles of 512x512 at M = 992
// rows, split-K slabs). Opt-in: only GEMMs entered through fpnmt_gemm_wgrad
// are queued (the caller keeps A and B alive until the flush: ops._wgrad,
// L.defer_keep); a plain fpnmt_gemm always launches immediately.
static bool wg_job_eligible(const GemmParams& p, int batch, int amode, int bmode, bool vec) {
  if (!wgrad_queue_ok() || !defer_active() || !g_split_ws.zero || !vec) return false;
  if (amode != A_COL || bmode != B_KN || !p.c_f32 || (p.accumulate != 1 && p.accumulate != 2)) return false;
  if (p.act != FPNMT_ACT_NONE || p.bias || p.R || p.col_scale || p.M2 || p.ngroups > 0 || p.c_mode != C_ROW ||
      p.drop_p > 0.f)
    return false;
  if (batch > 1 && (p.batch_inner != 1 || !c_batches_disjoint(p, batch))) return false;
  if (p.M < 128 || p.N < 128 || p.K < 1 || p.M % 8 || p.N % 8 || p.lda % 8 || p.ldb % 8 || (p.a_so | p.b_so) % 8)
    return false;
  return (((uintptr_t)p.A | (uintptr_t)p.B) & 15) == 0;
}

static int defer_wg_jobs(const GemmParams& p, int batch, hipStream_t s) {
  for (int z = 0; z < batch; ++z) {
    DefGemmJob J{};
    J.A = (const bf16*)p.A + z * p.a_so;
    J.B = (const bf16*)p.B + z * p.b_so;
    J.C = (float*)p.C + z * p.c_so;
    J.M = p.M; J.N = p.N; J.K = p.K;
    J.lda = (int)p.lda; J.ldb = (int)p.ldb; J.ldc = (int)p.ldc;
    J.alpha = p.alpha;
    const int st = defer_gemm_job(J, s);
    if (st) return st;
  }
  return 0;
}

// Strided 1x1 bwd-data (C_SCATTER: row m of the (n, ho, wo) grid lands at
// (n, s ho, s wo) of dx): the register-staged kernel is the only one with the
// scattered row epilogue, and at the projection shortcuts' shapes (M = 6272,
// N = 512, K = 1024 at C2; 784 64x64 tiles) it ran 56 us for 6.6 GFLOP. Round
// 6: the product goes to the LDS-DMA pipe kernels as a 1x1 implicit GEMM over
// the dz rows into fp32 rows in the workspace, then scatter_rows_kernel applies
// the scattered epilogue (M2 mask at the scattered row, bf16 store or
// read-modify-write) with the register-staged kernel's arithmetic: one
// rounding of acc (+ old) per element.
static __global__ __launch_bounds__(256) void scatter_rows_kernel(const GemmParams p, const float* __restrict__ src) {
  const int g8 = p.N / 8;
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= (long long)p.M * g8) return;
  const int row = (int)(i / g8), col = (int)(i - (long long)row * g8) * 8;
  const uint32_t n = fdiv((uint32_t)row, p.fd_sHoWo);
  const int rem = row - (int)n * (int)p.fd_sHoWo.d;
  const uint32_t ho = fdiv((uint32_t)rem, p.fd_sWo);
  const int wo = rem - (int)ho * (int)p.fd_sWo.d;
  const long long orow = ((long long)n * p.scat_Hd + (long long)ho * p.scat_s) * p.scat_Wd + (long long)wo * p.scat_s;
  const f32x4 lo = *(const f32x4*)(src + (long long)row * p.N + col), hi = *(const f32x4*)(src + (long long)row * p.N + col + 4);
  float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  if (p.M2) {
    const bf16x8 yv = *(const bf16x8*)((const bf16*)p.M2 + orow * p.ldr + col);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= act_mask_from_y((float)yv[j], p.m2_act);
  }
  bf16* Cp = (bf16*)p.C + orow * p.ldc + col;
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
}

// the pipe form of a C_SCATTER GEMM when every operand allows it (1 = not taken)
static int scatter_via_pipe(const GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  if (batch != 1 || amode != A_ROW || bmode != B_NK || p.bias || p.R || p.act != FPNMT_ACT_NONE ||
      p.drop_p > 0.f || p.alpha != 1.f || p.col_scale || p.c_f32 || (p.accumulate != 0 && p.accumulate != 1) ||
      p.ngroups > 0 || p.K % 64 || p.N % 8 || p.ldc % 8 || (p.M2 && p.ldr % 8))
    return 1;
  if ((((uintptr_t)p.C | (uintptr_t)p.M2) & 15) || !g_split_ws.part || (long long)p.M * p.N > g_split_ws.part_floats)
    return 1;
  GemmParams q = p;  // dz rows as a 1x1 implicit GEMM (a 1-wide image of M rows)
  q.c_mode = C_ROW;
  q.M2 = nullptr;
  q.c_f32 = 1;
  q.accumulate = 0;
  q.C = g_split_ws.part;
  q.ldc = p.N;
  q.c_so = q.c_si = 0;
  q.H = q.Ho = p.M; q.W = q.Wo = 1; q.Cc = p.K; q.Rk = q.Sk = 1; q.sh = q.sw = 1; q.pt = q.pl = 0;
  q.fd_HoWo = make_fastdiv(p.M); q.fd_Wo = make_fastdiv(1); q.fd_C = make_fastdiv(p.K); q.fd_S = make_fastdiv(1);
  if (!pipe_eligible<bf16>(q, 1, A_IM2COL, B_NK, vec) || pipe_split_for(q, 1) != 1) return 1;
  log_gemm<bf16>(p, batch, amode, bmode, 160 + pipe_cfg(q, 1));
  const int st = launch_pipe_auto<A_IM2COL>(q, 1, s);
  if (st) return st;
  const long long items = (long long)p.M * (p.N / 8);
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, p,
                     (const float*)g_split_ws.part);
  return check_launch("scatter_rows_kernel");
}

// Tall row GEMMs the row pipe class does not take (M > 4096 rows, fewer than
// 128 tiles of 128x256: the encoder views' K / V projection dgrads, M = 6272,
// N = 512, K = 6144 at C2) as a 1x1 implicit GEMM over the A rows, which the
// conv pipe classes tile by their own tile-count rules (128x128 loader tile
// there) instead of the register-staged 64x64 kernel. Same epilogue fields;
// 1 = not taken.
template <typename T>
static int rows_via_im2col(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  if constexpr (!std::is_same<T, bf16>::value) return 1;
  if (batch != 1 || amode != A_ROW || bmode != B_NK || p.c_mode != C_ROW || p.ngroups > 0 || p.M <= 4096 ||
      p.N < 256 || p.K % 64 || p.lda != p.K || (p.a_so | p.a_si) != 0)
    return 1;
  GemmParams q = p;
  q.H = q.Ho = p.M; q.W = q.Wo = 1; q.Cc = p.K; q.Rk = q.Sk = 1; q.sh = q.sw = 1; q.pt = q.pl = 0;
  q.fd_HoWo = make_fastdiv(p.M); q.fd_Wo = make_fastdiv(1); q.fd_C = make_fastdiv(p.K); q.fd_S = make_fastdiv(1);
  if (!pipe_eligible<bf16>(q, 1, A_IM2COL, B_NK, vec)) return 1;
  if (q.M2 && pipe_split_for(q, 1) != 1) return 1;  // the M2 mask rides in the pipe epilogue only
  log_gemm<bf16>(p, batch, amode, bmode, 170 + pipe_cfg(q, 1));
  return launch_pipe_auto<A_IM2COL>(q, 1, s);
}

template <typename T>
int dispatch_gemm_impl(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  if constexpr (std::is_same<T, bf16>::value) {
    if (wg_job_eligible(p, batch, amode, bmode, vec)) {
      log_gemm<T>(p, batch, amode, bmode, 150);
      return defer_wg_jobs(p, batch, s);
    }
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (p.c_mode == C_SCATTER) {
      const int st = scatter_via_pipe(p, batch, amode, bmode, vec, s);
      if (st != 1) return st;
    }
  }
  if (p.M2) {
    const int st = dispatch_with_m2<T>(p, batch, amode, bmode, vec, s);
    if (st != 1) return st;
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (pipe_eligible<T>(p, batch, amode, bmode, vec)) {
      log_gemm<T>(p, batch, amode, bmode,
                  130 + (amode == A_ROW ? (pipe_row_short(p, batch) ? row_short_cfg(p) : 3) : pipe_cfg(p, batch)));
      return amode == A_IM2COL ? launch_pipe_auto<A_IM2COL>(p, batch, s) : launch_pipe_auto<A_ROW>(p, batch, s);
    }
    const int st = rows_via_im2col<T>(p, batch, amode, bmode, vec, s);
    if (st != 1) return st;
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (pipe_wg_eligible(p, batch, amode, bmode, vec)) {
      const int st = amode == A_IM2COL_T ? launch_pipe_wg<A_IM2COL_T>(p, s) : launch_pipe_wg<A_COL>(p, s);
      log_gemm<T>(p, batch, amode, bmode, 110);
      return st;
    }
  }
  const int cfg = choose_cfg(amode, bmode, p.M, p.N, p.K, batch, p.accumulate, p.c_mode);
  if (cfg == CFG_SMALL) {
    if (p.accumulate == 2) {  // atomic C: no split needed (and no workspace)
      // one writer per element: a read-modify-write is the same sum on one
      // stream, at a fraction of the per-element atomics' cost
      if (batch == 1) p.accumulate = 1;
      p.split_k = 1;
      p.k_per_split = p.K;
      p.ws_part = nullptr;
      {
        const int st = touch_c(p, batch, s);
        if (st) return st;
      }
      dim3 grid(cdiv(p.M, 32) * cdiv(p.N, 64), 1, batch);
      log_gemm<T>(p, batch, amode, bmode, cfg);
      hipLaunchKernelGGL((gemm_small_kernel<T, 4>), grid, dim3(256), 0, s, p);
      return check_launch("gemm_small_kernel");
    }
    const int st = launch_small<T>(p, batch, s);
    log_gemm<T>(p, batch, amode, bmode, cfg);
    return st;
  }
  int BK = kCfg[cfg].bk;
  if (cfg == CFG_128_128_64 && !(amode == A_IM2COL || amode == A_ROW || amode == A_IM2COL_T || amode == A_COL)) BK = 32;
  if (cfg == CFG_64_64_64 && !(amode == A_IM2COL || amode == A_ROW || amode == A_IM2COL_T)) BK = 32;
  BK = bk_of<T>(BK);
  // split-K (only with fp32 atomic accumulation)
  if (p.ngroups > 0 && p.group_k) {
    // k-grouped: every group's reduction range is cut into splits of kt_per
    // K-tiles; grid.y enumerates the splits of all groups
    long long tot_kt = 0;
    for (int g = 0; g < p.ngroups; ++g) tot_kt += cdiv(p.groups[g].K, BK);
    const long long blocks = blocks_for(p.M, p.N, batch, cfg);
    const long long want = (768 + blocks - 1) / blocks;
    int kt_per = (int)((tot_kt + want - 1) / want);
    if (kt_per < 4) kt_per = 4;
    int sp = 0;
    for (;;) {
      sp = 0;
      for (int g = 0; g < p.ngroups; ++g) {
        p.groups[g].start = sp;
        sp += cdiv(cdiv(p.groups[g].K, BK), kt_per);
      }
      if (sp <= p.ngroups || slab_fits(p, batch, sp)) break;
      kt_per *= 2;
    }
    p.k_per_split = kt_per * BK;
    p.split_k = sp;
  } else if (p.accumulate == 2) {
    const int nkt = cdiv(p.K, BK);
    const long long blocks = blocks_for(p.M, p.N, batch, cfg);
    int split = p.split_k;
    if (split <= 0) {
      split = (int)((768 + blocks - 1) / blocks);  // 256 / 384 measured slower
      int max_split = nkt / 4;  // keep >= 4 K-tiles per split
      if (split > max_split) split = max_split;
      if (split < 1) split = 1;
    }
    int kt_per = cdiv(nkt, split);
    while (cdiv(nkt, kt_per) > 1 && !slab_fits(p, batch, cdiv(nkt, kt_per))) kt_per *= 2;
    p.k_per_split = kt_per * BK;
    p.split_k = cdiv(nkt, kt_per);
    if (p.split_k < 1) p.split_k = 1;
    // unsplit launch whose batch entries own disjoint C slices: one writer
    // per element -> RMW instead of atomics (e.g. the encoder's M = 32 weight
    // gradients: 512x512 fp32 by atomics took 12.7 us; the views' grouped
    // output-projection gradients, batch 4 of them, likewise)
    if (p.split_k == 1 && (batch == 1 || c_batches_disjoint(p, batch))) p.accumulate = 1;
  } else {
    const int S = ws_split_for(p, batch, cfg, BK);
    if (S > 1) {
      // partial slabs (no epilogue) into the workspace, then sum + epilogue
      GemmParams q = p;
      const int nkt = cdiv(p.K, BK);
      const int kt_per = cdiv(nkt, S);
      q.split_k = cdiv(nkt, kt_per);
      q.k_per_split = kt_per * BK;
      q.bias = nullptr;
      q.col_scale = nullptr;
      q.R = nullptr;
      q.act = FPNMT_ACT_NONE;
      q.drop_p = 0.f;
      q.drop_seed_dev = nullptr;
      q.alpha = 1.f;
      q.c_f32 = 1;
      q.accumulate = 0;
      q.C = g_split_ws.part;
      q.ldc = p.N;
      q.c_so = q.c_si = 0;
      q.c_split = (long long)p.M * p.N;  // p.M = the groups' rows in total
      RowOffsets ro{};
      for (int g = 0, r = 0; g < p.ngroups; ++g) {  // groups' slab rows back to back
        ro.off[g] = r;
        q.groups[g].C = g_split_ws.part + (long long)r * p.N;
        q.groups[g].R = nullptr;
        r += p.groups[g].M;
        ro.off[g + 1] = r;
      }
      log_gemm<T>(q, batch, amode, bmode, cfg);
      int st = launch_modes<T>(cfg, q, batch, amode, bmode, vec, s);
      if (st) return st;
      const long long items = (long long)p.M * cdiv(p.N, 4);
      hipLaunchKernelGGL((gemm_splitk_reduce_kernel<T>), dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, p,
                         (const float*)g_split_ws.part, q.split_k, ro);
      return check_launch("gemm_splitk_reduce_kernel");
    }
    p.split_k = 1;
    p.k_per_split = ((p.K + BK - 1) / BK) * BK;
    if (p.k_per_split == 0) p.k_per_split = BK;
  }
  if (p.accumulate == 2 && p.split_k > 1 && slab_fits(p, batch, p.split_k)) {
    // several adders per C element: partial slabs + ordered reduce
    float* base = slab_alloc(p, batch, p.split_k);
    GemmParams q = slab_params(p, batch, base);
    log_gemm<T>(q, batch, amode, bmode, cfg);
    const int st = launch_modes<T>(cfg, q, batch, amode, bmode, vec, s);
    return st ? st : launch_wgrad_reduce(p, batch, base, s);
  }
  if (p.accumulate != 0 && p.c_f32) {
    const int st = touch_c(p, batch, s);
    if (st) return st;
  }
  log_gemm<T>(p, batch, amode, bmode, cfg);
  return launch_modes<T>(cfg, p, batch, amode, bmode, vec, s);
}

}  // namespace fpnmt
