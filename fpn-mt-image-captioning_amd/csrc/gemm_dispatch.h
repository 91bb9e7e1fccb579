// Host-side tile-config selection and launch for gemm_kernel<T,...>.
// Included once per element type (gemm_bf16.hip, gemm_f32.hip) so the two
// instantiation sets compile in parallel.
#pragma once
#include "gemm_impl.h"

namespace fpnmt {

struct TileCfg {
  int bm, bn;
};

template <typename T, int BM, int BN, int WM, int WN, int AM, int BMODE>
static int launch_one(GemmParams& p, int batch, bool vec, hipStream_t s) {
  p.tiles_m = cdiv(p.M, BM);
  p.tiles_n = cdiv(p.N, BN);
  dim3 grid(p.tiles_m * p.tiles_n, p.split_k, batch);
  dim3 block(64 * WM * WN);
  if (vec)
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, AM, BMODE, true>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, AM, BMODE, false>), grid, block, 0, s, p);
  return check_launch("gemm_kernel");
}

// Config table per operand-mode pair. Index: 0=128x128, 1=128x64, 2=64x128, 3=64x64, 4=32x32
template <typename T, int AM, int BMODE>
static int launch_cfg(int cfg, GemmParams& p, int batch, bool vec, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_one<T, 128, 128, 2, 2, AM, BMODE>(p, batch, vec, s);
    case 1: return launch_one<T, 128, 64, 2, 2, AM, BMODE>(p, batch, vec, s);
    case 2: return launch_one<T, 64, 128, 2, 2, AM, BMODE>(p, batch, vec, s);
    case 3: return launch_one<T, 64, 64, 2, 2, AM, BMODE>(p, batch, vec, s);
    default: return launch_one<T, 32, 32, 1, 1, AM, BMODE>(p, batch, vec, s);
  }
}

static const TileCfg kCfgs[5] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}, {32, 32}};

// Pick the largest tile that still yields >= ~1 block per CU; tiny problems
// fall back to 32x32 (one wave) tiles.
static int choose_cfg(int M, int N, long long batch) {
  if (M <= 32 && N <= 32) return 4;
  for (int c = 0; c < 4; ++c) {
    long long blocks = (long long)cdiv(M, kCfgs[c].bm) * cdiv(N, kCfgs[c].bn) * batch;
    // avoid tiles that are mostly padding
    if (kCfgs[c].bm > 64 && M <= 64) continue;
    if (kCfgs[c].bn > 64 && N <= 64) continue;
    if (blocks >= 240) return c;
  }
  if (M <= 32 || N <= 32) return 4;
  return 3;
}

template <typename T>
int dispatch_gemm_impl(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  constexpr int BK = TT<T>::BK;
  int cfg = choose_cfg(p.M, p.N, batch);
  // split-K (only with fp32 atomic accumulation)
  if (p.accumulate == 2) {
    const int nkt = cdiv(p.K, BK);
    long long blocks = (long long)cdiv(p.M, kCfgs[cfg].bm) * cdiv(p.N, kCfgs[cfg].bn) * batch;
    int split = p.split_k;
    if (split <= 0) {
      split = (int)((512 + blocks - 1) / blocks);
      int max_split = nkt / 4;  // keep >= 4 K-tiles per split
      if (split > max_split) split = max_split;
      if (split < 1) split = 1;
    }
    int kt_per = cdiv(nkt, split);
    p.k_per_split = kt_per * BK;
    p.split_k = cdiv(nkt, kt_per);
    if (p.split_k < 1) p.split_k = 1;
  } else {
    p.split_k = 1;
    p.k_per_split = ((p.K + BK - 1) / BK) * BK;
    if (p.k_per_split == 0) p.k_per_split = BK;
  }
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

}  // namespace fpnmt
