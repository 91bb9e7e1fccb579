// Halo-staged weight gradient of a 3x3 stride-1 'same' convolution:
//   dW[(r*3 + s)*C + c][k] += sum over pixels (img, h, w) of
//     x[img][h + r - 1][w + s - 1][c] * dz[img][h][w][k]
// gemm_pipe_wg_kernel DMAs the im2col^T operand: every input pixel crosses
// L2 -> LDS once per tap (9x), 48 KB per 4.2 MFLOP K-tile of the 256x128
// tile, and the kernel runs at the LDS-DMA fill rate. Here a block owns 32
// input channels x ALL nine taps (M = 288) x 128 output channels; a K-tile
// is RT output rows x WS pixel slots (64 pixels, WS = W rounded up to a power
// of two >= 8); the block stages the (RT + 2) x (WS + 2) x 32-channel x patch
// once ([pixel][32 ch], 64-B rows: four consecutive pixel rows cover the 64
// banks) and the dz tile ([pixel][128 ch], the weight-gradient kernel's
// swizzled B image), ~29 KB per 4.1 MFLOP. Wave w = tap (r, s) reads its A
// operand as the patch shifted by (r, s) with transposing LDS reads; split-K
// over blocks into fp32 slabs (summed in split order elsewhere).
// Not part of the library (tools/wg_bench.hip -DWB_HALO).
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_pipe.h"

namespace fpnmt {

constexpr int HALO_MAXLV = 5;
struct HaloLevel {
  const bf16* x;   // [n][H][W][C]
  const bf16* dz;  // [n][H][W][N]
  int H, W, WS, lws, RT, rowtiles, t0;  // WS = 1 << lws; K-tiles of the level: n * rowtiles from t0
};
struct HaloArgs {
  HaloLevel lv[HALO_MAXLV];
  int nlv;
  int n, C, N;
  int tot_kt, kt_per, splits;
  int cgroups, ngroups;  // C / 32, N / 128
  float* slab;           // [split][9 C][N]
  const void* zero;      // >= 16 B of zeros
};

template <int STAGES>
__global__ __launch_bounds__(576) void wg_halo3x3_kernel(const HaloArgs a) {
  typedef bf16 T;
  constexpr int NT = 576, CB = 32, NB = 128;
  constexpr int A_BYTES = 2 * NT * 16;  // patch (<= 198 pixels x 64 B) + the second DMA round's tail
  constexpr int B_BYTES = 2 * NT * 16;  // dz tile (64 pixels x 256 B = 1024 chunks) + tail
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int PER_STAGE = 4;  // DMA instructions per thread per stage
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // the tap
  const int tr_ = wave / 3, ts_ = wave - 3 * tr_;
  const int lh = lane >> 5, lr = lane & 31;
  const int ntile = a.cgroups * a.ngroups;
  const int wv = xcd_remap(blockIdx.x, ntile * a.splits);
  const int split = wv / ntile, bid = wv - split * ntile;
  const int cg = bid / a.ngroups, ng = bid - cg * a.ngroups;
  const int c0 = cg * CB, n0 = ng * NB;
  const int kt0 = split * a.kt_per;
  const int nk = max(0, min(a.kt_per, a.tot_kt - kt0));
  const T* zero = (const T*)a.zero;
  typedef __attribute__((address_space(3))) void lds_void;

  auto level_of = [&](int kt) {
    HaloLevel L = a.lv[0];
#pragma unroll
    for (int q = 1; q < HALO_MAXLV; ++q)
      if (q < a.nlv && kt >= a.lv[q].t0) L = a.lv[q];
    return L;
  };
  auto issue = [&](int kt, int stage) {
    const HaloLevel L = level_of(kt0 + kt);
    const int local = kt0 + kt - L.t0;
    const int img = local / L.rowtiles;
    const int h0 = (local - img * L.rowtiles) * L.RT;
    char* sb = smem + stage * STAGE_BYTES;
    const int pw = L.WS + 2, npix = (L.RT + 2) * pw;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // the x patch, [pixel][32 channels]
      const int q = i * NT + tid;
      const int pix = q >> 2, cc = q & 3;
      const int pr = pix / pw, pc = pix - pr * pw;
      const int h = h0 - 1 + pr, w = pc - 1;
      const T* src = zero;
      if (pix < npix && (unsigned)h < (unsigned)L.H && (unsigned)w < (unsigned)L.W)
        src = L.x + ((long long)(img * L.H + h) * L.W + w) * a.C + c0 + 8 * cc;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (i * NT + wave * 64) * 16), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // the dz tile, [pixel][128 channels], chunk slot ^ wg_sw(pixel)
      const int q = i * NT + tid;
      const int pk = q >> 4, cn = (q & 15) ^ wg_sw(q >> 4);
      const int rt = pk >> L.lws, slot = pk & (L.WS - 1);
      const int h = h0 + rt;
      const T* src = zero;
      if (q < 1024 && slot < L.W && h < L.H)
        src = L.dz + ((long long)(img * L.H + h) * L.W + slot) * a.N + n0 + 8 * cn;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + A_BYTES + (i * NT + wave * 64) * 16), 16,
                                       0, 0);
    }
  };

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  const int g16 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  auto compute = [&](int kt, int stage) {
    const HaloLevel L = level_of(kt0 + kt);
    const char* As = smem + stage * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
    const int pw = L.WS + 2;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kk = 16 * ks + 8 * lh + tq;
      const int rt = kk >> L.lws, slot = kk & (L.WS - 1);
      const int pix = (rt + tr_) * pw + slot + ts_;
      const char* ap = As + pix * 64 + (16 * g16 + 4 * tp) * 2;
      const s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(ap));
      const s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(ap + 4 * 64));
      __attribute__((ext_vector_type(8))) short a8 = {alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
      const bf16x8 fa = __builtin_bit_cast(bf16x8, a8);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = 32 * t + 16 * g16 + 4 * tp;
        const char* bp = Bs + kk * 256 + ((((col >> 3) ^ wg_sw(kk)) << 4) | ((col & 7) << 1));
        const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(bp));
        const s16x4 bhi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(bp + 4 * 256));
        __attribute__((ext_vector_type(8))) short b8 = {blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]};
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, __builtin_bit_cast(bf16x8, b8), acc[t], 0, 0, 0);
      }
    }
  };

#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < nk) issue(i, i);
  for (int t = 0; t < nk; ++t) {
    const int ahead = nk - 1 - t;
    if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
    else if (STAGES > 3 && ahead == 1) wait_vmcnt<PER_STAGE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every thread's DMA of tile t landed; stage (t - 1) % STAGES is free
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    compute(t, t % STAGES);
  }
  float* slab = a.slab + (long long)split * 9 * a.C * a.N;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * lh;
      slab[(long long)(wave * a.C + c0 + row) * a.N + n0 + 32 * t + lr] = acc[t][i];
    }
}

}  // namespace fpnmt
