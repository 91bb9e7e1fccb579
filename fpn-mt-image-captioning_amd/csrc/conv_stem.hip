// ResNet stem: the 7x7 stride-2 conv over the 3-channel NHWC image
// (keras-resnet conv1 after ZeroPadding2D(3); models/resnet.py, reference
// models/resnet.py:78-112). It is the one backbone conv whose implicit-GEMM
// rows (K = 7*7*3 = 147) do not vectorise: the generic loader falls back to
// one 2-byte load per element (R50-FPN forward, batch 64: 202 us = 75 TF for a
// layer that moves ~120 MB).
//
// A block owns a tile of 8 output rows x 32 output columns (x 64 channels).
// Its 21 input rows are staged in LDS with the channels padded 3 -> 4, so for
// output column j and kernel row r the 7 taps x 4 channels are 28 consecutive
// elements starting at element 8*j: every 8-element MFMA k-group (2 taps x 4
// channels) is one 16-B aligned ds_read_b128 (conflict-free: lanes are 16 B
// apart). K = 7 rows x 4 groups = 14 k-steps of v_mfma_f32_32x32x16_bf16;
// the 4th group's second tap (tap 7) is zeroed in registers, the pad channel
// holds zeros in LDS and zero weights. The input rows arrive as aligned 16-B
// global loads (absolute 8-element chunks, each entirely inside or outside
// the tensor) scattered into the padded layout.
//
// Roles are swapped (A = weights, B = pixels): each lane ends with 4
// consecutive output channels of one pixel, staged in LDS so the tile leaves
// as full 128-B pixel lines (16-B stores). Waves split the 64 channels in
// halves (56 weight VGPRs). The block is persistent over tiles: weights stay
// in registers for its lifetime and the next tile's input is loaded while the
// current one computes.
#include <algorithm>
#include <cstdlib>
#include "common.h"

namespace fpnmt {

namespace {
constexpr int ST_TH = 8;                   // output rows per tile (2 row groups of 4)
constexpr int ST_TW = 32;                  // output columns per tile (MFMA N)
constexpr int ST_ROWS = 2 * ST_TH + 5;     // staged input rows (21)
constexpr int ST_PIX = 2 * (ST_TW - 1) + 7;  // staged pixels per row (69)
constexpr int ST_SEG = 3 * ST_PIX;         // input elements per staged row (207)
constexpr int ST_RP = 280;                 // staged row pitch: 69 px x 4 ch, padded to 16 B
constexpr int ST_CPR = 27;                 // 8-element global chunks per staged row (covers 207 + misalign)
constexpr int ST_ITEMS = ST_ROWS * ST_CPR;  // 567
constexpr int ST_PF = (ST_ITEMS + 255) / 256;  // chunks per thread (3)
static_assert(ST_PIX == 69 && ST_ROWS * ST_PIX <= 1449, "pixel-pass division constant (950 / 2^16 = 1/69)");
constexpr int ST_KS = 14;                  // k-steps: 7 kernel rows x 4 groups of 8 / 2

struct StemArgs {
  const unsigned short* x;  // bf16 (n, h, w, 3), 16-B aligned, n*h*w*3 % 8 == 0
  const unsigned short* w;  // bf16 OHWI (k, 7, 7, 3)
  const float* scale;       // per output channel or null
  const float* bias;        // per output channel or null
  unsigned short* y;        // bf16 (n, ho, wo, k)
  int n, h, w_, ho, wo, k, pt, pl, act;
  float act_alpha;
  int tiles_h, tiles_w, tiles;
  int total;  // n*h*w*3
};

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

__device__ __forceinline__ void stem_tile_coords(const StemArgs& a, int t, int& img, int& ho0, int& wo0) {
  wo0 = (t % a.tiles_w) * ST_TW;
  t /= a.tiles_w;
  ho0 = (t % a.tiles_h) * ST_TH;
  img = t / a.tiles_h;
}

// chunk u of this thread for tile (img, ho0, wo0): staged row hh, absolute
// element index cs of its first element (multiple of 8), row-segment start E
// and the row's first element R0; ok = the chunk lies inside the tensor and
// its row inside the image
struct StemChunk {
  int hh, cs, E, R0;
  bool row_ok, ok;
};
__device__ __forceinline__ StemChunk stem_chunk(const StemArgs& a, int tid, int u, int img, int ho0, int wo0) {
  StemChunk c;
  const int item = tid + 256 * u;
  c.hh = item / ST_CPR;
  const int ci = item - c.hh * ST_CPR;
  const int hi = 2 * ho0 - a.pt + c.hh;
  c.row_ok = item < ST_ITEMS && (unsigned)hi < (unsigned)a.h;
  c.R0 = (img * a.h + hi) * (3 * a.w_);
  c.E = c.R0 + 3 * (2 * wo0 - a.pl);
  c.cs = ((c.E >> 3) << 3) + 8 * ci;  // arithmetic shift: floor for negative E
  c.ok = c.row_ok && c.cs >= 0 && c.cs + 8 <= a.total;
  return c;
}

__device__ __forceinline__ void stem_prefetch(const StemArgs& a, int t, u32x4 (&pf)[ST_PF]) {
  int img, ho0, wo0;
  stem_tile_coords(a, t, img, ho0, wo0);
  // opaque thread index: keeps the per-chunk index math from being hoisted
  // out of the tile loop as loop-invariant registers
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int u = 0; u < ST_PF; ++u) {
    const StemChunk c = stem_chunk(a, tid, u, img, ho0, wo0);
    // unconditional 16-B load (chunk 0 when outside); masked at the LDS write
    pf[u] = *(const u32x4*)(a.x + (c.ok ? c.cs : 0));
  }
}

template <int ACT>
__global__ __launch_bounds__(256, 3) void stem7x7s2_kernel(StemArgs a) {
  constexpr int OP = 72;  // output stage pitch (elements): 144 B, 2-way banked writes
  static_assert(ST_TH * ST_TW * OP >= 64 * 147, "weight staging fits the output stage");
  static_assert(ST_TH * ST_TW * OP >= ST_ITEMS * 8, "chunk staging fits the output stage");
  __shared__ __attribute__((aligned(16))) unsigned short raw[ST_ROWS * ST_RP];
  __shared__ __attribute__((aligned(16))) unsigned short ost[ST_TH * ST_TW * OP];
  __shared__ __attribute__((aligned(16))) float s_bias[64], s_scale[64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nl = lane & 31, hf = lane >> 5;
  const int chh = wave & 1;  // channel half of the 64-channel chunk
  const int rg = wave >> 1;  // row group: output rows 4*rg .. 4*rg+3 of the tile
  const int z = blockIdx.y;  // 64-channel chunk of the output
  // prologue: the weight block, the first tile's input and the per-channel
  // bias/scale are all requested before any of them is waited for (one
  // global latency instead of three)
  constexpr int WC = 64 * 147 / 8;  // 1176 16-B chunks (contiguous, 16-B aligned)
  constexpr int WU = (WC + 255) / 256;
  const u32x4* wz = (const u32x4*)(a.w + (long long)64 * z * 147);
  u32x4 wv[WU];
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    const int i = threadIdx.x + 256 * u;
    wv[u] = wz[i < WC ? i : 0];
  }
  u32x4 pf[ST_PF];
  int tile = blockIdx.x;
  stem_prefetch(a, tile < a.tiles ? tile : 0, pf);
  const int ch = 64 * z + (threadIdx.x & 63);
  const float bias_v = a.bias ? a.bias[ch] : 0.f;
  const float scale_v = a.scale ? a.scale[ch] : 1.f;
  // pad channel (and the row pitch tail) must read as zeros
  for (int i = threadIdx.x; i < ST_ROWS * ST_RP / 8; i += 256) ((u32x4*)raw)[i] = u32x4{0u, 0u, 0u, 0u};
  // weights into the output stage (free until the first tile)
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < WC) ((u32x4*)ost)[i] = wv[u];
  }
  if (threadIdx.x < 64) {
    s_bias[threadIdx.x] = bias_v;
    s_scale[threadIdx.x] = scale_v;
  }
  __syncthreads();
  // weight operand: wreg[ks] = 8 k-values of group (kernel row ks/2,
  // t = 2*(ks&1) + hf) for output channel 64z + 32chh + nl: taps 2t, 2t+1 x
  // channels 0..3 (channel 3 and tap 7 are zero)
  bf16x8 wreg[ST_KS];
  {
    const unsigned short* wrow = ost + (32 * chh + nl) * 147;
#pragma unroll
    for (int ks = 0; ks < ST_KS; ++ks) {
      const int r = ks >> 1, t = 2 * (ks & 1) + hf;
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int sx = 2 * t + (e >> 2), c = e & 3;
        const bool ok = sx <= 6 && c < 3;
        const unsigned short u = wrow[r * 21 + (ok ? sx * 3 + c : 0)];
        v[e] = __builtin_bit_cast(bf16, (unsigned short)(ok ? u : 0));
      }
      wreg[ks] = v;
    }
  }
  for (; tile < a.tiles; tile += gridDim.x) {
    int img, ho0, wo0;
    stem_tile_coords(a, tile, img, ho0, wo0);
    __syncthreads();  // previous tile's operand and stage reads are done
    // (1) the chunks as loaded -> the output stage (free until the compute
    // phase): row hh holds elements floor8(E) .. +216 of its input row
    unsigned short* craw = ost;
#pragma unroll
    for (int u = 0; u < ST_PF; ++u) {
      const int item = threadIdx.x + 256 * u;
      if (item < ST_ITEMS) ((u32x4*)craw)[item] = pf[u];
    }
    __syncthreads();
    // (2) one staged pixel per step: its 3 elements (row-segment offset
    // (E mod 8) + 3p) -> one 8-B write of the channel-padded layout; pixels
    // outside the image (or rows outside it) -> zeros
    const int rowm = (img * a.h + 2 * ho0 - a.pt) * 3 * a.w_ + 3 * (2 * wo0 - a.pl);  // E of row 0 (mod 8 used)
#pragma unroll
    for (int pj = 0; pj < (ST_ROWS * ST_PIX + 255) / 256; ++pj) {
      const int pi = threadIdx.x + 256 * pj;
      if (pi >= ST_ROWS * ST_PIX) break;
      const int hh = (int)__umul24((unsigned)pi, 950u) >> 16;  // pi / 69 for pi < 1449
      const int px = pi - (int)__umul24((unsigned)hh, (unsigned)ST_PIX);
      const int hi = 2 * ho0 - a.pt + hh, wi = 2 * wo0 - a.pl + px;
      const bool ok = (unsigned)hi < (unsigned)a.h && (unsigned)wi < (unsigned)a.w_;
      const int d = (rowm + (int)__umul24((unsigned)hh, (unsigned)(3 * a.w_))) & 7;  // E mod 8 of row hh
      const unsigned short* src = craw + hh * (8 * ST_CPR) + d + 3 * px;
      u32x2 v;
      v[0] = (unsigned)src[0] | ((unsigned)src[1] << 16);
      v[1] = (unsigned)src[2];
      if (!ok) v = u32x2{0u, 0u};
      *(u32x2*)(raw + hh * ST_RP + 4 * px) = v;
    }
    __syncthreads();
    const int next = tile + gridDim.x;
    // unconditional (the last tile re-loads itself): a conditional prefetch
    // makes the registers a phi the compiler resolves right after the load
    stem_prefetch(a, next < a.tiles ? next : tile, pf);
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
      const int lrow = 4 * rg + q;
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
      const unsigned short* rb = raw + 2 * lrow * ST_RP + 8 * nl + 8 * hf;
#pragma unroll
      for (int ks = 0; ks < ST_KS; ++ks) {
        const int r = ks >> 1;
        u32x4 b = *(const u32x4*)(rb + r * ST_RP + 16 * (ks & 1));
        if ((ks & 1) && hf) { b[2] = 0u; b[3] = 0u; }  // tap 7
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[ks], __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
      }
      // lane holds pixel nl of row lrow, channels 32chh + 8qq + 4hf + i
      unsigned short* op = ost + (lrow * ST_TW + nl) * OP + 32 * chh + 4 * hf;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int c0 = 32 * chh + 8 * qq + 4 * hf;
        const f32x4 bi = *(const f32x4*)(s_bias + c0);
        const f32x4 sc = *(const f32x4*)(s_scale + c0);
        unsigned short o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[4 * qq + i];
          if (a.scale) v *= sc[i];
          v = act_apply(v + bi[i], ACT, a.act_alpha);
          o[i] = __builtin_bit_cast(unsigned short, (bf16)v);
        }
        u32x2 pk;
        pk[0] = (unsigned)o[0] | ((unsigned)o[1] << 16);
        pk[1] = (unsigned)o[2] | ((unsigned)o[3] << 16);
        *(u32x2*)(op + 8 * qq) = pk;
      }
    }
    __syncthreads();
    // tile output: 8 rows x 32 px x 8 chunks of 16 B; consecutive threads
    // write consecutive chunks (a pixel's 64 channels = one 128-B line)
    {
      const int px = (threadIdx.x >> 3) & 31, cc = threadIdx.x & 7;
      const int wo = wo0 + px;
      unsigned short* yb = a.y + (((long long)img * a.ho + ho0) * a.wo + wo) * a.k + 64 * z + 8 * cc;
      const long long rs = (long long)a.wo * a.k;
      const unsigned short* sb = ost + px * OP + 8 * cc;
#pragma unroll
      for (int j = 0; j < ST_TH; ++j) {  // thread -> (row j, pixel, 16-B chunk)
        const u32x4 v = *(const u32x4*)(sb + j * ST_TW * OP);
        if (ho0 + j < a.ho && wo < a.wo) *(u32x4*)(yb + j * rs) = v;
      }
    }
  }
}


// ---- stem weight gradient -----------------------------------------------
// dW[r][s][c][k] += sum over output pixels (img, ho, wo) of
//   x[img][2ho - pt + r][2wo - pl + s][c] * dz[img][ho][wo][k]
// (M = 147 rows (r, s, c), N = 64, K = n*ho*wo). The implicit GEMM gathers
// the 3-channel im2col^T two bytes at a time (135 us at batch 32, 54 TF for a
// layer whose operands are 60 MB). Here persistent blocks walk output rows
// (img, ho); per row the block stages the 7 input rows it reads (16-B loads)
// and the dz row, then builds in LDS
//   T[m][wo]   = the im2col^T tile (zero outside the image),
//   DZT[k][wo] = the dz row transposed,
// so both operands of v_mfma_f32_32x32x16_bf16 (8 consecutive pixels of one
// row m / one channel k per lane) are single 16-B LDS reads (pitch WP + 8
// elements: 16 distinct 4-bank groups per 16 lanes). Five waves each own a
// 32-row m tile and both 32-channel k tiles. A block's fp32 partial goes to
// slab[block], summed in block order by the ordered weight-gradient reduce
// (the rows each block walks are fixed: deterministic).
constexpr int SW_M = 147, SW_MP = 160, SW_THREADS = 320;
typedef __attribute__((ext_vector_type(4))) short s16x4;

struct StemWgradArgs {
  const unsigned short* x;   // bf16 (n, h, w, 3), 16-B aligned
  const unsigned short* dz;  // bf16 (n, ho, wo, 64), 16-B aligned
  float* slab;               // fp32 [gridDim.x][147][64]
  int n, h, w, ho, wo, pt, pl, rows;  // rows = n * ho
};

template <int WP>
__global__ __launch_bounds__(SW_THREADS, WP <= 112 ? 2 : 1) void stem_wgrad_kernel(StemWgradArgs a) {
  constexpr int TP = WP + 8;        // T / DZT row pitch (elements)
  constexpr int RE = 6 * WP;        // staged input row: 3 * w elements, w <= 2 * WP
  constexpr int XC = (7 * RE / 8 + SW_THREADS - 1) / SW_THREADS;  // 16-B x chunks per thread
  constexpr int DC = (WP * 8 + SW_THREADS - 1) / SW_THREADS;      // 16-B dz chunks per thread
  constexpr int NP = (WP / 2 + 63) / 64;                          // T pixel pairs per lane per row
  __shared__ __attribute__((aligned(16))) unsigned short xr[7 * RE];
  __shared__ __attribute__((aligned(16))) unsigned short tt[SW_MP * TP];
  // dz row as [wo][64] (128-B rows), 16-B chunk slot = chunk ^ ((wo >> 1) & 1) << 2,
  // read k-major by ds_read_b64_tr_b16 (the weight-gradient kernel's B image)
  __shared__ __attribute__((aligned(16))) unsigned short dzi[WP * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int rc = 3 * a.w / 8;  // 16-B chunks per input row
  // zero once: T's pad rows and every pad column (never written below), dz's pad pixels
  for (int i = tid; i < SW_MP * TP; i += SW_THREADS) tt[i] = 0;
  for (int i = tid; i < WP * 64; i += SW_THREADS) dzi[i] = 0;
  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
  typedef __attribute__((ext_vector_type(4))) unsigned u4;
  // the global chunks of output row t into registers (zeros outside the image / range)
  u4 xv[XC], dv[DC];
  auto fetch = [&](int t) {
    const int img = t / a.ho, ho = t - img * a.ho;
#pragma unroll
    for (int u = 0; u < XC; ++u) {
      const int q = tid + u * SW_THREADS;
      const int r = q / rc, j = q - r * rc;
      const int hi = 2 * ho - a.pt + r;
      xv[u] = u4{0u, 0u, 0u, 0u};
      if (t < a.rows && r < 7 && (unsigned)hi < (unsigned)a.h)
        xv[u] = *(const u4*)(a.x + ((long long)(img * a.h + hi) * a.w) * 3 + 8 * j);
    }
    const unsigned short* dzr = a.dz + (long long)t * a.wo * 64;
#pragma unroll
    for (int u = 0; u < DC; ++u) {
      const int q = tid + u * SW_THREADS;
      dv[u] = u4{0u, 0u, 0u, 0u};
      if (t < a.rows && q < a.wo * 8) dv[u] = *(const u4*)(dzr + (long long)(q >> 3) * 64 + (q & 7) * 8);
    }
  };
  int t = blockIdx.x;
  fetch(t);
  for (; t < a.rows; t += gridDim.x) {
    __syncthreads();  // the previous row's MFMA reads (and the zeroing) are done
#pragma unroll
    for (int u = 0; u < XC; ++u) {
      const int q = tid + u * SW_THREADS;
      const int r = q / rc, j = q - r * rc;
      if (r < 7) *(u4*)(xr + r * RE + 8 * j) = xv[u];
    }
#pragma unroll
    for (int u = 0; u < DC; ++u) {
      const int q = tid + u * SW_THREADS;
      if (q < a.wo * 8) {
        const int wo = q >> 3, j = q & 7;
        *(u4*)(dzi + wo * 64 + ((j ^ (((wo >> 1) & 1) << 2)) << 3)) = dv[u];
      }
    }
    __syncthreads();
    fetch(t + gridDim.x);  // the next row's loads fly under this row's build and MFMAs
    // this wave's 32 rows of T (wave-private: no block barrier before its
    // MFMAs). Every read of the rows first (clamped addresses, zeros selected
    // after the load: one LDS latency), then the 4-B pixel-pair writes
    const int npair = (a.wo + 1) >> 1;
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      const int p = lane + 64 * pp;
      const int wo0 = 2 * p;
      constexpr int HR = NP == 1 ? 16 : 8;  // rows at a time: 2 HR values in flight
#pragma unroll
      for (int h = 0; h < 32 / HR; ++h) {
        unsigned short v0[HR], v1[HR];
#pragma unroll
        for (int mm = 0; mm < HR; ++mm) {
          const int m = min(32 * wave + HR * h + mm, SW_M - 1);  // uniform
          const int rs = m / 3, c = m - 3 * rs, r = rs / 7, sx = rs - 7 * r;
          const int col0 = 2 * wo0 - a.pl + sx, col1 = col0 + 2;
          const unsigned short* xrow = xr + r * RE + c;
          v0[mm] = xrow[3 * min(max(col0, 0), a.w - 1)];
          v1[mm] = xrow[3 * min(max(col1, 0), a.w - 1)];
          if (!((unsigned)col0 < (unsigned)a.w)) v0[mm] = 0;
          if (!(wo0 + 1 < a.wo && (unsigned)col1 < (unsigned)a.w)) v1[mm] = 0;
        }
        if (p < npair) {
#pragma unroll
          for (int mm = 0; mm < HR; ++mm) {
            const int m = 32 * wave + HR * h + mm;
            if (m < SW_M) *(unsigned*)(tt + m * TP + wo0) = (unsigned)v0[mm] | ((unsigned)v1[mm] << 16);
          }
        }
      }
    }
    // 32x32 tiles: rows 32 * wave .. +31 of T, channels 0..31 / 32..63. The
    // dz operand by transposing reads: lane (g16, tq, tp) supplies pixel rows
    // k = 16 ks + 8 lh + tq and k + 4, channels 16 g16 + 4 tp .. +3 of a tile
    const unsigned short* ta = tt + (32 * wave + lr) * TP + 8 * lh;
    const int g16 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
    auto dz_frag = [&](int k, int col) {
      auto addr = [&](int kk) {
        return (const char*)dzi + kk * 128 + ((((col >> 3) ^ (((kk >> 1) & 1) << 2)) << 4) | ((col & 7) << 1));
      };
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(addr(k)));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(addr(k + 4)));
      __attribute__((ext_vector_type(8))) short w8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, w8);
    };
#pragma unroll
    for (int ks = 0; ks < WP / 16; ++ks) {
      const int k = 16 * ks + 8 * lh + tq;
      const bf16x8 fa = *(const bf16x8*)(ta + 16 * ks);
      const bf16x8 fb0 = dz_frag(k, 16 * g16 + 4 * tp);
      const bf16x8 fb1 = dz_frag(k, 32 + 16 * g16 + 4 * tp);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb1, acc1, 0, 0, 0);
    }
  }
  float* slab = a.slab + (long long)blockIdx.x * SW_M * 64;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 32 * wave + (i & 3) + 8 * (i >> 2) + 4 * lh;
    if (m < SW_M) {
      slab[m * 64 + lr] = acc0[i];
      slab[m * 64 + 32 + lr] = acc1[i];
    }
  }
}

}  // namespace

// The ResNet stem's weight gradient (x: 3 channels, 7x7 stride 2, k = 64,
// bf16): 1 = launched (partials in slabs from wgrad_slab_alloc, their
// ordered sum into dw queued / run by wgrad_slab_reduce), 0 = not handled
// here (the caller's implicit GEMM), < 0 = error.
int stem_conv_bwd_filter(const fpnmt_conv_desc* d, const void* x, const void* dz, const float* col_scale,
                         float* dw_hwio, hipStream_t s) {
  if (d->dtype != FPNMT_BF16 || d->c != 3 || d->r != 7 || d->s != 7 || d->stride_h != 2 || d->stride_w != 2 ||
      d->k != 64 || ((uintptr_t)x & 15) || ((uintptr_t)dz & 15) || d->w % 8 != 0)
    return 0;
  const int ho = (d->h + d->pad_t + d->pad_b - 7) / 2 + 1;
  const int wo = (d->w + d->pad_l + d->pad_r - 7) / 2 + 1;
  if (ho <= 0 || wo <= 0 || 2 * wo > 512 || d->w > 2 * 256 ||
      (long long)d->n * d->h * d->w * 3 >= (1LL << 31) || (long long)d->n * ho * wo * 64 >= (1LL << 31))
    return 0;
  const int WP = ((wo + 15) / 16) * 16;
  if (WP > 256 || d->w > 2 * WP) return 0;
  const int rows = d->n * ho;
  // two blocks per CU (63 KB of LDS at wo <= 112): one block's loads and
  // barriers under the other's T build and MFMAs
  const int grid = std::min(rows, WP <= 112 ? 512 : 256);
  float* slab = wgrad_slabs(SW_M, 64, grid);
  if (!slab) return 0;  // no room for the partials: the implicit GEMM
  StemWgradArgs a;
  a.x = (const unsigned short*)x;
  a.dz = (const unsigned short*)dz;
  a.slab = slab;
  a.n = d->n; a.h = d->h; a.w = d->w; a.ho = ho; a.wo = wo; a.pt = d->pad_t; a.pl = d->pad_l; a.rows = rows;
  if (WP <= 112)
    hipLaunchKernelGGL(stem_wgrad_kernel<112>, dim3(grid), dim3(SW_THREADS), 0, s, a);
  else
    hipLaunchKernelGGL(stem_wgrad_kernel<256>, dim3(grid), dim3(SW_THREADS), 0, s, a);
  int st = check_launch("stem_wgrad_kernel");
  if (!st) st = wgrad_slabs_reduce(dw_hwio, SW_M, 64, 64, grid, col_scale, slab, s);
  return st ? st : 1;
}

// 1 = launched, 0 = shape not handled here (caller uses the implicit GEMM),
// < 0 = launch error
int stem_conv_fwd(const fpnmt_conv_desc* d, const void* x, const void* w_ohwi, const float* scale,
                  const float* bias, const void* residual, void* y, hipStream_t s) {
  const long long total = (long long)d->n * d->h * d->w * 3;
  if (d->dtype != FPNMT_BF16 || residual || d->c != 3 || d->r != 7 || d->s != 7 ||
      d->stride_h != 2 || d->stride_w != 2 || d->k % 64 != 0 || ((uintptr_t)y & 15) || ((uintptr_t)x & 15) ||
      ((uintptr_t)w_ohwi & 15) || total % 8 != 0 || total >= (1LL << 31))
    return 0;
  const int ho = (d->h + d->pad_t + d->pad_b - 7) / 2 + 1;
  const int wo = (d->w + d->pad_l + d->pad_r - 7) / 2 + 1;
  StemArgs a;
  a.x = (const unsigned short*)x;
  a.w = (const unsigned short*)w_ohwi;
  a.scale = scale;
  a.bias = bias;
  a.y = (unsigned short*)y;
  a.n = d->n; a.h = d->h; a.w_ = d->w; a.ho = ho; a.wo = wo; a.k = d->k;
  a.pt = d->pad_t; a.pl = d->pad_l; a.act = d->act; a.act_alpha = d->act_alpha;
  a.tiles_h = cdiv(ho, ST_TH);
  a.tiles_w = cdiv(wo, ST_TW);
  const long long tiles = (long long)d->n * a.tiles_h * a.tiles_w;
  if (tiles >= (1LL << 31)) return 0;
  a.tiles = (int)tiles;
  a.total = (int)total;
  // persistent: 3 blocks per CU (LDS-bound) per 64-channel chunk
  const int grid = (int)std::min<long long>(tiles, 768);
  const dim3 g(grid, d->k / 64);
  if (d->act == FPNMT_ACT_RELU)
    hipLaunchKernelGGL(stem7x7s2_kernel<FPNMT_ACT_RELU>, g, dim3(256), 0, s, a);
  else if (d->act == FPNMT_ACT_LEAKY)
    hipLaunchKernelGGL(stem7x7s2_kernel<FPNMT_ACT_LEAKY>, g, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(stem7x7s2_kernel<FPNMT_ACT_NONE>, g, dim3(256), 0, s, a);
  const int st = check_launch("stem7x7s2_kernel");
  return st ? st : 1;
}

}  // namespace fpnmt
