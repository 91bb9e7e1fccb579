// Fused ResNet identity bottleneck, inference (keras-resnet bottleneck_2d,
// reference models/resnet.py:99-112 -> keras_resnet.blocks.bottleneck_2d with
// freeze_bn=True, blocks 1.. of a stage):
//   y = relu(x + bc + Wc * relu(b3 + W3 (*) pad1(relu(ba + Wa * x))))
// with the frozen BN folded (scale into the bf16 OHWI weights, shift into the
// fp32 biases). One kernel per block instead of three launches: the 64/128-
// channel intermediates stay in LDS over a tile of TR output rows (full image
// width) plus its one-row halo; only x (once, + the halo rows) and y touch HBM.
//
// Layout: every operand the MFMAs read is an LDS image of rows (pixels or
// output channels) of 16-B chunks, chunk slot XOR-swizzled per row (RC = 8
// chunks of 128-B rows: slot ^ ((row >> 1) & 7); RC = 16: slot ^ (row & 15)),
// filled by LDS-DMA (lane-linear destination, swizzle on the source address).
// Pixels are enumerated on a PADDED grid of WP = W + 2 columns, so the 3x3's
// tap (dr, dc) reads mid1 row m + dr * WP + dc: nine shifted GEMMs over one
// image, no gather. mid1 holds rows (h0 - 1 .. h0 + TR) x padded columns,
// zero outside the image (TF 'same' zero padding of the 2b conv, ZeroPadding2D(1)).
//
// Schedule: ONE stream of DMA "units" per block, in a ring of NSLOT LDS slots,
// continuing across the phases and the tiles of a persistent block:
//   A-unit kc (C / 64 of them): the tile's x rows (halo grid), channels
//     64 kc .. +63, and Wa[:, 64 kc .. +63]      -> acc_a += x * Wa^T
//   B-unit (9 / TPU): W3 taps [CM][CM] each       -> acc_b += mid1(shift t) * W3t^T
//   C-unit j (C / 64): Wc rows 64 j .. +63 and the residual x of the tile's
//     output pixels in those channels        -> y chunk = relu(mid2 * Wcj^T + bc + x)
// Unit u+NSLOT-1's DMA is issued right after the barrier that retires unit u
// (a C-unit issues it after its y stores); the phase ends (mid1 / mid2 to
// LDS, y to HBM) ride between units. mid1 and mid2 share one region.
// Measured (tools/bn_bench.hip, profiles/r05/bn_probe_r5k.txt, batch 64):
// two slots beat three (res2 98.7 against 103.9 us; res3 at TR = 4 with two
// slots 75.0 against 117 us at TR = 2 with three, which is what fits LDS), the
// residual and y traffic through the epilogue ~40 % of the time, s_memtime
// buckets: ~1/3 waiting at the unit barrier, the rest split over the phases
// (each unit's LDS-DMA issue sits in every wave's stream).
//
// MFMA: v_mfma_f32_16x16x32_bf16 with the operands swapped (the output
// channel tile as srcA), so lane l holds 4 consecutive channels of pixel
// (l & 15): 8-B LDS writes of mid1 / mid2, 16-B y stores after a
// v_permlane16_swap pair (gemm_pipe.h epilogue_direct16).
#include "gemm_impl.h"
#include "gemm_pipe.h"

// timing probes of tools/bn_bench.hip only (the library builds 0): bit 0 =
// no residual loads, bit 1 = no y stores (wrong results; where the time goes),
// bit 2 = per-block s_memtime buckets (wait + barrier / phase A / B / C) into g.dbg
#ifndef BN_PROBE
#define BN_PROBE 0
#endif

namespace fpnmt {

namespace {

__device__ __forceinline__ void wait_lgkm0_all() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int RC>
__device__ __forceinline__ int bn_swz(int row) {
  if constexpr (RC == 8) return (row >> 1) & 7;
  else return row & 15;
}
template <int RC>
__device__ __forceinline__ int bn_off(int row, int chunk) {
  return row * (RC * 16) + ((chunk ^ bn_swz<RC>(row)) << 4);
}

struct BnArgs {
  const bf16* x;
  const bf16* wa;  // [CM][C]        (OHWI of the 1x1 2a conv)
  const bf16* w3;  // [CM][3][3][CM] (OHWI of the 3x3 2b conv)
  const bf16* wc;  // [C][CM]        (OHWI of the 1x1 2c conv)
  const float* ba;
  const float* b3;
  const float* bc;
  bf16* y;
  const bf16* zero;  // >= 256 B of zeros (out-of-image rows)
  int n;             // images
  unsigned long long* dbg;  // BN_PROBE & 4 only
};

// C: block channels, CM: bottleneck channels, H x W: image, TR: output rows
// per tile, MB: padded output rows (>= TR * (W + 2)), NC: output channels per
// C-unit, TPU: 3x3 taps per B-unit; wave layouts (WM x WN = 8) per phase:
// A (MA x CM), B (MB x CM), C (MB x NC)
template <int C, int CM, int H, int W, int TR, int MB, int NC, int TPU, int AWM, int BWM, int CWM, int NSLOT>
__global__ __launch_bounds__(512) void bottleneck_fwd_kernel(const BnArgs g) {
  constexpr int NT = 512;
  constexpr int WP = W + 2;
  constexpr int MA_VALID = (TR + 2) * WP, MB_VALID = TR * WP;
  static_assert(MB_VALID <= MB && MB % 64 == 0, "output rows of a tile");
  constexpr int MA = ((MB - 1 + 2 * WP + 2 + 1 + 63) / 64) * 64;  // rows the shifted taps may read
  static_assert(MA >= MA_VALID, "");
  constexpr int RCM = CM / 8;                      // chunks per mid1 / mid2 / W3 / Wc row
  static_assert(RCM == 8 || RCM == 16, "CM = 64 or 128");
  static_assert(9 % TPU == 0, "taps per B-unit");
  constexpr int KA = C / 64, KB = 9 / TPU, KC = C / NC;  // units per phase
  constexpr int UNITS = KA + KB + KC;
  // LDS: a ring of three unit slots (two units in flight), then ONE
  // intermediate region: mid1 during phase B, mid2 (written after the last
  // tap's reads, behind a barrier) during phase C
  constexpr int XA_BYTES = MA * 128, WA_BYTES = CM * 128;
  // a C-unit carries Wc's NC rows and the residual x of the tile's MB output
  // pixels in those NC channels (the epilogue reads it from LDS: a plain
  // global load used while LDS-DMA is in flight drains the whole ring)
  static_assert(NC == 64, "C-unit residual image: 64 channels (128-B rows)");
  constexpr int W3_BYTES = CM * CM * 2, WC_BYTES = NC * CM * 2, RS_BYTES = MB * 128;
  constexpr int UA = XA_BYTES + WA_BYTES, UB = TPU * W3_BYTES, UC = WC_BYTES + RS_BYTES;
  constexpr int SLOT = UA > UB ? (UA > UC ? UA : UC) : (UB > UC ? UB : UC);
  constexpr int MID1 = MA * CM * 2, MID2 = MB * CM * 2;
  constexpr int MID = MID1 > MID2 ? MID1 : MID2;
  static_assert(NSLOT == 2 || NSLOT == 3, "unit ring depth");
  constexpr int BIAS = (2 * CM + C) * 4;  // ba, b3, bc staged in LDS (no global loads in the loop)
  constexpr int SMEM = NSLOT * SLOT + MID + BIAS;
  static_assert(SMEM <= 160 * 1024, "LDS");
  // DMA instructions per thread per unit
  constexpr int NXA = MA * 8 / NT, NWA = CM * 8 / NT, NW3 = CM * RCM / NT, NWC = NC * RCM / NT, NRS = MB * 8 / NT;
  static_assert(NXA * NT == MA * 8 && NWA * NT == CM * 8 && NW3 * NT == CM * RCM && NWC * NT == NC * RCM &&
                    NRS * NT == MB * 8,
                "");
  constexpr int DA = NXA + NWA, DB = TPU * NW3, DC = NWC + NRS;  // per unit type
  // wave tiles (16x16 MFMA tiles per wave)
  constexpr int AWN = 8 / AWM, BWN = 8 / BWM, CWN = 8 / CWM;
  constexpr int ATM = MA / AWM / 16, ATN = CM / AWN / 16;
  constexpr int BTM = MB / BWM / 16, BTN = CM / BWN / 16;
  constexpr int CTM = MB / CWM / 16, CTN = NC / CWN / 16;
  static_assert(ATM * AWM * 16 == MA && ATN * AWN * 16 == CM, "phase A waves");
  static_assert(BTM * BWM * 16 == MB && BTN * BWN * 16 == CM, "phase B waves");
  static_assert(CTM * CWM * 16 == MB && CTN * CWN * 16 == NC, "phase C waves");
  constexpr int TILES_PER_IMG = H / TR;
  static_assert(TILES_PER_IMG * TR == H, "");

  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  char* const mid = smem + NSLOT * SLOT;
  float* const sb = (float*)(mid + MID);  // [ba | b3 | bc]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = g.n * TILES_PER_IMG;
  // persistent blocks, XCD-aware: the blocks of one XCD (blockIdx % 8) walk
  // one contiguous range of tiles together, so neighbouring tiles' shared
  // halo rows meet in that XCD's L2 (fewer than 8 blocks: as many groups)
  const int ng = gridDim.x < 8 ? (int)gridDim.x : 8;
  const int xcd = blockIdx.x % ng, slot = blockIdx.x / ng, per_xcd = ((int)gridDim.x - xcd + ng - 1) / ng;
  const int t_lo = (int)((long long)ntiles * xcd / ng), t_hi = (int)((long long)ntiles * (xcd + 1) / ng);
  const int my_tiles = t_lo + slot < t_hi ? (t_hi - t_lo - slot + per_xcd - 1) / per_xcd : 0;
  const int total_units = my_tiles * UNITS;
  auto tile_of = [&](int i) { return t_lo + slot + i * per_xcd; };
  auto unit_kind = [&](int u) { return u - (u / UNITS) * UNITS; };  // position within the tile's units
  auto dma_count = [&](int u) {  // this thread's DMA instructions of unit u (0 past the end)
    if (u >= total_units) return 0;
    const int k = unit_kind(u);
    return k < KA ? DA : (k < KA + KB ? DB : DC);
  };

  typedef __attribute__((address_space(3))) void lds_void;
  auto dma = [&](const void* src, char* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_wave_base, 16, 0, 0);
  };
  // issue DMA unit u (tile i = u / UNITS) into slot u % 3
  auto issue = [&](int u) {
    const int i = u / UNITS, k = u - i * UNITS;
    const int tile = tile_of(i);
    const int img = tile / TILES_PER_IMG, h0 = (tile - img * TILES_PER_IMG) * TR;
    char* hb = smem + (u % NSLOT) * SLOT;
    if (k < KA) {
      // x rows on the halo grid (row q: image row h0 - 1 + q / WP, column q % WP - 1)
#pragma unroll
      for (int j = 0; j < NXA; ++j) {
        const int q = j * NT + tid, row = q >> 3, ch = (q & 7) ^ bn_swz<8>(row);
        const int hh = h0 - 1 + row / WP, ww = row % WP - 1;
        const bool ok = row < MA_VALID && hh >= 0 && hh < H && ww >= 0 && ww < W;
        const bf16* src = ok ? g.x + (((long long)img * H + hh) * W + ww) * C + k * 64 + ch * 8 : g.zero;
        dma(src, hb + (j * NT + wave * 64) * 16);
      }
#pragma unroll
      for (int j = 0; j < NWA; ++j) {
        const int q = j * NT + tid, row = q >> 3, ch = (q & 7) ^ bn_swz<8>(row);
        dma(g.wa + (long long)row * C + k * 64 + ch * 8, hb + XA_BYTES + (j * NT + wave * 64) * 16);
      }
    } else if (k < KA + KB) {
      const int t0 = (k - KA) * TPU;
#pragma unroll
      for (int tt = 0; tt < TPU; ++tt)
#pragma unroll
        for (int j = 0; j < NW3; ++j) {
          const int q = j * NT + tid, row = q / RCM, ch = (q % RCM) ^ bn_swz<RCM>(row);
          dma(g.w3 + ((long long)row * 9 + t0 + tt) * CM + ch * 8, hb + tt * W3_BYTES + (j * NT + wave * 64) * 16);
        }
    } else {
      const int c0 = (k - KA - KB) * NC;
#pragma unroll
      for (int j = 0; j < NWC; ++j) {
        const int q = j * NT + tid, row = q / RCM, ch = (q % RCM) ^ bn_swz<RCM>(row);
        dma(g.wc + (long long)(c0 + row) * CM + ch * 8, hb + (j * NT + wave * 64) * 16);
      }
      // residual rows (padded output grid: image row h0 + m / WP, column m % WP)
#pragma unroll
      for (int j = 0; j < NRS; ++j) {
        const int q = j * NT + tid, m = q >> 3, ch = (q & 7) ^ bn_swz<8>(m);
        const int hh = h0 + m / WP, ww = m % WP;
        const bool ok = m < MB_VALID && ww < W;
        const bf16* src = ok ? g.x + (((long long)img * H + hh) * W + ww) * C + c0 + ch * 8 : g.zero;
        dma(src, hb + WC_BYTES + (j * NT + wave * 64) * 16);
      }
    }
  };

  // fragment read of a 16-row MFMA tile: lane l reads row r0 + (l & 15),
  // chunk c0 + (l >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  auto frag = [&](const char* img, auto rc_c, int r0, int c0) -> bf16x8 {
    constexpr int RC = decltype(rc_c)::value;
    return *(const bf16x8*)(img + bn_off<RC>(r0 + fr, c0 + fq));
  };
  // acc[a][b] += A[arow0 + 16 a ..][k] * B[brow0 + 16 b ..][k] over nks 32-deep k-steps
  // NSEG segments of NKS 32-deep k-steps each; segment s reads A rows from
  // arow(s) and B rows of the image bimg(s); the next step's fragments are
  // read while the current step's MFMAs run (two register sets)
  auto mma = [&](auto& acc, const char* Aimg, auto rca, auto arow, auto bimg, auto rcb, int brow0, auto nks_c,
                 auto nseg_c) {
    constexpr int TMx = std::extent<std::remove_reference_t<decltype(acc)>, 0>::value;
    constexpr int TNx = std::extent<std::remove_reference_t<decltype(acc)>, 1>::value;
    constexpr int NKS = decltype(nks_c)::value, NSTEP = NKS * decltype(nseg_c)::value;
    bf16x8 af[2][TMx], bfr[2][TNx];
    auto load = [&](int step, bf16x8 (&a_)[TMx], bf16x8 (&b_)[TNx]) {
      const int sg = step / NKS, ks = step - sg * NKS;
      const int r0 = arow(sg);
      const char* Bimg = bimg(sg);
#pragma unroll
      for (int a = 0; a < TMx; ++a) a_[a] = frag(Aimg, rca, r0 + 16 * a, 4 * ks);
#pragma unroll
      for (int b = 0; b < TNx; ++b) b_[b] = frag(Bimg, rcb, brow0 + 16 * b, 4 * ks);
    };
    load(0, af[0], bfr[0]);
    static_for<0, NSTEP>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j + 1 < NSTEP) load(j + 1, af[(j + 1) & 1], bfr[(j + 1) & 1]);
#pragma unroll
      for (int a = 0; a < TMx; ++a)
#pragma unroll
        for (int b = 0; b < TNx; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j & 1][b], af[j & 1][a], acc[a][b], 0, 0, 0);
    });
  };
  auto zero_acc = [](auto& acc) {
    constexpr int TMx = std::extent<std::remove_reference_t<decltype(acc)>, 0>::value;
    constexpr int TNx = std::extent<std::remove_reference_t<decltype(acc)>, 1>::value;
#pragma unroll
    for (int a = 0; a < TMx; ++a)
#pragma unroll
      for (int b = 0; b < TNx; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // relu(acc + bias) -> bf16 rows of an LDS image (lane: 4 channels of one pixel)
  auto to_lds = [&](auto& acc, char* img, int row0, int col0, const float* bias, auto valid_fn) {
    constexpr int TMx = std::extent<std::remove_reference_t<decltype(acc)>, 0>::value;
    constexpr int TNx = std::extent<std::remove_reference_t<decltype(acc)>, 1>::value;
#pragma unroll
    for (int b = 0; b < TNx; ++b) {
      const int col = col0 + 16 * b + 4 * fq;
      const f32x4 bi = *(const f32x4*)(bias + col);
#pragma unroll
      for (int a = 0; a < TMx; ++a) {
        const int row = row0 + 16 * a + fr;
        const bool ok = valid_fn(row);
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)(ok ? fmaxf(acc[a][b][j] + bi[j], 0.f) : 0.f);
        *(bf16x4*)(img + bn_off<RCM>(row, col >> 3) + (col & 4) * 2) = o;
      }
    }
  };

  const int awm = wave / AWN, awn = wave % AWN;
  const int bwm = wave / BWN, bwn = wave % BWN;
  const int cwm = wave / CWN, cwn = wave % CWN;
  f32x4 acc_a[ATM][ATN], acc_b[BTM][BTN], acc_c[CTM][CTN];

  // the biases go to LDS before any DMA is in flight: a plain global load
  // used while LDS-DMA is outstanding makes hipcc wait vmcnt(0), i.e. drain
  // the unit ring (cdna_hip_programming.md 'Pipelining across barriers')
  for (int q = tid; q < 2 * CM + C; q += NT)
    sb[q] = q < CM ? g.ba[q] : (q < 2 * CM ? g.b3[q - CM] : g.bc[q - 2 * CM]);
  __syncthreads();
  if (total_units > 0) issue(0);
  if (NSLOT == 3 && total_units > 1) issue(1);
  unsigned long long tb[4] = {0, 0, 0, 0}, tprev = 0;
  auto stamp = [&](int bucket) {
    if constexpr ((BN_PROBE & 4) != 0) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (bucket >= 0) tb[bucket] += now - tprev;
      tprev = now;
    }
  };
  stamp(-1);
  for (int u = 0; u < total_units; ++u) {
    // unit u landed (this thread's part; unit u+1 may stay in flight) and
    // this wave's LDS writes retired; after the barrier: everyone's, and
    // every read of unit u-1 (slot (u+2) % 3) is done
    const int ahead = NSLOT == 3 ? dma_count(u + 1) : 0;
    if (ahead == DA) wait_vmcnt<DA>();
    else if (ahead == DB) wait_vmcnt<DB>();
    else if (ahead == DC) wait_vmcnt<DC>();
    else wait_vmcnt<0>();
    wait_lgkm0_all();
    __builtin_amdgcn_s_barrier();
    stamp(0);
    const int i = u / UNITS, k = u - i * UNITS;
    // unit u+2 into the slot unit u-1 left; a C-unit issues it after its y
    // stores, so the next iteration's counted wait (everything but unit
    // u+2's DMA) covers the stores and does not wait out unit u+2
    const bool c_unit = k >= KA + KB;
    if (!c_unit && u + NSLOT - 1 < total_units) issue(u + NSLOT - 1);
    const char* hb = smem + (u % NSLOT) * SLOT;
    if (k < KA) {
      if (k == 0) zero_acc(acc_a);
      const int ar = awm * ATM * 16;
      mma(acc_a, hb, std::integral_constant<int, 8>{}, [&](int) { return ar; }, [&](int) { return hb + XA_BYTES; },
          std::integral_constant<int, 8>{}, awn * ATN * 16, std::integral_constant<int, 2>{},
          std::integral_constant<int, 1>{});
      if (k == KA - 1) {
        // mid1 (the previous tile's mid2 is no longer read: barriers since)
        const int tile = tile_of(i);
        const int h0 = (tile % TILES_PER_IMG) * TR;
        to_lds(acc_a, mid, awm * ATM * 16, awn * ATN * 16, sb, [&](int q) {
          const int hh = h0 - 1 + q / WP, ww = q % WP - 1;
          return q < MA_VALID && hh >= 0 && hh < H && ww >= 0 && ww < W;
        });
      }
    } else if (k < KA + KB) {
      const int t0 = (k - KA) * TPU;
      if (t0 == 0) zero_acc(acc_b);
      const int br = bwm * BTM * 16;
      mma(acc_b, mid, std::integral_constant<int, RCM>{},
          [&](int tt) { const int t = t0 + tt; return br + (t / 3) * WP + (t % 3); },
          [&](int tt) { return hb + tt * W3_BYTES; }, std::integral_constant<int, RCM>{}, bwn * BTN * 16,
          std::integral_constant<int, CM / 32>{}, std::integral_constant<int, TPU>{});
      if (k == KA + KB - 1) {
        // mid2 overwrites mid1: every wave's reads of mid1 retired first
        wait_lgkm0_all();
        __builtin_amdgcn_s_barrier();
        to_lds(acc_b, mid, bwm * BTM * 16, bwn * BTN * 16, sb + CM, [](int) { return true; });
      }
    } else {
      const int c0 = (k - KA - KB) * NC;
      zero_acc(acc_c);
      const int cr = cwm * CTM * 16;
      mma(acc_c, mid, std::integral_constant<int, RCM>{}, [&](int) { return cr; }, [&](int) { return hb; },
          std::integral_constant<int, RCM>{}, cwn * CTN * 16, std::integral_constant<int, CM / 32>{},
          std::integral_constant<int, 1>{});
      // y = relu(acc + bc + x) at the tile's valid pixels (padded-grid row m:
      // image row h0 + m / WP, column m % WP)
      const int tile = tile_of(i);
      const int img = tile / TILES_PER_IMG, h0 = (tile - img * TILES_PER_IMG) * TR;
#pragma unroll
      for (int a = 0; a < CTM; ++a) {
        const int m = cwm * CTM * 16 + 16 * a + fr;
        const int hh = h0 + m / WP, ww = m % WP;
        const bool ok = m < MB_VALID && ww < W;
        const long long pix = ((long long)img * H + (ok ? hh : h0)) * W + (ok ? ww : 0);
        static_for<0, (CTN + 1) / 2>([&](auto pc) {
          constexpr int b0 = 2 * decltype(pc)::value;
          if constexpr (b0 + 1 < CTN) {
            float v0[4], v1[4];
            const int col0 = c0 + cwn * CTN * 16 + 16 * b0 + 4 * fq;
            const f32x4 bi0 = *(const f32x4*)(sb + 2 * CM + col0), bi1 = *(const f32x4*)(sb + 2 * CM + col0 + 16);
            bf16x4 r0 = {}, r1 = {};
            if constexpr (!(BN_PROBE & 1)) {  // the unit's residual image [MB][64]
              const int cl = col0 - c0;
              r0 = *(const bf16x4*)(hb + WC_BYTES + bn_off<8>(m, cl >> 3) + (cl & 4) * 2);
              r1 = *(const bf16x4*)(hb + WC_BYTES + bn_off<8>(m, (cl + 16) >> 3) + (cl & 4) * 2);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v0[j] = fmaxf(acc_c[a][b0][j] + bi0[j] + (float)r0[j], 0.f);
              v1[j] = fmaxf(acc_c[a][b0 + 1][j] + bi1[j] + (float)r1[j], 0.f);
            }
            const bf16x4 o0 = {(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]};
            const bf16x4 o1 = {(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
            u32x2 x0 = __builtin_bit_cast(u32x2, o0), x1 = __builtin_bit_cast(u32x2, o1);
            const auto s0 = __builtin_amdgcn_permlane16_swap(x0[0], x1[0], false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(x0[1], x1[1], false, false);
            const u32x4 out = {s0[0], s1[0], s0[1], s1[1]};
            const int colw = c0 + cwn * CTN * 16 + 16 * b0 + 16 * (fq & 1) + 8 * (fq >> 1);
            if (ok && !(BN_PROBE & 2)) *(u32x4*)(g.y + pix * C + colw) = out;
          } else {
            const int col = c0 + cwn * CTN * 16 + 16 * b0 + 4 * fq;
            const f32x4 bi = *(const f32x4*)(sb + 2 * CM + col);
            const int cl = col - c0;
            const bf16x4 r = *(const bf16x4*)(hb + WC_BYTES + bn_off<8>(m, cl >> 3) + (cl & 4) * 2);
            bf16x4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)fmaxf(acc_c[a][b0][j] + bi[j] + (float)r[j], 0.f);
            if (ok) *(bf16x4*)(g.y + pix * C + col) = o;
          }
        });
      }
    }
    if (c_unit && u + NSLOT - 1 < total_units) issue(u + NSLOT - 1);
    stamp(k < KA ? 1 : (k < KA + KB ? 2 : 3));
  }
  if constexpr ((BN_PROBE & 4) != 0) {
    if (tid == 0)
      for (int b = 0; b < 4; ++b) g.dbg[blockIdx.x * 4 + b] = tb[b];
  }
}

template <int C, int CM, int H, int W, int TR, int MB, int NC, int TPU, int AWM, int BWM, int CWM, int NSLOT>
int launch_bottleneck(const BnArgs& a, hipStream_t s) {
  const int tiles = a.n * (H / TR);
  const int grid = tiles < 256 ? tiles : 256;
  hipLaunchKernelGGL((bottleneck_fwd_kernel<C, CM, H, W, TR, MB, NC, TPU, AWM, BWM, CWM, NSLOT>), dim3(grid), dim3(512),
                     0, s, a);
  return check_launch("bottleneck_fwd_kernel");
}

}  // namespace

}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

int fpnmt_bottleneck_fwd(int n, int h, int w, int c, int cm, const void* x, const void* wa, const float* ba,
                         const void* w3, const float* b3, const void* wc, const float* bc, void* y,
                         fpnmt_stream_t stream) {
  if (n <= 0) return 0;
  if (!x || !wa || !ba || !w3 || !b3 || !wc || !bc || !y) return fail(FPNMT_E_ARG, "bottleneck_fwd: null pointer");
  if (x == y) return fail(FPNMT_E_ARG, "bottleneck_fwd: y must not alias x (x is the residual)");
  if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)wa | (uintptr_t)w3 | (uintptr_t)wc | (uintptr_t)ba |
       (uintptr_t)b3 | (uintptr_t)bc) & 15)
    return fail(FPNMT_E_ARG, "bottleneck_fwd: operands must be 16-B aligned");
  BnArgs a{(const bf16*)x, (const bf16*)wa, (const bf16*)w3, (const bf16*)wc, ba, b3, bc, (bf16*)y,
           (const bf16*)zero16_ptr(), n, nullptr};
  if (!a.zero) return fail(FPNMT_E_ARG, "bottleneck_fwd: no workspace (fpnmt_set_workspace)");
  if (c == 256 && cm == 64 && h == 56 && w == 56)
    return launch_bottleneck<256, 64, 56, 56, 2, 128, 64, 3, 4, 4, 4, 2>(a, S(stream));
  if (c == 512 && cm == 128 && h == 28 && w == 28)
    return launch_bottleneck<512, 128, 28, 28, 4, 128, 64, 1, 4, 4, 4, 2>(a, S(stream));
  return FPNMT_E_UNSUPPORTED;  // quietly: the caller runs the three convs
}

}  // extern "C"
