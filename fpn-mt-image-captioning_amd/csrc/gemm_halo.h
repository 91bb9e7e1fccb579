// Halo-staged implicit-GEMM for stride-1 'same' KxK convs (forward, and the
// stride-1 bwd-data, which is the same conv on flipped weights), bf16.
//
// Why: the im2col A operand of a 3x3 conv re-reads every input pixel nine
// times. For stride 1 and Ho == H, Wo == W, output pixel m at filter tap
// (r, s) reads input pixel m + (r - pt) * W + (s - pl) of the flattened NHWC
// tensor (when that tap is inside the image), so the A rows of ALL taps of a
// BM-row tile lie in ONE contiguous pixel range
//     [m0 - pt*W - pl, m0 + BM + (R-1-pt)*W + (S-1-pl))
// of BM + (R-1)*W + (S-1) rows. The block DMAs that "halo" range once per
// 64-channel chunk into LDS and builds every tap's A fragments from it, so
// per K-tile the block loads BN*64*2 B of weights plus 1/(R*S) of the halo
// instead of (BM + BN)*64*2 B: 20 KB instead of 48 KB at 256x128 for 3x3.
//
// Structure (same pipeline idiom as gemm_pipe_kernel): 8 waves, BM x BN tile,
// BK = 64; the K loop runs channel chunk by chunk and tap by tap inside a
// chunk (K index = tap * Cc + c, the OHWI weight layout); weights stream
// through a 3-stage LDS-DMA ring (two K-tiles in flight across each raw
// s_barrier), the halo image is double buffered and the next chunk's halo is
// issued at the chunk's first tap, so it has R*S - 1 K-tiles to land. Every
// wait is a counted vmcnt that leaves the younger DMAs in flight. LDS images
// are [row][64] bf16 with the 16-B chunk index XOR-swizzled by (row >> 1) & 7
// on the source address (conflict-free ds_read_b128 for any run of 32
// consecutive rows, whatever the tap's row shift). A lane whose (pixel, tap)
// falls outside the image reads the halo buffer's last row, which is never
// part of the range (hrows < HALO_MAX_ROWS) and so is always DMA'd from the
// zero page.
//
// BST: weight stages (3: two K-tiles in flight; 4: three). RD: fragment
// reads 0 = one k-step ahead (two register sets), 1 = the whole K-tile's
// reads issued right after the barrier (counted lgkmcnt per k-step). (Reading
// K-tile t+1's fragments under K-tile t's MFMAs, with two whole-K-tile
// register sets at 223 VGPRs, measured 3-8 % slower and was dropped.) PRIO 1:
// waves 4-7 (the second-dispatched half, which loses issue arbitration to
// its SIMD partner) run at s_setprio 1 through the K loop. PROBE (timing
// probes of tools/halo_bench.hip only; the library instantiates 0):
// 1 = no DMA inside the K loop, 2 = no MFMA, 3 = no DMA and no fragment
// reads (register operands), 4 = no DMA and no MFMA.
#pragma once
#include "gemm_pipe.h"

namespace fpnmt {

constexpr int HALO_MAX_ROWS = 384;  // LDS rows per halo buffer (6 DMA rounds of 64 rows)

template <int BM, int BN, int WM, int WN, int BST = 3, int RD = 0, int PRIO = 0, int PROBE = 0>
__global__ __launch_bounds__(512) void gemm_halo_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int NT = 512;
  constexpr int BK = 64;
  static_assert(WM * WN == 8, "8 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "");
  constexpr int HROWS = HALO_MAX_ROWS;
  constexpr int H_BYTES = HROWS * 128;
  constexpr int NH = HROWS * 8 / NT;        // halo DMA chunks per thread per chunk
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int NB = BN * 8 / NT;           // weight DMA chunks per thread per K-tile
  static_assert((BN * 8) % NT == 0 && (HROWS * 8) % NT == 0, "");
  constexpr int STAGES = BST;
  static_assert(STAGES == 3 || STAGES == 4, "stages");
  constexpr int ZROW = HROWS - 1;  // always-zero halo row (hrows < HROWS)
  constexpr int SMEM = 2 * H_BYTES + STAGES * B_BYTES;
  constexpr int EPI_BYTES = (NT / 64) * 32 * (WTN + 4) * 4;
  static_assert(EPI_BYTES <= SMEM && SMEM <= 160 * 1024, "LDS");
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
  int gH = p.H, gW = p.W;
  FastDiv gfdHW = p.fd_HoWo, gfdW = p.fd_Wo;
  if (p.ngroups > 0) {  // m-grouped launch (shared B), static kernarg indices only
    GemmGroup G = p.groups[0];
#pragma unroll
    for (int q = 1; q < MAX_GROUPS; ++q)
      if (q < p.ngroups && tmi >= p.groups[q].start) G = p.groups[q];
    tmi -= G.start;
    Ap = G.A; Cp0 = G.C; Rp = G.R;
    M = G.M;
    gH = G.H; gW = G.W;
    gfdHW = G.fd_HoWo; gfdW = G.fd_Wo;
  }
  const int N = p.N;
  const int Cc = p.Cc;
  const int taps = p.Rk * p.Sk;
  const int nc = Cc / BK;
  const int nk = nc * taps;
  const int m0 = tmi * BM, n0 = tni * BN;
  const int z = blockIdx.z;
  const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
  const T* __restrict__ Ag = (const T*)Ap + zo * p.a_so + zi * p.a_si;
  const T* __restrict__ Bg = (const T*)p.B + zo * p.b_so + zi * p.b_si;
  const T* zero = (const T*)p.zero16;
  const int hbase = m0 - p.pt * gW - p.pl;  // flat input pixel of halo row 0
  const int hrows = BM + (p.Rk - 1) * gW + (p.Sk - 1);

  // ---- per-thread DMA sources ------------------------------------------
  // halo: chunk q = i*NT + tid -> LDS byte q*16: row q>>3, slot q&7 holding
  // logical 8-channel chunk slot ^ sw(row); rows past the range or outside
  // the tensor read the zero page
  int h_off[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const int q = i * NT + tid;
    const int row = q >> 3;
    const int kc = ((q & 7) ^ ((row >> 1) & 7)) * 8;
    const int pix = hbase + row;
    h_off[i] = (row < hrows && pix >= 0 && pix < M) ? pix * Cc + kc : -1;
  }
  int b_off[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int q = i * NT + tid;
    const int row = q >> 3;
    const int kc = ((q & 7) ^ ((row >> 1) & 7)) * 8;
    b_off[i] = n0 + row < N ? (n0 + row) * (int)p.ldb + kc : -1;
  }
  // per fragment row: local row and its in-image tap mask (bit r*S + s)
  int f_row[TM];
  unsigned f_vm[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const int mr = wm * WTM + t * 32 + lr;
    const int m = m0 + mr;
    f_row[t] = mr;
    unsigned vm = 0;
    if (m < M) {
      const uint32_t nimg = fdiv((uint32_t)m, gfdHW);
      const int rem = m - (int)nimg * gH * gW;
      const uint32_t ho = fdiv((uint32_t)rem, gfdW);
      const int wo = rem - (int)ho * gW;
      for (int r = 0; r < p.Rk; ++r)
        for (int s2 = 0; s2 < p.Sk; ++s2) {
          const int hi = (int)ho + r - p.pt, wi = wo + s2 - p.pl;
          if (hi >= 0 && hi < gH && wi >= 0 && wi < gW) vm |= 1u << (r * p.Sk + s2);
        }
    }
    f_vm[t] = vm;
  }

  typedef __attribute__((address_space(3))) void lds_void;
  auto issue_halo = [&](int cc, int buf) {
    char* hb = smem + buf * H_BYTES;
    const int coff = cc * BK;
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const T* src = h_off[i] >= 0 ? Ag + (h_off[i] + coff) : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(hb + (i * NT + wave * 64) * 16), 16, 0, 0);
    }
  };
  auto issue_b = [&](int kt, int stage) {
    const int cc = kt / taps;
    const int tap = kt - cc * taps;
    const int k0 = tap * Cc + cc * BK;
    char* sb = smem + 2 * H_BYTES + stage * B_BYTES;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const T* src = b_off[i] >= 0 ? Bg + (b_off[i] + k0) : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sb + (i * NT + wave * 64) * 16), 16, 0, 0);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  auto compute = [&](int kt, int stage) {
    const int cc = kt / taps;
    const int tap = kt - cc * taps;
    const int r = tap / p.Sk;
    const int shift = r * gW + (tap - r * p.Sk);
    const char* Hs = smem + (cc & 1) * H_BYTES;
    const char* Bs = smem + 2 * H_BYTES + stage * B_BYTES;
    // this tap's A row per fragment (or the zero row)
    int arow[TM];
    bool aok[TM];
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      arow[t] = f_row[t] + shift;
      aok[t] = (f_vm[t] >> tap) & 1u;
    }
    auto frag = [&](int ks, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
      const int c = ks * 2 + lh;
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int row = arow[t];
        const int hr = aok[t] ? row : ZROW;
        const char* a = Hs + hr * 128 + ((c ^ ((hr >> 1) & 7)) << 4);
        af[t] = *(const bf16x8*)a;
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int row = wn * WTN + t * 32 + lr;
        bfr[t] = *(const bf16x8*)(Bs + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
      }
    };
    constexpr int NSET = RD ? BK / 16 : 2;
    bf16x8 fa[NSET][TM], fb[NSET][TN];
    if constexpr (PROBE == 3) {
      typedef __attribute__((ext_vector_type(8))) short s16x8;
#pragma unroll
      for (int q = 0; q < NSET; ++q) {
#pragma unroll
        for (int a = 0; a < TM; ++a) fa[q][a] = __builtin_bit_cast(bf16x8, (s16x8){(short)lane, 1, 2, 3, 4, 5, 6, (short)q});
#pragma unroll
        for (int b = 0; b < TN; ++b) fb[q][b] = __builtin_bit_cast(bf16x8, (s16x8){(short)tap, 1, 2, 3, 4, 5, 6, (short)b});
      }
    } else if constexpr (RD) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) frag(ks, fa[ks], fb[ks]);
    } else {
      frag(0, fa[0], fb[0]);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cur = RD ? ks : (ks & 1);
      if (PROBE != 3 && !RD && ks + 1 < BK / 16) frag(ks + 1, fa[(ks + 1) % NSET], fb[(ks + 1) % NSET]);
      if constexpr (PROBE == 2 || PROBE == 4) {
#pragma unroll
        for (int a = 0; a < TM; ++a) asm volatile("" ::"v"(fa[cur][a]));
#pragma unroll
        for (int b = 0; b < TN; ++b) asm volatile("" ::"v"(fb[cur][b]));
      } else {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][a], fb[cur][b], acc[a][b], 0, 0, 0);
      }
    }
  };

  // ---- main loop ----------------------------------------------------------
  // issue order: halo(0), B(0) .. B(D-1) (D = STAGES - 1 K-tiles ahead);
  // at K-tile t: [B(t+D)], then at a chunk's first tap the next chunk's
  // halo. At t, the DMAs younger than B(t) are B(t+1) .. B(t+D-1) (those
  // issued) and, for the first D taps of a chunk, the next halo; the current
  // chunk's halo is older than B(t) (taps > D), so a counted wait for B(t)
  // retires it too.
  constexpr int D = STAGES - 1;
  if (PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  issue_halo(0, 0);
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < nk) issue_b(i, i);
  for (int t = 0; t < nk; ++t) {
    const int cc = t / taps;
    const int j = t - cc * taps;
    const int b_young = min(nk - 1 - t, D - 1);
    const bool h_young = j >= 1 && j <= D && cc + 1 < nc;
    if constexpr (PROBE == 1 || PROBE == 3 || PROBE == 4) {
      if (t == 0) wait_vmcnt<0>();
    } else if (h_young) {
      if (b_young >= 2) wait_vmcnt<2 * NB + NH>();
      else if (b_young == 1) wait_vmcnt<NB + NH>();
      else wait_vmcnt<NH>();
    } else {
      if (b_young >= 2) wait_vmcnt<2 * NB>();
      else if (b_young == 1) wait_vmcnt<NB>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();  // everyone's part landed; stage (t-1)%S and the previous halo are free
    constexpr bool LOOP_DMA = PROBE == 0 || PROBE == 2;
    if (LOOP_DMA && t + D < nk) issue_b(t + D, (t + D) % STAGES);
    if (LOOP_DMA && j == 0 && cc + 1 < nc) issue_halo(cc + 1, (cc + 1) & 1);
    compute(t, t % STAGES);
  }
  if (PRIO && wave >= 4) __builtin_amdgcn_s_setprio(0);
  __syncthreads();  // all DMA retired and all fragment reads done: reuse LDS

  char* Cg = (char*)Cp0;
  const long long c_off = zo * p.c_so + zi * p.c_si;
  const T* Rg = Rp ? (const T*)Rp + zo * p.r_so + zi * p.r_si : nullptr;
  epilogue_rows<T, TM, TN, WTN>(p, acc, (float*)smem, wave, lane, m0 + wm * WTM, n0 + wn * WTN, M, N, Cg, c_off, Rg,
                                true);
}

}  // namespace fpnmt
