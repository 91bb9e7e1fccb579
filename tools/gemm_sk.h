// Round-4 negative result, kept for tools/fwd_bench.hip -DFB_SPREAD only (the
// library does not build it): a stream-K form of the 8-wave 128x256 pipe conv
// kernel. Correct (the bench checks the first and the last timed launch, i.e.
// the tile counters across replays) but slower: C2 P3 3x3 70.5 us against
// 51.8 us for the shipped kernel (51.8 us for this kernel with one block per
// tile, so the loop itself is not the cost). Each split segment stores a
// 128 KB fp32 slab from one CU, and the per-CU store issue rate (~7-14 B per
// cycle, MI355X_MICROARCH.md) makes two such stores plus the last arriver's
// reads and the agent-scope fences ~10-20 us per block against the ~10 us
// that filling the idle quarter of the chip could save.
#pragma once
#include "../fpn-mt-image-captioning_amd/csrc/gemm_dispatch.h"

namespace fpnmt {

// ---------------------------------------------------------------------------
// Stream-K form of gemm_pipe_kernel (direct epilogue, 3-stage ring with the
// spread DMA issue) for launches whose tile count leaves part of the chip idle
// in the last wave of blocks (the C2 P3 conv: 196 128x256 tiles on 256 CUs;
// P3 at batch 64: 392 = 1.53 waves). The ntile * nkt (tile, K-tile) units are
// cut into gridDim.x contiguous ranges, one per block; a block walks its
// range as segments (the part of one tile inside it). A tile covered by one
// segment gets the normal epilogue. A tile split over several blocks: every
// segment stores its fp32 accumulators to a slab (slot 2 * block + 0 for a
// block's first segment, + 1 for its last) and takes a ticket on the tile's
// counter (cdna_hip_programming.md §5 "In-launch split-K reduction", counter
// form: plain slab stores, vmcnt drain, barrier, one agent-scope release,
// relaxed agent fetch_add); the block drawing the last ticket acquires, sums
// the tile's segments in segment (k) order — its own from registers, the
// others from their slabs, so the sum is the same whoever arrives last — and
// runs the epilogue. No block waits for another (nothing depends on dispatch
// order or co-residency); the last arriver re-zeroes the counter (the
// workspace starts zeroed), so a graph replays it as is.
template <int BM, int BN, int WM, int WN, int AM, int NT, int STAGES>
__global__ __launch_bounds__(NT) void gemm_pipe_sk_kernel(const GemmParams p) {
  typedef bf16 T;
  constexpr int BK = 64, CPR = BK / 8, ROWB = BK * 2;
  static_assert(WM * WN * 64 == NT && STAGES >= 2, "");
  static_assert(AM == A_ROW || AM == A_IM2COL, "k-contiguous A only");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int NA = BM * CPR / NT, NB = BN * CPR / NT;
  static_assert((BM * CPR) % NT == 0 && (BN * CPR) % NT == 0 && NA >= 1 && NB >= 1, "");
  constexpr int NQ = TM * TN * 4;                 // f32x4 accumulator groups per thread
  constexpr long long SLAB = (long long)NT * NQ;  // f32x4 per slab (= BM * BN / 4)
  constexpr int PER_STAGE = NA + NB;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int ntile = p.tiles_m * p.tiles_n;
  const int nkt = p.K / BK;
  // 32-bit unit arithmetic (host-checked: gridDim.x * units < 2^31)
  const unsigned U = (unsigned)(ntile * nkt);
  const unsigned G = gridDim.x;
  const int blk = xcd_remap(blockIdx.x, (int)G);  // consecutive ranges (a tile's segments) share an XCD
  auto start_of = [&](unsigned bb) { return bb * U / G; };
  const unsigned s_b = start_of(blk), e_b = start_of(blk + 1);
  const T* zero = (const T*)p.zero16;
  const T* __restrict__ Bg = (const T*)p.B;
  const int N = p.N;
  f32x4* slabs = (f32x4*)p.ws_part;
  typedef __attribute__((address_space(3))) void lds_void;

  for (unsigned u = s_b; u < e_b;) {
    const int tile = (int)(u / (unsigned)nkt);
    const int k0 = (int)(u - (unsigned)tile * nkt);
    const int k1 = min(nkt, k0 + (int)(e_b - u));
    const bool first_seg = u == s_b;
    u += k1 - k0;
    const int nk = k1 - k0;
    __syncthreads();  // the previous segment's fragment reads / flag read are done: the ring is free

    // (no m-grouped launches: the host takes this form for single problems)
    const int tmi = tile / p.tiles_n;
    const int tni = tile - tmi * p.tiles_n;
    void* Cp0 = p.C;
    const void* Rp = p.R;
    const int M = p.M;
    const int gH = p.H, gW = p.W, gHo = p.Ho, gWo = p.Wo;
    const FastDiv gfdHoWo = p.fd_HoWo, gfdWo = p.fd_Wo;
    const int m0 = tmi * BM, n0 = tni * BN;
    const T* __restrict__ Ag = (const T*)p.A;

    // per-thread DMA sources of this tile (gemm_pipe_kernel's setup)
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
    struct TileSrc { int k0, tap, tap_off; };
    auto tile_src = [&](int kt) {  // kt: absolute K-tile index
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

    f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int bb = 0; bb < TN; ++bb)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][bb][i] = 0.f;
    auto frag = [&](const char* As, const char* Bs, int ks, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
      const int c = ks * 2 + lh;
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const int row = wm * WTM + t * 32 + lr;
        af[t] = *(const bf16x8*)(As + row * ROWB + ((c ^ pipe_sw<BK>(row)) << 4));
      }
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int row = wn * WTN + t * 32 + lr;
        bfr[t] = *(const bf16x8*)(Bs + row * ROWB + ((c ^ pipe_sw<BK>(row)) << 4));
      }
    };
    auto compute_mid = [&](int stage, auto&& mid) {
      const char* As = smem + stage * STAGE_BYTES;
      const char* Bs = As + A_BYTES;
      bf16x8 fa[2][TM], fb[2][TN];
      frag(As, Bs, 0, fa[0], fb[0]);
      static_for<0, BK / 16>([&](auto ksc) {
        constexpr int ks = decltype(ksc)::value;
        if constexpr (ks + 1 < BK / 16) frag(As, Bs, ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
        mid(ksc);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int bb = 0; bb < TN; ++bb)
            acc[a][bb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[ks & 1][bb], fa[ks & 1][a], acc[a][bb], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      });
    };

    bf16x4 rpre[TM][TN][4];
    const T* Rg0 = (const T*)Rp;
    if (Rg0) prefetch_r_direct<TM, TN>(p, Rg0, m0 + wm * WTM, n0 + wn * WTN, M, N, rpre);

#pragma unroll
    for (int i = 0; i < STAGES - 1; ++i)
      if (i < nk) issue_range(tile_src(k0 + i), i, std::integral_constant<int, 0>{}, std::integral_constant<int, PER_STAGE>{});
    for (int t = 0; t < nk; ++t) {
      const int ahead = min(nk - 1 - t, STAGES - 2);
      if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * PER_STAGE>();
      else if (STAGES > 3 && ahead == 2) wait_vmcnt<(STAGES > 3 ? 2 : 0) * PER_STAGE>();
      else if (ahead == 1) wait_vmcnt<PER_STAGE>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      const bool more = t + STAGES - 1 < nk;
      const TileSrc ts = tile_src(k0 + t + STAGES - 1);
      const int st = (t + STAGES - 1) % STAGES;
      compute_mid(t % STAGES, [&](auto ksc) {
        constexpr int ks = decltype(ksc)::value, NKS = BK / 16;
        if (more)
          issue_range(ts, st, std::integral_constant<int, ks * PER_STAGE / NKS>{},
                      std::integral_constant<int, (ks + 1) * PER_STAGE / NKS>{});
      });
    }

    if (!(k0 == 0 && k1 == nkt)) {
      // ---- split tile: slab, ticket, the last arriver sums in segment order ----
      const unsigned tstart = (unsigned)tile * nkt, tlast = tstart + nkt - 1;
      unsigned bf = tstart * G / U;  // first / last block whose range meets the tile
      while (bf + 1 < G && start_of(bf + 1) <= tstart) ++bf;
      while (bf > 0 && start_of(bf) > tstart) --bf;
      unsigned bl = tlast * G / U;
      while (bl + 1 < G && start_of(bl + 1) <= tlast) ++bl;
      while (bl > 0 && start_of(bl) > tlast) --bl;
      const int nseg = (int)(bl - bf) + 1;
      f32x4* mine = slabs + (long long)(2 * blk + (first_seg ? 0 : 1)) * SLAB;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int bb = 0; bb < TN; ++bb)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 v = {acc[a][bb][4 * g], acc[a][bb][4 * g + 1], acc[a][bb][4 * g + 2], acc[a][bb][4 * g + 3]};
            mine[(long long)((a * TN + bb) * 4 + g) * NT + tid] = v;
          }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = (int*)smem;  // the one __shared__ array (a second object de-pipelines the loop)
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(p.ws_cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == (unsigned)(nseg - 1);
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(p.ws_cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        flag[0] = last;
      }
      __syncthreads();
      const bool last = flag[0] != 0;
      if (!last) continue;  // (the next segment starts with a barrier before its DMA)
      const int myidx = blk - (int)bf;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int bb = 0; bb < TN; ++bb) {
          f32x4 own[4], tot[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            own[g] = f32x4{acc[a][bb][4 * g], acc[a][bb][4 * g + 1], acc[a][bb][4 * g + 2], acc[a][bb][4 * g + 3]};
            tot[g] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
          for (int i = 0; i < nseg; ++i) {
            const unsigned bb2 = bf + i;
            const f32x4* src = slabs + (long long)(2 * bb2 + (start_of(bb2) < tstart ? 1 : 0)) * SLAB +
                               (long long)((a * TN + bb) * 4) * NT + tid;
            f32x4 v[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) v[g] = src[(long long)g * NT];  // (own slot too: loads stay unconditional)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const f32x4 x = i == myidx ? own[g] : v[g];
              tot[g] = i == 0 ? x : tot[g] + x;
            }
          }
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[a][bb][4 * g + e] = tot[g][e];
        }
    }
    epilogue_direct<TM, TN>(p, acc, m0 + wm * WTM, n0 + wn * WTN, M, N, (char*)Cp0, 0, Rg0 != nullptr, rpre);
  }
}

// Stream-K for the 8-wave 128x256 tiles (gemm_pipe_sk_kernel): when the
// last wave of tiles would leave >= 15 % of the CUs idle (C2 P3: 196 tiles
// on 256 CUs; P3 at batch 64: 392), one block per CU walks an equal share of
// the (tile, K-tile) units; split tiles are summed in k order by their last
// arriving block through the workspace's slabs and tile counters.
template <int AM>
static bool launch_pipe_sk(GemmParams& p, int batch, int splits, hipStream_t s, int* rc) {
  constexpr int BM = 128, BN = 256;
  if (batch != 1 || splits > 1 || p.ngroups > 0 || !g_split_ws.part || !g_split_ws.cnt || p.K % 64) return false;
  const int tm = cdiv(p.M, BM);
  const long long ntile = (long long)tm * cdiv(p.N, BN), cus = cu_count_dispatch(), nkt = p.K / 64;
  const long long rem = ntile % cus;
  if (rem == 0 || rem * 100 >= cus * 85 || nkt < 8) return false;
  const long long U = ntile * nkt;
  const int G = (int)std::min<long long>(cus, U);
  if ((long long)G * U >= (1LL << 31)) return false;  // the kernel's 32-bit unit arithmetic
  if (2LL * G * BM * BN > g_split_ws.part_floats || ntile > g_split_ws.cnt_n) return false;
  p.tiles_m = tm;
  p.tiles_n = cdiv(p.N, BN);
  p.split_k = 1;
  p.k_per_split = p.K;
  p.zero16 = g_split_ws.zero;
  p.ws_part = g_split_ws.part;
  p.ws_cnt = g_split_ws.cnt;
  hipLaunchKernelGGL((gemm_pipe_sk_kernel<BM, BN, 2, 4, AM, 512, 3>), dim3(G), dim3(512), 0, s, p);
  *rc = check_launch("gemm_pipe_sk_kernel");
  return true;
}

}  // namespace fpnmt
