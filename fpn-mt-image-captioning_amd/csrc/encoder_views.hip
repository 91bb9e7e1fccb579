// The multi-view encoder layer's output side (reference models/transformer.py
// EncoderLayer.call, :184-190):
//   out = baseline + sum_i Dropout(MHA_i.dense(attention_i))   i = 0 .. NSEG-1
// with the NSEG views' attention outputs side by side in one (M, NSEG*K)
// buffer. The views' output Dense layers (K -> N) are ONE launch here: one
// wave per view computes its view's partial tile on MFMA, and the epilogue
// adds each view's bias, applies its dropout mask and sums the views onto
// the residual. The M rows are the baseline tokens (B images x Lq: 32 rows
// at the C2 batch), so the former chain of NSEG latency-bound launches
// becomes one.
//
// Dropout mask of view i at (row, col): keep = uniform01(key, row * (NSEG*N)
// + i*N + col) >= p — the fpnmt_dropout mask of the virtual (M, NSEG*N)
// matrix of the views' pre-sum outputs, so the backward recomputes it over
// that matrix (fpnmt_view_proj_bwd_dz).
#include "common.h"

namespace fpnmt {
namespace {

__device__ __forceinline__ unsigned long long vp_key(unsigned long long seed, const long long* seed_dev) {
  return seed + (seed_dev ? (unsigned long long)(*seed_dev) * 0x9E3779B97F4A7C15ull : 0ull);
}

// epilogue shared by both element types: red[w][i][l] holds view w's
// partial for accumulator element i of lane l (32x32 MFMA layout)
template <typename T, int NSEG>
__device__ __forceinline__ void vp_epilogue(const float (*red)[16][64], int m0, int n0, int M, int N,
                                            const float* __restrict__ bias, const T* __restrict__ R,
                                            long long ldr, T* __restrict__ out, long long ldo, float p,
                                            unsigned long long key) {
  const float inv = p > 0.f ? 1.f / (1.f - p) : 1.f;
#pragma unroll
  for (int j = 0; j < 32 * 32 / (64 * NSEG); ++j) {
    const int e = threadIdx.x + 64 * NSEG * j;
    const int i = (e >> 6) & 15, l = e & 63;
    const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    const int col = n0 + (l & 31);
    if (row >= M || col >= N) continue;
    float s = R ? to_f32(R[(long long)row * ldr + col]) : 0.f;
#pragma unroll
    for (int w = 0; w < NSEG; ++w) {
      float v = red[w][i][l] + (bias ? bias[w * N + col] : 0.f);
      if (p > 0.f)
        v = uniform01(key, (uint64_t)row * (uint64_t)(NSEG * N) + (uint64_t)(w * N + col)) >= p ? v * inv : 0.f;
      s += v;
    }
    out[(long long)row * ldo + col] = from_f32<T>(s);
  }
}

// bf16: block = 32 rows x 32 columns, NSEG waves (wave w = view w), each
// wave's K range on v_mfma_f32_32x32x16_bf16 with 16-B fragment loads
// straight from global memory, U k-steps per register round (all loads of
// a round in flight together, the next round's issued under the MFMAs)
template <int NSEG>
__global__ __launch_bounds__(64 * NSEG) void view_proj_fwd_bf16_kernel(
    int M, int N, int K, const bf16* __restrict__ A, long long lda, const bf16* __restrict__ W,
    const float* __restrict__ bias, const bf16* __restrict__ R, long long ldr, bf16* __restrict__ out,
    long long ldo, float p, unsigned long long seed, const long long* __restrict__ seed_dev) {
  constexpr int U = 8;
  __shared__ float red[NSEG][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int tiles_n = (N + 31) / 32;
  const int m0 = (blockIdx.x / tiles_n) * 32, n0 = (blockIdx.x % tiles_n) * 32;
  const int arow = min(m0 + lr, M - 1), bcol = min(n0 + lr, N - 1);
  const bf16* ar = A + (long long)arow * lda + (long long)w * K + 8 * lh;
  const bf16* br = W + ((long long)w * N + bcol) * K + 8 * lh;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const int nks = K / 16;
  bf16x8 a0[U], b0[U], a1[U], b1[U];
  auto load = [&](int ks, bf16x8 (&av)[U], bf16x8 (&bv)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(ks + u, nks - 1) * 16;  // clamped: no branch around a load
      av[u] = *(const bf16x8*)(ar + k);
      bv[u] = *(const bf16x8*)(br + k);
    }
  };
  auto mma = [&](int ks, const bf16x8 (&av)[U], const bf16x8 (&bv)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (ks + u < nks) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[u], bv[u], acc, 0, 0, 0);
  };
  int ks = 0;
  load(0, a0, b0);
  while (ks < nks) {
    if (ks + U < nks) load(ks + U, a1, b1);
    mma(ks, a0, b0);
    ks += U;
    if (ks >= nks) break;
    if (ks + U < nks) load(ks + U, a0, b0);
    mma(ks, a1, b1);
    ks += U;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) red[w][i][lane] = acc[i];
  __syncthreads();
  vp_epilogue<bf16, NSEG>(red, m0, n0, M, N, bias, R, ldr, out, ldo, p, p > 0.f ? vp_key(seed, seed_dev) : 0ull);
}

// fp32 (the exact parity mode): the same block / epilogue, each lane's 16
// accumulator elements by plain fp32 FMAs in k order
template <int NSEG>
__global__ __launch_bounds__(64 * NSEG) void view_proj_fwd_f32_kernel(
    int M, int N, int K, const float* __restrict__ A, long long lda, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ R, long long ldr, float* __restrict__ out,
    long long ldo, float p, unsigned long long seed, const long long* __restrict__ seed_dev) {
  __shared__ float red[NSEG][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tiles_n = (N + 31) / 32;
  const int m0 = (blockIdx.x / tiles_n) * 32, n0 = (blockIdx.x % tiles_n) * 32;
  const int col = min(n0 + (lane & 31), N - 1);
  const float* br = W + ((long long)w * N + col) * K;
  float acc[16];
  const float* ar[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc[i] = 0.f;
    const int row = min(m0 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5), M - 1);
    ar[i] = A + (long long)row * lda + (long long)w * K;
  }
  for (int k = 0; k < K; ++k) {
    const float b = br[k];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = fmaf(ar[i][k], b, acc[i]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) red[w][i][lane] = acc[i];
  __syncthreads();
  vp_epilogue<float, NSEG>(red, m0, n0, M, N, bias, R, ldr, out, ldo, p, p > 0.f ? vp_key(seed, seed_dev) : 0ull);
}

// backward of the epilogue: dz[row, i*N + col] = dy[row, col] * keep_i / (1 - p)
// over the virtual (M, NSEG*N) matrix, and db[i*N + col] += its column sums
// (4 row groups, summed in group order: deterministic)
template <typename T>
__global__ __launch_bounds__(256) void view_proj_dz_kernel(int M, int N, int NSEG, const T* __restrict__ dy,
                                                           long long lddy, T* __restrict__ dz,
                                                           float* __restrict__ db, float p,
                                                           unsigned long long seed,
                                                           const long long* __restrict__ seed_dev) {
  __shared__ float red[4][64];
  const int NV = NSEG * N;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const unsigned long long key = p > 0.f ? vp_key(seed, seed_dev) : 0ull;
  const float inv = p > 0.f ? 1.f / (1.f - p) : 1.f;
  float sum = 0.f;
  if (c < NV) {
    const int cc = c % N;
    for (int r = rg; r < M; r += 4) {
      float v = to_f32(dy[(long long)r * lddy + cc]);
      if (p > 0.f) v = uniform01(key, (uint64_t)r * (uint64_t)NV + (uint64_t)c) >= p ? v * inv : 0.f;
      dz[(long long)r * NV + c] = from_f32<T>(v);
      sum += v;
    }
  }
  red[rg][threadIdx.x & 63] = sum;
  __syncthreads();
  if (rg == 0 && c < NV && db) db[c] += ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                        red[3][threadIdx.x];
}

}  // namespace
}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

int fpnmt_view_proj_fwd(int dtype, int m, int n, int k, int nseg, const void* A, long long lda, const void* W,
                        const float* bias, const void* R, long long ldr, void* out, long long ldo, float drop_p,
                        unsigned long long seed, const long long* seed_dev, fpnmt_stream_t stream) {
  if (dtype != FPNMT_BF16 && dtype != FPNMT_F32) return fail(FPNMT_E_ARG, "view_proj_fwd: bad dtype");
  if (nseg != 4) return fail(FPNMT_E_UNSUPPORTED, "view_proj_fwd: nseg must be 4 (NUM_OF_PYRAMIDS - 1)");
  if (m < 0 || n <= 0 || k <= 0 || k % 16 || lda < (long long)nseg * k || ldo < n || (R && ldr < n))
    return fail(FPNMT_E_ARG, "view_proj_fwd: bad shape (k % 16 == 0, lda >= nseg*k, ldo / ldr >= n)");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return fail(FPNMT_E_ARG, "view_proj_fwd: drop_p must be in [0, 1)");
  if (m == 0) return 0;
  if (!A || !W || !out) return fail(FPNMT_E_ARG, "view_proj_fwd: null pointer");
  const dim3 grid((unsigned)(cdiv(m, 32) * cdiv(n, 32)));
  if (dtype == FPNMT_BF16) {
    if (lda % 8 || k % 8 || ((uintptr_t)A | (uintptr_t)W) & 15)
      return fail(FPNMT_E_ARG, "view_proj_fwd: bf16 operands need 16-B aligned rows");
    hipLaunchKernelGGL((view_proj_fwd_bf16_kernel<4>), grid, dim3(256), 0, S(stream), m, n, k, (const bf16*)A, lda,
                       (const bf16*)W, bias, (const bf16*)R, ldr, (bf16*)out, ldo, drop_p, seed, seed_dev);
  } else {
    hipLaunchKernelGGL((view_proj_fwd_f32_kernel<4>), grid, dim3(256), 0, S(stream), m, n, k, (const float*)A, lda,
                       (const float*)W, bias, (const float*)R, ldr, (float*)out, ldo, drop_p, seed, seed_dev);
  }
  return check_launch("view_proj_fwd");
}

int fpnmt_view_proj_bwd_dz(int dtype, int m, int n, int nseg, const void* dy, long long lddy, void* dz, float* db,
                           float drop_p, unsigned long long seed, const long long* seed_dev,
                           fpnmt_stream_t stream) {
  if (dtype != FPNMT_BF16 && dtype != FPNMT_F32) return fail(FPNMT_E_ARG, "view_proj_bwd_dz: bad dtype");
  if (m < 0 || n <= 0 || nseg <= 0 || lddy < n) return fail(FPNMT_E_ARG, "view_proj_bwd_dz: bad shape");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return fail(FPNMT_E_ARG, "view_proj_bwd_dz: drop_p must be in [0, 1)");
  if (m == 0) return 0;
  if (!dy || !dz) return fail(FPNMT_E_ARG, "view_proj_bwd_dz: null pointer");
  if (db) {  // an immediate accumulation into db: queued reductions into it run first
    const int st = defer_touch(db, db + (long long)nseg * n, S(stream));
    if (st) return st;
  }
  const dim3 grid((unsigned)cdiv((long long)nseg * n, 64));
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((view_proj_dz_kernel<bf16>), grid, dim3(256), 0, S(stream), m, n, nseg, (const bf16*)dy,
                       lddy, (bf16*)dz, db, drop_p, seed, seed_dev);
  else
    hipLaunchKernelGGL((view_proj_dz_kernel<float>), grid, dim3(256), 0, S(stream), m, n, nseg, (const float*)dy,
                       lddy, (float*)dz, db, drop_p, seed, seed_dev);
  return check_launch("view_proj_bwd_dz");
}

}  // extern "C"
