// HBM-bound kernels of the hot path: activation backward (+ bias grad),
// casts, dropout, adds, max pooling, the fused FPN top-down sweep, the
// co-attention spatial softmax, LayerNorm, embedding+posenc, masked CE.
// All NHWC / row-major, vectorised 16 B per lane where the shape allows.
#include "common.h"
#include <initializer_list>

namespace fpnmt {

template <typename T> struct V16;
template <> struct V16<bf16> { typedef bf16x8 type; static constexpr int n = 8; };
template <> struct V16<float> { typedef f32x4 type; static constexpr int n = 4; };

static inline int grid_for(long long work, int block, int cap = 4096) {
  long long g = (work + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

// ------------------------------------------------------------------------
// activation backward: dz = dy * act'(y); db[col] += sum_rows dz
// Block = 256 threads as (row lanes RL, a power of two) x (column groups GT):
// every thread is busy even for narrow C (64 channels = 8 groups -> 32 row
// lanes); column sums are reduced through LDS in a fixed tree order.
// grid: x = column tiles of GT groups, y = row chunks of rows_per_chunk rows.
// One row chunk: the block adds its sums to db (the column's only writer);
// several: per-chunk partials to ws, summed in chunk order by act_colsum.
static inline __host__ __device__ int pow2_floor(int v) {
  int r = 1;
  while (r * 2 <= v) r *= 2;
  return r;
}
// one block of act_bwd_kernel: column tile bx, row chunk by (also run by the
// batched deferred bias-gradient kernel with the immediate launch's grid)
template <typename T, bool VEC>
__device__ __forceinline__ void act_bwd_block(int bx, int by, long long rows, int c, int act, float a,
                                              const T* __restrict__ dy, const T* __restrict__ y, T* dz, float* db,
                                              float* __restrict__ ws, int rows_per_chunk, bool write, float dp,
                                              unsigned long long dseed, const long long* dseed_dev, int GT,
                                              float* red) {
  constexpr int VN = VEC ? V16<T>::n : 1;
  const int groups = c / VN;
  const int RL = pow2_floor(256 / GT);
  const int tg = threadIdx.x % GT, tr = threadIdx.x / GT;
  const int g = bx * GT + tg;
  const bool active = tr < RL && g < groups;
  const long long r0 = (long long)by * rows_per_chunk;
  const long long r1 = min(rows, r0 + rows_per_chunk);
  float sum[VN];
#pragma unroll
  for (int j = 0; j < VN; ++j) sum[j] = 0.f;
  // fused-dropout mask of the forward GEMM epilogue (keep / (1 - p))
  const unsigned long long dkey =
      dp > 0.f ? dseed + (dseed_dev ? (unsigned long long)(*dseed_dev) * 0x9E3779B97F4A7C15ull : 0ull) : 0ull;
  const float dsc = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  if constexpr (VEC) {
    // 4 rows per iteration: all loads issued before any use (hides HBM latency)
    typedef typename V16<T>::type VT;
    constexpr int UR = 4;
    for (long long rb = r0 + tr; active && rb < r1; rb += (long long)UR * RL) {
      VT d[UR], yy[UR];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        // clamped row: loads are unconditional (no branch around a load), the
        // rows past the chunk are skipped below
        const long long r = min(rb + (long long)u * RL, r1 - 1);
        const long long idx = r * c + (long long)g * VN;
        d[u] = *(const VT*)(dy + idx);
        if (act != FPNMT_ACT_NONE) yy[u] = *(const VT*)(y + idx);
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const long long r = rb + (long long)u * RL;
        if (r >= r1) break;
        if (act != FPNMT_ACT_NONE || dp > 0.f) {
#pragma unroll
          for (int j = 0; j < VN; ++j) {
            float t = to_f32(d[u][j]);
            if (dp > 0.f)
              t = uniform01(dkey, (uint64_t)r * (uint64_t)c + (uint64_t)(g * VN + j)) >= dp ? t * dsc : 0.f;
            if (act != FPNMT_ACT_NONE) t *= act_grad_from_y(to_f32(yy[u][j]), act, a);
            d[u][j] = from_f32<T>(t);
          }
        }
        if (write) *(VT*)(dz + r * c + (long long)g * VN) = d[u];
#pragma unroll
        for (int j = 0; j < VN; ++j) sum[j] += to_f32(d[u][j]);
      }
    }
  }
  for (long long r = r0 + tr; !VEC && active && r < r1; r += RL) {
    const long long idx = r * c + (long long)g * VN;
    {
      float d = to_f32(dy[idx]);
      if (dp > 0.f) d = uniform01(dkey, (uint64_t)idx) >= dp ? d * dsc : 0.f;
      if (act != FPNMT_ACT_NONE) d *= act_grad_from_y(to_f32(y[idx]), act, a);
      T dt = from_f32<T>(d);
      if (write) dz[idx] = dt;
      sum[0] += to_f32(dt);
    }
  }
  if (db) {
#pragma unroll
    for (int j = 0; j < VN; ++j) red[threadIdx.x * VN + j] = sum[j];
    __syncthreads();
    for (int off = RL / 2; off > 0; off >>= 1) {  // fixed-order tree over the row lanes
      if (tr < off) {
#pragma unroll
        for (int j = 0; j < VN; ++j) red[threadIdx.x * VN + j] += red[(threadIdx.x + off * GT) * VN + j];
      }
      __syncthreads();
    }
    if (tr == 0 && g < groups) {
      if (ws) {  // per-chunk partials, summed in chunk order by act_colsum_kernel
#pragma unroll
        for (int j = 0; j < VN; ++j) ws[(long long)by * c + g * VN + j] = red[tg * VN + j];
      } else {  // one row chunk: this block is the column's only writer
#pragma unroll
        for (int j = 0; j < VN; ++j) db[g * VN + j] += red[tg * VN + j];
      }
    }
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void act_bwd_kernel(long long rows, int c, int act, float a,
                                                      const T* __restrict__ dy,
                                                      const T* __restrict__ y, T* dz, float* db,
                                                      float* __restrict__ ws, int rows_per_chunk, bool write,
                                                      float dp, unsigned long long dseed,
                                                      const long long* dseed_dev, int GT) {
  __shared__ float red[256 * (VEC ? V16<T>::n : 1)];
  act_bwd_block<T, VEC>(blockIdx.x, blockIdx.y, rows, c, act, a, dy, y, dz, db, ws, rows_per_chunk, write, dp,
                        dseed, dseed_dev, GT, red);
}

// the queued bias gradients of a deferred region, one block per (job, column
// tile, row chunk): exactly the blocks of their immediate act_bwd launches
__global__ __launch_bounds__(256) void direct_colsum_kernel(const DirectBatch B) {
  __shared__ float red[256 * 8];
  int k = 0;
#pragma unroll
  for (int i = 1; i < DIRECT_PER_LAUNCH; ++i)
    if (i < B.n && (int)blockIdx.x >= B.j[i].blk0) k = i;
  DefDirect J = B.j[0];
#pragma unroll
  for (int i = 1; i < DIRECT_PER_LAUNCH; ++i)
    if (i == k) J = B.j[i];
  const int local = blockIdx.x - J.blk0;
  const int by = local / J.gx, bx = local - by * J.gx;
  float* ws = J.ws;  // null: one chunk adding into db itself
  if (J.dtype == FPNMT_BF16) {
    if (J.vec)
      act_bwd_block<bf16, true>(bx, by, J.rows, J.c, FPNMT_ACT_NONE, 0.f, (const bf16*)J.dy, nullptr, nullptr, J.db,
                                ws, J.rpc, false, 0.f, 0ull, nullptr, J.gt, red);
    else
      act_bwd_block<bf16, false>(bx, by, J.rows, J.c, FPNMT_ACT_NONE, 0.f, (const bf16*)J.dy, nullptr, nullptr,
                                 J.db, ws, J.rpc, false, 0.f, 0ull, nullptr, J.gt, red);
  } else {
    if (J.vec)
      act_bwd_block<float, true>(bx, by, J.rows, J.c, FPNMT_ACT_NONE, 0.f, (const float*)J.dy, nullptr, nullptr,
                                 J.db, ws, J.rpc, false, 0.f, 0ull, nullptr, J.gt, red);
    else
      act_bwd_block<float, false>(bx, by, J.rows, J.c, FPNMT_ACT_NONE, 0.f, (const float*)J.dy, nullptr, nullptr,
                                  J.db, ws, J.rpc, false, 0.f, 0ull, nullptr, J.gt, red);
  }
}

int direct_colsum_launch(const DirectBatch& B, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(direct_colsum_kernel, dim3(blocks), dim3(256), 0, s, B);
  return check_launch("direct_colsum_kernel");
}

// db[col] += sum_k ws[k][col]: CB columns x (1024/CB) chunk lanes per block,
// each lane keeping 4 independent partial sums so 4 loads are in flight (the
// chunk count reaches ~1000 while narrow c gives only a few blocks); the sum
// order is fixed, so the result is deterministic. Columns >= c_split go to
// db2[col - c_split] (the LayerNorm gamma / beta pair).
template <int CB>
__global__ __launch_bounds__(1024) void act_colsum_kernel(int chunks, int c, const float* __restrict__ ws,
                                                          float* __restrict__ db, int c_split = 1 << 30,
                                                          float* __restrict__ db2 = nullptr) {
  constexpr int KL = 1024 / CB;
  __shared__ float red[KL][CB];
  const int cl = threadIdx.x % CB, kl = threadIdx.x / CB;
  const int col = blockIdx.x * CB + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < c) {
    int k = kl;
    for (; k + 3 * KL < chunks; k += 4 * KL) {
      s0 += ws[(long long)k * c + col];
      s1 += ws[(long long)(k + KL) * c + col];
      s2 += ws[(long long)(k + 2 * KL) * c + col];
      s3 += ws[(long long)(k + 3 * KL) * c + col];
    }
    for (; k < chunks; k += KL) s0 += ws[(long long)k * c + col];
  }
  red[kl][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (kl == 0 && col < c) {
    float s = red[0][cl];
#pragma unroll 8
    for (int q = 1; q < KL; ++q) s += red[q][cl];
    if (col < c_split) {
      if (db) db[col] += s;  // one writer per column
    } else if (db2) {
      db2[col - c_split] += s;
    }
  }
}

void colsum_launch(int chunks, int c, const float* ws, float* db, hipStream_t s, int c_split, float* db2) {
  // narrow c: fewer columns per block so more CUs share the chunk reads
  if (defer_owns(ws)) {  // partials in the deferred arena: queued, same CB
    defer_colsum(chunks, c, ws, db, c_split, db2, c >= 64 * 64 ? 64 : c >= 32 * 32 ? 32 : 16, s);
    return;
  }
  if (defer_active()) {  // partials fell back to the scratch (arena full): an immediate add
    // into db / db2 — run any queued sum into them first, keeping immediate-mode order
    const int n1 = std::min(c, c_split);
    if (db && n1 > 0) defer_touch(db, db + n1, s);
    if (db2 && c > c_split) defer_touch(db2, db2 + (c - c_split), s);
  }
  if (c >= 64 * 64)
    hipLaunchKernelGGL(act_colsum_kernel<64>, dim3(cdiv(c, 64)), dim3(1024), 0, s, chunks, c, ws, db, c_split, db2);
  else if (c >= 32 * 32)
    hipLaunchKernelGGL(act_colsum_kernel<32>, dim3(cdiv(c, 32)), dim3(1024), 0, s, chunks, c, ws, db, c_split, db2);
  else
    hipLaunchKernelGGL(act_colsum_kernel<16>, dim3(cdiv(c, 16)), dim3(1024), 0, s, chunks, c, ws, db, c_split, db2);
}

struct ActBwdGrid {
  bool vec;
  int gx, gy, rpc, gt;
};
template <typename T>
static ActBwdGrid act_bwd_grid(long long rows, int c, bool aligned, bool colsum) {
  ActBwdGrid G;
  G.vec = (c % V16<T>::n) == 0 && aligned;
  const int groups = G.vec ? c / V16<T>::n : c;
  if (colsum) {
    // column sums in ONE launch when a block can walk every row: narrow column
    // tiles (~64 blocks across the columns) with <= 8 rows per row lane —
    // e.g. the decoder's 992 x 512 Dense biases (the two-launch partials +
    // act_colsum form costs two latency-bound launches; at 16 rows per lane,
    // 992 x 2048, one launch took 19 us against 11 for the two)
    const int gt = std::max(1, std::min(256, groups / 64));
    const int rl = pow2_floor(256 / gt);
    if ((rows + rl - 1) / rl <= 8) {
      G.gt = gt;
      G.gx = cdiv(groups, gt);
      G.gy = 1;
      G.rpc = (int)rows;
      return G;
    }
  }
  const int GT = groups < 256 ? groups : 256;
  const int RL = pow2_floor(256 / GT);
  G.gt = GT;
  G.gx = cdiv(groups, GT);
  // ~1024 blocks in total, each thread walking >= 4 rows when possible
  long long chunks = 1024 / G.gx;
  if (chunks < 1) chunks = 1;
  const long long max_chunks = (rows + 4LL * RL - 1) / (4LL * RL);
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  G.rpc = (int)((rows + chunks - 1) / chunks);
  G.gy = (int)((rows + G.rpc - 1) / G.rpc);
  return G;
}

template <typename T>
static int act_bwd_t(long long rows, int c, int act, float a, const void* dy, const void* y,
                     void* dz, float* db, float* ws, float dp, unsigned long long dseed,
                     const long long* dseed_dev, hipStream_t s) {
  const bool write = !(act == FPNMT_ACT_NONE && dp <= 0.f && dz == dy);
  if (!write && !db) return 0;
  const bool aligned = ((uintptr_t)dy % 16 == 0) && ((uintptr_t)dz % 16 == 0) &&
                       (y == nullptr || (uintptr_t)y % 16 == 0);
  const ActBwdGrid G = act_bwd_grid<T>(rows, c, aligned, db != nullptr);
  // one row chunk: the block adds its column sums directly; several: per-chunk
  // partials (caller's ws, else the process scratch) + act_colsum_kernel,
  // summed in chunk order (no atomics: the same bits on every run)
  if (!db || G.gy == 1) ws = nullptr;
  else if (defer_active() || !ws) ws = partial_f32((long long)G.gy * c);
  if (db && G.gy == 1) {  // the block adds into db directly: keep the order of queued sums into it
    const int st = defer_touch(db, db + c, s);
    if (st) return st;
  }
  if (db && G.gy > 1 && !ws) return fail(FPNMT_E_ARG, "act_bwd: column sums need a workspace (fpnmt_act_bwd_ws_bytes)");
  dim3 grid(G.gx, G.gy);
  if (G.vec)
    hipLaunchKernelGGL((act_bwd_kernel<T, true>), grid, dim3(256), 0, s, rows, c, act, a,
                       (const T*)dy, (const T*)y, (T*)dz, db, ws, G.rpc, write, dp, dseed, dseed_dev, G.gt);
  else
    hipLaunchKernelGGL((act_bwd_kernel<T, false>), grid, dim3(256), 0, s, rows, c, act, a,
                       (const T*)dy, (const T*)y, (T*)dz, db, ws, G.rpc, write, dp, dseed, dseed_dev, G.gt);
  if (ws) colsum_launch(G.gy, c, ws, db, s);
  return check_launch("act_bwd");
}

// ------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void cast_kernel(long long n, const TI* __restrict__ in, TO* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = from_f32<TO>(to_f32(in[i]));
}

template <typename T>
__global__ void dropout_kernel(long long n, float p, unsigned long long seed,
                               const long long* seed_dev, const T* x, T* y) {
  const unsigned long long key = seed + (seed_dev ? (unsigned long long)(*seed_dev) * 0x9E3779B97F4A7C15ull : 0ull);
  const float sc = 1.f / (1.f - p);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float u = uniform01(key, (uint64_t)i);
    y[i] = from_f32<T>(u >= p ? to_f32(x[i]) * sc : 0.f);
  }
}

template <typename T>
__global__ void add_kernel(long long n, const T* a, const T* b, T* out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = from_f32<T>(to_f32(a[i]) + to_f32(b[i]));
}

// ------------------------------------------------------------------------
// max pooling (NHWC). Thread per output element x VN channels (c fastest).
// Optional argmax: window tap (r*kw+q) of the first max, 255 if no tap is valid.
template <typename T, int VN>
struct Ld8 {
  static __device__ __forceinline__ void load(const T* p, float* v) {
#pragma unroll
    for (int j = 0; j < VN; ++j) v[j] = to_f32(p[j]);
  }
  static __device__ __forceinline__ void store(T* p, const float* v) {
#pragma unroll
    for (int j = 0; j < VN; ++j) p[j] = from_f32<T>(v[j]);
  }
};
template <>
struct Ld8<bf16, 8> {
  static __device__ __forceinline__ void load(const bf16* p, float* v) {
    const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = to_f32(t[j]);
  }
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    bf16x8 t;
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = from_f32<bf16>(v[j]);
    *(bf16x8*)p = t;
  }
};
template <>
struct Ld8<float, 8> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[j + 4]; }
    *(f32x4*)p = a;
    *(f32x4*)(p + 4) = b;
  }
};

template <typename T, int VN>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(int n, int h, int w, int c, int kh, int kw, int sh,
                                                          int sw, int pt, int pl, int ho, int wo,
                                                          const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ argmax) {
  const int cg = c / VN;
  const long long total = (long long)n * ho * wo * cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cg) * VN;
    long long t = i / cg;
    const int ow = (int)(t % wo);
    t /= wo;
    const int oh = (int)(t % ho);
    const int nn = (int)(t / ho);
    float m[VN], v[VN];
    int am[VN];
#pragma unroll
    for (int j = 0; j < VN; ++j) { m[j] = -INFINITY; am[j] = 255; }
    for (int r = 0; r < kh; ++r) {
      const int ih = oh * sh - pt + r;
      if (ih < 0 || ih >= h) continue;
      for (int q = 0; q < kw; ++q) {
        const int iw = ow * sw - pl + q;
        if (iw < 0 || iw >= w) continue;
        Ld8<T, VN>::load(x + (((long long)nn * h + ih) * w + iw) * c + ch, v);
#pragma unroll
        for (int j = 0; j < VN; ++j)
          if (v[j] > m[j] || am[j] == 255) { m[j] = v[j]; am[j] = r * kw + q; }
      }
    }
    const long long o = (((long long)nn * ho + oh) * wo + ow) * c + ch;
    Ld8<T, VN>::store(y + o, m);
    if (argmax) {
#pragma unroll
      for (int j = 0; j < VN; ++j) argmax[o + j] = (uint8_t)am[j];
    }
  }
}

// gather form: thread per INPUT element x VN channels; sums dy over the windows
// whose first max it is (from argmax when given, else recomputed from x).
// xact (optional): the pool's input again, as the producer's activation
// output; the sum is then multiplied by that activation's derivative at x
// (one coalesced 16-B load per thread; reading it off the routed windows'
// maxima instead cost a load per window: stem 55 -> 66 us)
template <typename T, int VN>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int n, int h, int w, int c, int kh, int kw, int sh,
                                                          int sw, int pt, int pl, int ho, int wo,
                                                          const T* __restrict__ x,
                                                          const uint8_t* __restrict__ argmax,
                                                          const T* __restrict__ dy, T* __restrict__ dx,
                                                          const T* __restrict__ xact, int act, float alpha) {
  const int cg = c / VN;
  const long long total = (long long)n * h * w * cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cg) * VN;
    long long t = i / cg;
    const int iw = (int)(t % w);
    t /= w;
    const int ih = (int)(t % h);
    const int nn = (int)(t / h);
    // output windows covering (ih, iw): oh*sh - pt <= ih <= oh*sh - pt + kh - 1
    const int oh_lo = max(0, (ih + pt - kh + sh) / sh), oh_hi = min(ho - 1, (ih + pt) / sh);
    const int ow_lo = max(0, (iw + pl - kw + sw) / sw), ow_hi = min(wo - 1, (iw + pl) / sw);
    float g[VN], d[VN], v[VN], mk[VN];
#pragma unroll
    for (int j = 0; j < VN; ++j) { g[j] = 0.f; mk[j] = 1.f; }
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = ih - (oh * sh - pt);
      if (r < 0 || r >= kh) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int q = iw - (ow * sw - pl);
        if (q < 0 || q >= kw) continue;
        const long long o = (((long long)nn * ho + oh) * wo + ow) * c + ch;
        int am[VN];
        if (argmax) {
          if constexpr (VN == 8) {
            const uint2 a = *(const uint2*)(argmax + o);
#pragma unroll
            for (int j = 0; j < 4; ++j) { am[j] = (a.x >> (8 * j)) & 255; am[j + 4] = (a.y >> (8 * j)) & 255; }
          } else {
#pragma unroll
            for (int j = 0; j < VN; ++j) am[j] = argmax[o + j];
          }
        } else {
          float m[VN];
#pragma unroll
          for (int j = 0; j < VN; ++j) { m[j] = -INFINITY; am[j] = 255; }
          for (int rr = 0; rr < kh; ++rr) {
            const int hh = oh * sh - pt + rr;
            if (hh < 0 || hh >= h) continue;
            for (int qq = 0; qq < kw; ++qq) {
              const int ww = ow * sw - pl + qq;
              if (ww < 0 || ww >= w) continue;
              Ld8<T, VN>::load(x + (((long long)nn * h + hh) * w + ww) * c + ch, v);
#pragma unroll
              for (int j = 0; j < VN; ++j)
                if (v[j] > m[j] || am[j] == 255) { m[j] = v[j]; am[j] = rr * kw + qq; }
            }
          }
        }
        const int tap = r * kw + q;
        bool any = false;
#pragma unroll
        for (int j = 0; j < VN; ++j) any |= am[j] == tap;
        if (!any) continue;
        Ld8<T, VN>::load(dy + o, d);
#pragma unroll
        for (int j = 0; j < VN; ++j)
          if (am[j] == tap) g[j] += d[j];
      }
    }
    if (xact) {
      Ld8<T, VN>::load(xact + (((long long)nn * h + ih) * w + iw) * c + ch, v);
#pragma unroll
      for (int j = 0; j < VN; ++j) mk[j] = act_mask_from_y(v[j], act, alpha);
    }
#pragma unroll
    for (int j = 0; j < VN; ++j) g[j] *= mk[j];
    Ld8<T, VN>::store(dx + (((long long)nn * h + ih) * w + iw) * c + ch, g);
  }
}

// 3x3 stride-2 pools whose 2x2 input blocks tile the input (the ResNet stem's
// 'same' pool): thread per pooled window (oh, ow) x 8 channels owning the 2x2
// input block at the window's top-left; the only windows that can route into
// that block are (oh-1..oh) x (ow-1..ow), each read once (argmax 8 B, dy 16 B
// when a tap lands in the block) — the gather form reads a window once per
// input it covers, ~2.25x. Sums in the gather form's window order: same bits.
template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(int n, int h, int w, int c, int pt, int pl, int ho,
                                                             int wo, const uint8_t* __restrict__ argmax,
                                                             const T* __restrict__ dy, T* __restrict__ dx,
                                                             const T* __restrict__ xact, int act, float alpha) {
  const int cg = c / 8;
  const long long total = (long long)n * ho * wo * cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cg) * 8;
    long long t = i / cg;
    const int ow = (int)(t % wo);
    t /= wo;
    const int oh = (int)(t % ho);
    const int nn = (int)(t / ho);
    float g[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) g[q][j] = 0.f;
#pragma unroll
    for (int dy_ = -1; dy_ <= 0; ++dy_) {
#pragma unroll
      for (int dx_ = -1; dx_ <= 0; ++dx_) {
        const int wy = oh + dy_, wx = ow + dx_;
        if (wy < 0 || wx < 0) continue;
        const long long o = (((long long)nn * ho + wy) * wo + wx) * c + ch;
        const uint2 a = *(const uint2*)(argmax + o);
        int slot[8];
        bool any = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int am = (int)(((j < 4 ? a.x : a.y) >> (8 * (j & 3))) & 255);
          const int r = am / 3, q = am - 3 * r;  // tap (r, q); 255 -> r = 85: outside
          const int dr = 2 * dy_ + r, dc = 2 * dx_ + q;
          slot[j] = ((unsigned)dr < 2u && (unsigned)dc < 2u) ? dr * 2 + dc : -1;
          any |= slot[j] >= 0;
        }
        if (!any) continue;
        float d[8];
        Ld8<T, 8>::load(dy + o, d);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (slot[j] == q) g[q][j] += d[j];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ih = 2 * oh - pt + (q >> 1), iw = 2 * ow - pl + (q & 1);
      if (ih < 0 || ih >= h || iw < 0 || iw >= w) continue;
      T* dst = dx + (((long long)nn * h + ih) * w + iw) * c + ch;
      if (xact) {
        float v[8];
        Ld8<T, 8>::load(xact + (dst - dx), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[q][j] *= act_mask_from_y(v[j], act, alpha);
      }
      Ld8<T, 8>::store(dst, g[q]);
    }
  }
}

template <typename T>
static void maxpool_launch(bool fwd, int n, int h, int w, int c, int kh, int kw, int sh, int sw, int pt, int pl,
                           int ho, int wo, const void* x, void* y, uint8_t* am, const void* dy, void* dx,
                           hipStream_t s, const void* xact = nullptr, int act = 0, float alpha = 0.f) {
  const bool vec = c % 8 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)(fwd ? y : dy) % 16 == 0 &&
                   (uintptr_t)(fwd ? y : dx) % 16 == 0 && (uintptr_t)am % 8 == 0 && (uintptr_t)xact % 16 == 0;
  const long long total = (long long)n * (fwd ? (long long)ho * wo : (long long)h * w) * (vec ? c / 8 : c);
  const int g = grid_for(total, 256, 8192);
  if (fwd) {
    if (vec)
      hipLaunchKernelGGL((maxpool_fwd_kernel<T, 8>), dim3(g), dim3(256), 0, s, n, h, w, c, kh, kw, sh, sw, pt, pl,
                         ho, wo, (const T*)x, (T*)y, am);
    else
      hipLaunchKernelGGL((maxpool_fwd_kernel<T, 1>), dim3(g), dim3(256), 0, s, n, h, w, c, kh, kw, sh, sw, pt, pl,
                         ho, wo, (const T*)x, (T*)y, am);
  } else if (vec && am && kh == 3 && kw == 3 && sh == 2 && sw == 2 && (unsigned)pt < 2u && (unsigned)pl < 2u &&
             2 * ho - pt >= h && 2 * wo - pl >= w) {
    const int g2 = grid_for((long long)n * ho * wo * (c / 8), 256, 8192);
    hipLaunchKernelGGL((maxpool3s2_bwd_kernel<T>), dim3(g2), dim3(256), 0, s, n, h, w, c, pt, pl, ho, wo,
                       (const uint8_t*)am, (const T*)dy, (T*)dx, (const T*)xact, act, alpha);
  } else {
    if (vec)
      hipLaunchKernelGGL((maxpool_bwd_kernel<T, 8>), dim3(g), dim3(256), 0, s, n, h, w, c, kh, kw, sh, sw, pt, pl,
                         ho, wo, (const T*)x, (const uint8_t*)am, (const T*)dy, (T*)dx, (const T*)xact, act, alpha);
    else
      hipLaunchKernelGGL((maxpool_bwd_kernel<T, 1>), dim3(g), dim3(256), 0, s, n, h, w, c, kh, kw, sh, sw, pt, pl,
                         ho, wo, (const T*)x, (const uint8_t*)am, (const T*)dy, (T*)dx, (const T*)xact, act, alpha);
  }
}

// ------------------------------------------------------------------------
// TF2 nearest resize (half_pixel_centers): src = min(floor((d+0.5)*in/out), in-1)
__device__ __forceinline__ int nn_src(int d, int in, int out) {
  int s = (int)floorf(((float)d + 0.5f) * ((float)in / (float)out));
  return s < in - 1 ? s : in - 1;
}

// FPN top-down fwd: part 1 (P3 grid) writes p3m, part 2 (P4 grid) writes p4m.
template <typename T>
__global__ void fpn_fwd_kernel(int n, int cg, int h5, int w5, int h4, int w4, int h3, int w3,
                               const T* __restrict__ l5, const T* __restrict__ l4,
                               const T* __restrict__ l3, T* __restrict__ p4m,
                               T* __restrict__ p3m) {
  typedef typename V16<T>::type VT;
  constexpr int VN = V16<T>::n;
  const int c = cg * VN;
  const long long tot3 = (long long)n * h3 * w3 * cg, tot4 = (long long)n * h4 * w4 * cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < tot3 + tot4;
       i += (long long)gridDim.x * blockDim.x) {
    const bool is3 = i < tot3;
    long long j = is3 ? i : i - tot3;
    const int g = (int)(j % cg);
    long long t = j / cg;
    const int W = is3 ? w3 : w4, H = is3 ? h3 : h4;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const int b = (int)(t / H);
    const int y4 = is3 ? nn_src(y, h4, h3) : y, x4 = is3 ? nn_src(x, w4, w3) : x;
    const int y5 = nn_src(y4, h5, h4), x5 = nn_src(x4, w5, w4);
    VT a4 = *(const VT*)(l4 + (((long long)b * h4 + y4) * w4 + x4) * c + g * VN);
    VT a5 = *(const VT*)(l5 + (((long long)b * h5 + y5) * w5 + x5) * c + g * VN);
    VT o;
    if (is3) {
      VT a3 = *(const VT*)(l3 + (((long long)b * h3 + y) * w3 + x) * c + g * VN);
#pragma unroll
      for (int k = 0; k < VN; ++k) {
        // P4m rounded to the activation dtype first, as the reference materialises it
        const float p4 = to_f32(from_f32<T>(to_f32(a4[k]) + to_f32(a5[k])));
        o[k] = from_f32<T>(to_f32(a3[k]) + p4);
      }
      *(VT*)(p3m + (((long long)b * h3 + y) * w3 + x) * c + g * VN) = o;
    } else {
#pragma unroll
      for (int k = 0; k < VN; ++k) o[k] = from_f32<T>(to_f32(a4[k]) + to_f32(a5[k]));
      *(VT*)(p4m + (((long long)b * h4 + y) * w4 + x) * c + g * VN) = o;
    }
  }
}

// children range of source pixel s under nearest resize in->out: [lo, hi)
__device__ __forceinline__ void nn_children(int s, int in, int out, int& lo, int& hi) {
  int d0 = (int)(((long long)s * out) / in) - 2;
  if (d0 < 0) d0 = 0;
  lo = -1;
  hi = -1;
  for (int d = d0; d < out; ++d) {
    const int src = nn_src(d, in, out);
    if (src == s && lo < 0) lo = d;
    if (src > s) { hi = d; break; }
  }
  if (lo < 0) { lo = 0; hi = 0; return; }
  if (hi < 0) hi = out;
}

// FPN top-down bwd: part 1 (P4 grid) d_lat4 = d_p4m + down(d_p3m);
// part 2 (P5 grid) d_lat5 (+)= down(d_p4m + down(d_p3m)).
template <typename T>
__global__ void fpn_bwd_kernel(int n, int cg, int h5, int w5, int h4, int w4, int h3, int w3,
                               const T* __restrict__ dp4, const T* __restrict__ dp3,
                               T* __restrict__ dl4, T* __restrict__ dl5, int acc5) {
  typedef typename V16<T>::type VT;
  constexpr int VN = V16<T>::n;
  const int c = cg * VN;
  const long long tot4 = (long long)n * h4 * w4 * cg, tot5 = (long long)n * h5 * w5 * cg;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < tot4 + tot5;
       i += (long long)gridDim.x * blockDim.x) {
    const bool is4 = i < tot4;
    long long j = is4 ? i : i - tot4;
    const int g = (int)(j % cg);
    long long t = j / cg;
    const int W = is4 ? w4 : w5, H = is4 ? h4 : h5;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const int b = (int)(t / H);
    float acc[VN];
#pragma unroll
    for (int k = 0; k < VN; ++k) acc[k] = 0.f;
    int y4lo, y4hi, x4lo, x4hi;
    if (is4) { y4lo = y; y4hi = y + 1; x4lo = x; x4hi = x + 1; }
    else { nn_children(y, h5, h4, y4lo, y4hi); nn_children(x, w5, w4, x4lo, x4hi); }
    for (int yy = y4lo; yy < y4hi; ++yy)
      for (int xx = x4lo; xx < x4hi; ++xx) {
        VT d4 = *(const VT*)(dp4 + (((long long)b * h4 + yy) * w4 + xx) * c + g * VN);
        float s4[VN];
#pragma unroll
        for (int k = 0; k < VN; ++k) s4[k] = to_f32(d4[k]);
        int y3lo, y3hi, x3lo, x3hi;
        nn_children(yy, h4, h3, y3lo, y3hi);
        nn_children(xx, w4, w3, x3lo, x3hi);
        for (int y3 = y3lo; y3 < y3hi; ++y3)
          for (int x3 = x3lo; x3 < x3hi; ++x3) {
            VT d3 = *(const VT*)(dp3 + (((long long)b * h3 + y3) * w3 + x3) * c + g * VN);
#pragma unroll
            for (int k = 0; k < VN; ++k) s4[k] += to_f32(d3[k]);
          }
        if (is4) {
#pragma unroll
          for (int k = 0; k < VN; ++k) acc[k] = s4[k];
        } else {
#pragma unroll
          for (int k = 0; k < VN; ++k) acc[k] += to_f32(from_f32<T>(s4[k]));
        }
      }
    VT o;
    if (is4) {
#pragma unroll
      for (int k = 0; k < VN; ++k) o[k] = from_f32<T>(acc[k]);
      *(VT*)(dl4 + (((long long)b * h4 + y) * w4 + x) * c + g * VN) = o;
    } else {
      T* dst = dl5 + (((long long)b * h5 + y) * w5 + x) * c + g * VN;
      if (acc5) {
        VT old = *(const VT*)dst;
#pragma unroll
        for (int k = 0; k < VN; ++k) o[k] = from_f32<T>(acc[k] + to_f32(old[k]));
      } else {
#pragma unroll
        for (int k = 0; k < VN; ++k) o[k] = from_f32<T>(acc[k]);
      }
      *(VT*)dst = o;
    }
  }
}

// ------------------------------------------------------------------------
// co-attention spatial softmax fwd: grid (n, chunks); each block recomputes the
// image's max / sum over hw (score is n x hw, tiny), then scales its chunk.
template <typename T>
__global__ __launch_bounds__(256) void ssm_fwd_kernel(int hw, int c, int chunk,
                                                      const T* __restrict__ score,
                                                      const T* __restrict__ hs,
                                                      T* __restrict__ ctx, float* __restrict__ a_out) {
  __shared__ float red[8];
  const int b = blockIdx.x;
  const T* sc = score + (long long)b * hw;
  float m = -INFINITY;
  for (int p = threadIdx.x; p < hw; p += 256) m = fmaxf(m, to_f32(sc[p]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int p = threadIdx.x; p < hw; p += 256) s += expf(to_f32(sc[p]) - m);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  const int p0 = blockIdx.y * chunk, p1 = min(hw, p0 + chunk);
  for (int p = p0 + threadIdx.x; p < p1; p += 256)
    a_out[(long long)b * hw + p] = expf(to_f32(sc[p]) - m) / s;
  // ctx = a * hs over (p, c) in this chunk
  const long long e0 = (long long)p0 * c, e1 = (long long)p1 * c;
  const T* h = hs + (long long)b * hw * c;
  T* o = ctx + (long long)b * hw * c;
  for (long long e = e0 + threadIdx.x; e < e1; e += 256) {
    const int p = (int)(e / c);
    const float a = expf(to_f32(sc[p]) - m) / s;
    o[e] = from_f32<T>(a * to_f32(h[e]));
  }
}

// bwd part 1: d_hs = a * d_ctx; da[p] = sum_c d_ctx*hs   (wave per position).
// The regression branch reaches the loss only through this shift-invariant
// softmax (d_score = a (da - sum a da) cancels), so da and its weighted sum
// are accumulated and kept in fp64 (products of two fp32 values are exact in
// fp64); the kernel is HBM-bound and the fp64 adds are free.
template <typename T>
__global__ __launch_bounds__(256) void ssm_bwd1_kernel(long long npos, int c, const float* __restrict__ a,
                                                       const T* __restrict__ hs,
                                                       const T* __restrict__ dctx, T* __restrict__ dhs,
                                                       double* __restrict__ da) {
  const long long wid = (blockIdx.x * 256LL + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  for (long long p = wid; p < npos; p += (long long)gridDim.x * 4) {
    const float ap = a[p];
    double dot = 0.0;
    for (int ch = lane; ch < c; ch += 64) {
      const long long e = p * c + ch;
      const float g = to_f32(dctx[e]);
      dot += (double)g * (double)to_f32(hs[e]);
      dhs[e] = from_f32<T>(ap * g);
    }
    dot = wave_sum(dot);
    if (lane == 0) da[p] = dot;
  }
}
// bwd part 2: d_score[p] = a[p] * (da[p] - sum_q a[q] da[q])  (block per image)
template <typename T>
__global__ __launch_bounds__(256) void ssm_bwd2_kernel(int hw, const float* __restrict__ a,
                                                       const double* __restrict__ da,
                                                       T* __restrict__ dscore) {
  __shared__ double red[4];
  const long long base = (long long)blockIdx.x * hw;
  double s = 0.0;
  for (int p = threadIdx.x; p < hw; p += 256) s += (double)a[base + p] * da[base + p];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  for (int p = threadIdx.x; p < hw; p += 256)
    dscore[base + p] = from_f32<T>((float)((double)a[base + p] * (da[base + p] - s)));
}

// ------------------------------------------------------------------------
// LayerNorm: one wave per row; row cached in registers (d <= 64*MAXE)
constexpr int LN_MAXE = 16;  // d <= 1024
// VEC (bf16, d % 8 == 0, 16-B aligned rows): lane owns 8-column chunks
// lane + 64 i (16-B loads / stores); otherwise columns lane + 64 i
template <bool VEC>
__device__ __forceinline__ int ln_col(int lane, int k) {
  if constexpr (VEC) return (lane + 64 * (k >> 3)) * 8 + (k & 7);
  else return lane + 64 * k;
}

// Rows wid, wid + nw, ... of one LayerNorm (block blk of nblk); op > 0: the
// output is dropout(y) with the mask of fpnmt_dropout on the (rows, d) tensor
// (key, element r * d + col), applied to the stored dtype value.
template <typename T, bool VEC>
__device__ __forceinline__ void ln_fwd_rows(long long blk, long long nblk, long long rows, int d, float eps,
                                            const T* __restrict__ x, const T* __restrict__ res,
                                            const float* __restrict__ gamma, const float* __restrict__ beta,
                                            const float* __restrict__ pe, int pe_rows, T* __restrict__ y,
                                            float* __restrict__ mean_out, float* __restrict__ rstd_out, float op,
                                            unsigned long long okey) {
  const int lane = threadIdx.x & 63;
  const long long wid = (blk * 256LL + threadIdx.x) >> 6;
  const long long nw = nblk * 4;
  const float osc = op > 0.f ? 1.f / (1.f - op) : 1.f;
  // gamma / beta of this lane's columns in registers before the first row
  // (they were loaded after the two wave reductions, one more exposed
  // latency per row; round 6), the row's posenc with its x / res loads
  float gm[LN_MAXE], bt[LN_MAXE];
#pragma unroll
  for (int i = 0; i < LN_MAXE; ++i) {
    const int col = ln_col<VEC>(lane, i);
    gm[i] = col < d ? gamma[col] : 0.f;
    bt[i] = col < d ? beta[col] : 0.f;
  }
  for (long long r = wid; r < rows; r += nw) {
    float v[LN_MAXE], pv[LN_MAXE];
    float s = 0.f;
    {
      const long long prow = pe ? (r % pe_rows) : 0;
#pragma unroll
      for (int i = 0; i < LN_MAXE; ++i) {
        const int col = ln_col<VEC>(lane, i);
        pv[i] = pe && col < d ? pe[prow * d + col] : 0.f;
      }
    }
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < LN_MAXE / 8; ++i) {
        const int c0 = (lane + 64 * i) * 8;
        bf16x8 xv = {}, rv = {};
        if (c0 < d) {
          xv = *(const bf16x8*)(x + r * d + c0);
          if (res) rv = *(const bf16x8*)(res + r * d + c0);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t = 0.f;
          if (c0 < d) {
            t = to_f32(xv[e]);
            if (res) t = to_f32(from_f32<T>(t + to_f32(rv[e])));
          }
          v[i * 8 + e] = t;
          s += t;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LN_MAXE; ++i) {
        const int col = lane + 64 * i;
        v[i] = 0.f;
        if (col < d) {
          float t = to_f32(x[r * d + col]);
          if (res) t = to_f32(from_f32<T>(t + to_f32(res[r * d + col])));
          v[i] = t;
          s += t;
        }
      }
    }
    const float mu = wave_sum(s) / (float)d;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXE; ++i) {
      const int col = ln_col<VEC>(lane, i);
      if (col < d) { const float t = v[i] - mu; q += t * t; }
    }
    const float var = wave_sum(q) / (float)d;
    const float rs = rsqrtf(var + eps);
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < LN_MAXE / 8; ++i) {
        const int c0 = (lane + 64 * i) * 8;
        if (c0 < d) {
          bf16x8 ov;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float o = (v[i * 8 + e] - mu) * rs * gm[i * 8 + e] + bt[i * 8 + e];
            if (pe) o += pv[i * 8 + e];
            ov[e] = from_f32<T>(o);
            if (op > 0.f)
              ov[e] = from_f32<T>(uniform01(okey, (uint64_t)r * (uint64_t)d + (uint64_t)(c0 + e)) >= op
                                      ? to_f32(ov[e]) * osc : 0.f);
          }
          *(bf16x8*)(y + r * d + c0) = ov;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LN_MAXE; ++i) {
        const int col = lane + 64 * i;
        if (col < d) {
          float o = (v[i] - mu) * rs * gm[i] + bt[i];
          if (pe) o += pv[i];
          T ot = from_f32<T>(o);
          if (op > 0.f)
            ot = from_f32<T>(uniform01(okey, (uint64_t)r * (uint64_t)d + (uint64_t)col) >= op ? to_f32(ot) * osc
                                                                                                 : 0.f);
          y[r * d + col] = ot;
        }
      }
    }
    if (lane == 0) { mean_out[r] = mu; rstd_out[r] = rs; }
  }
}

template <typename T, bool VEC = false>
__global__ __launch_bounds__(256) void ln_fwd_kernel(long long rows, int d, float eps,
                                                     const T* __restrict__ x, const T* __restrict__ res,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     const float* __restrict__ pe, int pe_rows,
                                                     T* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out) {
  ln_fwd_rows<T, VEC>(blockIdx.x, gridDim.x, rows, d, eps, x, res, gamma, beta, pe, pe_rows, y, mean_out, rstd_out,
                      0.f, 0ull);
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma: one row per wave.
// part != nullptr: also the block's partial column sums of dy * xhat (dgamma)
// and dy (dbeta), part[block][0, d) / [d, 2d) — reduced in block order by
// act_colsum_kernel (deterministic; x / res / dy are read once for both).
// Block blk of nblk of one LayerNorm backward. dz: the producing Dense's
// dropout backward on the stored dx (act_bwd's arithmetic on the same bf16
// dx, bit for bit): dz = keep(row * d + col) ? dx / (1 - p) : 0. ip > 0: dy
// is first the backward of a dropout applied to the LayerNorm's OUTPUT
// (fpnmt_dropout's arithmetic, key ikey): dy' = keep ? dy / (1 - ip) : 0.
template <typename T, bool VEC>
__device__ __forceinline__ void ln_bwd_rows(long long blk, long long nblk, long long rows, int d,
                                            const T* __restrict__ x, const T* __restrict__ res,
                                            const float* __restrict__ gamma, const float* __restrict__ mean,
                                            const float* __restrict__ rstd, const T* __restrict__ dy,
                                            T* __restrict__ dx, float* __restrict__ part, float dp,
                                            unsigned long long dkey, T* __restrict__ dz, float ip,
                                            unsigned long long ikey) {
  const int lane = threadIdx.x & 63;
  const float dsc = dz ? 1.f / (1.f - dp) : 1.f;
  const float isc = ip > 0.f ? 1.f / (1.f - ip) : 1.f;
  const long long wid = (blk * 256LL + threadIdx.x) >> 6;
  const long long nw = nblk * 4;
  float pg[LN_MAXE], pb[LN_MAXE];
#pragma unroll
  for (int i = 0; i < LN_MAXE; ++i) pg[i] = pb[i] = 0.f;
  for (long long r = wid; r < rows; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    float xh[LN_MAXE], g[LN_MAXE];
    float s1 = 0.f, s2 = 0.f;
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < LN_MAXE / 8; ++i) {
        const int c0 = (lane + 64 * i) * 8;
        bf16x8 xv = {}, rv = {}, dv = {};
        if (c0 < d) {
          xv = *(const bf16x8*)(x + r * d + c0);
          if (res) rv = *(const bf16x8*)(res + r * d + c0);
          dv = *(const bf16x8*)(dy + r * d + c0);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = i * 8 + e;
          xh[k] = 0.f;
          g[k] = 0.f;
          if (c0 < d) {
            float t = to_f32(xv[e]);
            if (res) t = to_f32(from_f32<T>(t + to_f32(rv[e])));
            xh[k] = (t - mu) * rs;
            float dyf = to_f32(dv[e]);
            if (ip > 0.f)
              dyf = to_f32(from_f32<T>(uniform01(ikey, (uint64_t)r * (uint64_t)d + (uint64_t)(c0 + e)) >= ip
                                           ? dyf * isc : 0.f));
            g[k] = dyf * gamma[c0 + e];
            pg[k] += dyf * xh[k];
            pb[k] += dyf;
            s1 += g[k];
            s2 += g[k] * xh[k];
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LN_MAXE; ++i) {
        const int col = lane + 64 * i;
        xh[i] = 0.f;
        g[i] = 0.f;
        if (col < d) {
          float t = to_f32(x[r * d + col]);
          if (res) t = to_f32(from_f32<T>(t + to_f32(res[r * d + col])));
          xh[i] = (t - mu) * rs;
          float dyf = to_f32(dy[r * d + col]);
          if (ip > 0.f)
            dyf = to_f32(from_f32<T>(uniform01(ikey, (uint64_t)r * (uint64_t)d + (uint64_t)col) >= ip ? dyf * isc
                                                                                                       : 0.f));
          g[i] = dyf * gamma[col];
          pg[i] += dyf * xh[i];
          pb[i] += dyf;
          s1 += g[i];
          s2 += g[i] * xh[i];
        }
      }
    }
    s1 = wave_sum(s1) / (float)d;
    s2 = wave_sum(s2) / (float)d;
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < LN_MAXE / 8; ++i) {
        const int c0 = (lane + 64 * i) * 8;
        if (c0 < d) {
          bf16x8 ov;
#pragma unroll
          for (int e = 0; e < 8; ++e) ov[e] = from_f32<T>(rs * (g[i * 8 + e] - s1 - xh[i * 8 + e] * s2));
          *(bf16x8*)(dx + r * d + c0) = ov;
          if (dz) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float t = to_f32(ov[e]);
              ov[e] = from_f32<T>(uniform01(dkey, (uint64_t)r * (uint64_t)d + (uint64_t)(c0 + e)) >= dp ? t * dsc
                                                                                                         : 0.f);
            }
            *(bf16x8*)(dz + r * d + c0) = ov;
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LN_MAXE; ++i) {
        const int col = lane + 64 * i;
        if (col < d) {
          const T v = from_f32<T>(rs * (g[i] - s1 - xh[i] * s2));
          dx[r * d + col] = v;
          if (dz) {
            const float t = to_f32(v);
            dz[r * d + col] =
                from_f32<T>(uniform01(dkey, (uint64_t)r * (uint64_t)d + (uint64_t)col) >= dp ? t * dsc : 0.f);
          }
        }
      }
    }
  }
  if (part) {  // the block's 4 waves in wave order, through LDS
    __shared__ float red[4][2 * 64 * LN_MAXE];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < LN_MAXE; ++i) {
      const int col = ln_col<VEC>(lane, i);
      if (col < d) {
        red[w][col] = pg[i];
        red[w][d + col] = pb[i];
      }
    }
    __syncthreads();
    float* dst = part + blk * 2 * d;
    for (int e = threadIdx.x; e < 2 * d; e += 256) dst[e] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
  }
}

__device__ __forceinline__ unsigned long long drop_key_of(unsigned long long seed, const long long* seed_dev) {
  return seed + (seed_dev ? (unsigned long long)(*seed_dev) * 0x9E3779B97F4A7C15ull : 0ull);
}

template <typename T, bool VEC = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(long long rows, int d, const T* __restrict__ x,
                                                     const T* __restrict__ res,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const T* __restrict__ dy, T* __restrict__ dx,
                                                     float* __restrict__ part, float dp,
                                                     unsigned long long dseed,
                                                     const long long* __restrict__ dseed_dev,
                                                     T* __restrict__ dz) {
  ln_bwd_rows<T, VEC>(blockIdx.x, gridDim.x, rows, d, x, res, gamma, mean, rstd, dy, dx, part, dp,
                      dz ? drop_key_of(dseed, dseed_dev) : 0ull, dz, 0.f, 0ull);
}

// ---- the Encoder's five view LayerNorms (shared gamma / beta / posenc,
// transformer.py:279-292: LN, + pe[:L], dropout) as one launch per pass:
// each view keeps the block count and row striding of its own launch
// (blocks [blk0, blk0 + nblk) of the grid), so per-row results and the
// backward's per-block partials are those of separate launches.
struct LnView {
  const void* x;
  void* y;     // fwd: dropout(LN(x) + pe);  bwd: dx
  const void* dy;
  float* mean;
  float* rstd;
  float* part;  // bwd: this view's partial rows
  long long rows;
  unsigned long long seed;
  int blk0, nblk, pe_rows;
};
struct LnViews {
  LnView v[FPNMT_MAX_LN_VIEWS];
  int n;
};

__device__ __forceinline__ int ln_view_of(const LnViews& A, int b) {
  int k = 0;
#pragma unroll
  for (int i = 1; i < FPNMT_MAX_LN_VIEWS; ++i)
    if (i < A.n && b >= A.v[i].blk0) k = i;
  return k;
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ln_views_fwd_kernel(const LnViews A, int d, float eps,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ pe, float p,
                                                           const long long* __restrict__ seed_dev) {
  const LnView& a = A.v[ln_view_of(A, blockIdx.x)];
  ln_fwd_rows<T, VEC>(blockIdx.x - a.blk0, a.nblk, a.rows, d, eps, (const T*)a.x, nullptr, gamma, beta, pe, a.pe_rows,
                      (T*)a.y, a.mean, a.rstd, p, p > 0.f ? drop_key_of(a.seed, seed_dev) : 0ull);
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ln_views_bwd_kernel(const LnViews A, int d, const float* __restrict__ gamma,
                                                           float p, const long long* __restrict__ seed_dev) {
  const LnView& a = A.v[ln_view_of(A, blockIdx.x)];
  ln_bwd_rows<T, VEC>(blockIdx.x - a.blk0, a.nblk, a.rows, d, (const T*)a.x, nullptr, gamma, a.mean, a.rstd,
                      (const T*)a.dy, (T*)a.y, a.part, 0.f, 0ull, nullptr, p,
                      p > 0.f ? drop_key_of(a.seed, seed_dev) : 0ull);
}

// ------------------------------------------------------------------------
// embedding + positional encoding
template <typename T>
__global__ void embed_fwd_kernel(int b, int t, int d, const int32_t* __restrict__ tok,
                                 const float* __restrict__ emb, const float* __restrict__ pe,
                                 T* __restrict__ y, float p, unsigned long long seed,
                                 const long long* __restrict__ seed_dev) {
  const long long total = (long long)b * t * d;
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const unsigned long long key = p > 0.f ? drop_key_of(seed, seed_dev) : 0ull;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(i % d);
    const long long row = i / d;
    const int pos = (int)(row % t);
    const int id = tok[row];
    T v = from_f32<T>(emb[(long long)id * d + col] + pe[(long long)pos * d + col]);
    // the decoder's Dropout after the embedding (transformer.py:331): fpnmt_dropout's mask / arithmetic
    if (p > 0.f) v = from_f32<T>(uniform01(key, (uint64_t)i) >= p ? to_f32(v) * sc : 0.f);
    y[i] = v;
  }
}

// dy of a dropout output, as fpnmt_dropout's backward stores it (p 0: dy)
template <typename T>
__device__ __forceinline__ float drop_grad(T g, float p, float sc, unsigned long long key, long long i) {
  if (p <= 0.f) return to_f32(g);
  return to_f32(from_f32<T>(uniform01(key, (uint64_t)i) >= p ? to_f32(g) * sc : 0.f));
}
// Train-step targets (utils/pipeline.py:66-69, transformer.py:42-67) from
// the padded (b, t + 1) int64 captions in one pass: tar_inp = tok[:, :-1],
// tar_real = tok[:, 1:] as int32, and the decoder self-attention mask
// max(padding(tar_inp), look_ahead) = 1 where tar_inp[b, j] == 0 or j > i.
template <typename I>
__global__ void decoder_targets_kernel(int b, int t, const I* __restrict__ tok, long long ld,
                                       int32_t* __restrict__ tin, int32_t* __restrict__ tout,
                                       float* __restrict__ mask) {
  const long long total = (long long)b * t * t;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(e % t);
    const long long bi = e / t;
    const int i = (int)(bi % t);
    const int bb = (int)(bi / t);
    const long long tj = (long long)tok[(long long)bb * ld + j];
    mask[e] = (tj == 0 || j > i) ? 1.f : 0.f;
    if (i == 0) {
      tin[(long long)bb * t + j] = (int32_t)tj;
      tout[(long long)bb * t + j] = (int32_t)tok[(long long)bb * ld + j + 1];
    }
  }
}

// Embedding backward without atomics (deterministic), in two passes over
// chunks of 64 positions:
//  A (block per chunk): per column, rows of the chunk are added in position
//    order into an LDS row per LOCAL leader (first position of each id in
//    the chunk); the leaders' partial rows go to part[leader position].
//  B (wave per position): rowsq[p] = ||dy[p]||^2 (the IndexedSlices clip
//    norm counts one row per position); the GLOBAL first position of an id
//    adds that id's chunk partials, in chunk order, to its row of demb (the
//    row's only writer).
// Heavily repeated ids (the padding id fills ~40 % of a caption batch) thus
// cost one LDS add per position, not a serial walk over all their rows.
constexpr int EMB_CHUNK = 64, EMB_COLS = 512;
template <typename T>
__global__ __launch_bounds__(256) void embed_chunk_kernel(long long rows, int d, const int32_t* __restrict__ tok,
                                                          const T* __restrict__ dy, float* __restrict__ part,
                                                          float p, unsigned long long seed,
                                                          const long long* __restrict__ seed_dev) {
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const unsigned long long key = p > 0.f ? drop_key_of(seed, seed_dev) : 0ull;
  __shared__ int s_tok[EMB_CHUNK], s_lead[EMB_CHUNK];
  __shared__ float acc[EMB_CHUNK][EMB_COLS];
  const int tid = threadIdx.x;
  const long long p0 = (long long)blockIdx.x * EMB_CHUNK;
  const int n = (int)min((long long)EMB_CHUNK, rows - p0);
  if (tid < EMB_CHUNK) s_tok[tid] = tid < n ? tok[p0 + tid] : -1;
  __syncthreads();
  if (tid < n) {
    int l = tid;
    for (int j = 0; j < tid; ++j)
      if (s_tok[j] == s_tok[tid]) { l = j; break; }
    s_lead[tid] = l;
  }
  __syncthreads();
  for (int c0 = 0; c0 < d; c0 += EMB_COLS) {
    const int w = min(EMB_COLS, d - c0);
    for (int e = tid; e < EMB_CHUNK * EMB_COLS; e += 256) (&acc[0][0])[e] = 0.f;
    __syncthreads();
    for (int col = tid; col < w; col += 256) {
#pragma unroll 8
      for (int i = 0; i < n; ++i)
        acc[s_lead[i]][col] += drop_grad(dy[(p0 + i) * d + c0 + col], p, sc, key, (p0 + i) * d + c0 + col);
    }
    __syncthreads();
    for (int i = 0; i < n; ++i) {
      if (s_lead[i] != i) continue;
      for (int col = tid; col < w; col += 256) part[(p0 + i) * d + c0 + col] = acc[i][col];
    }
    __syncthreads();
  }
}

// tokens staged in LDS (dynamic, rows * 4 B) when they fit, else read from HBM
template <typename T>
__global__ __launch_bounds__(64) void embed_leader_kernel(long long rows, int d, const int32_t* __restrict__ tok,
                                                          const T* __restrict__ dy, const float* __restrict__ part,
                                                          float* __restrict__ demb, float* __restrict__ rowsq,
                                                          int tok_in_lds, float dp, unsigned long long seed,
                                                          const long long* __restrict__ seed_dev) {
  const float dsc = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  const unsigned long long key = dp > 0.f ? drop_key_of(seed, seed_dev) : 0ull;
  extern __shared__ int s_tok[];
  __shared__ int s_lead[EMB_CHUNK];
  const int lane = threadIdx.x;
  const long long p = blockIdx.x;
  if (tok_in_lds) {
    for (long long q = lane; q < rows; q += 64) s_tok[q] = tok[q];
    __syncthreads();
  }
  const int32_t* tk = tok_in_lds ? (const int32_t*)s_tok : tok;
  const int id = tk[p];
  float sq = 0.f;
  for (int col = lane; col < d; col += 64) {
    const float g = drop_grad(dy[p * d + col], dp, dsc, key, p * d + col);
    sq += g * g;
  }
  sq = wave_sum(sq);
  if (lane == 0 && rowsq) rowsq[p] = sq;
  bool seen = false;
  for (long long q = lane; q < p; q += 64) seen |= tk[q] == id;
  if (__any(seen)) return;
  const long long nch = (rows + EMB_CHUNK - 1) / EMB_CHUNK;
  for (int c0 = 0; c0 < d; c0 += 64 * 8) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = 0.f;
    for (long long cb = p / EMB_CHUNK; cb < nch; cb += EMB_CHUNK) {
      // local leaders of id in chunks cb .. cb+63: lane l checks chunk cb+l
      int nl = 0;
      for (int l = 0; l < EMB_CHUNK && cb + l < nch; ++l) {
        const long long q = (cb + l) * EMB_CHUNK + lane;
        const unsigned long long m = __ballot(q < rows && tk[q] == id);
        if (m) {
          if (lane == 0) s_lead[nl] = (int)((cb + l) * EMB_CHUNK + __ffsll((long long)m) - 1);
          ++nl;
        }
      }
      __syncthreads();
      // partial rows in chunk order, four in flight
      for (int i = 0; i < nl; i += 4) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int col = c0 + lane + 64 * j;
            v[u][j] = (i + u < nl && col < d) ? part[(long long)s_lead[i + u] * d + col] : 0.f;
          }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] += v[u][j];
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c0 + lane + 64 * j;
      if (col < d) demb[(long long)id * d + col] += a[j];
    }
  }
}

// out[0] (+)= sum_i v[i] in a fixed order (one block): the per-position
// norms of the embedding, the per-row CE losses
__global__ __launch_bounds__(256) void ordered_sum_kernel(long long n, const float* __restrict__ v, float scale,
                                                          float* __restrict__ out, int accumulate) {
  __shared__ float red[4];
  float s = 0.f;
  for (long long i = threadIdx.x; i < n; i += 256) s += v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
    out[0] = accumulate ? out[0] + t : t;
  }
}

// ------------------------------------------------------------------------
// masked sparse CE: block per row
template <typename T>
__global__ __launch_bounds__(256) void xent_kernel(long long rows, int v, const float* __restrict__ logits,
                                                   long long ld, const int32_t* __restrict__ labels,
                                                   float* __restrict__ loss, T* __restrict__ dlog,
                                                   long long ldd, float gscale) {
  __shared__ float red[4];
  const long long r = blockIdx.x;
  const float* x = logits + r * ld;
  float m = -INFINITY;
  for (int j = threadIdx.x; j < v; j += 256) m = fmaxf(m, x[j]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int j = threadIdx.x; j < v; j += 256) s += expf(x[j] - m);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  const int lab = labels[r];
  const float mask = lab != 0 ? 1.f : 0.f;
  if (threadIdx.x == 0) loss[r] = mask != 0.f ? (m + logf(s)) - x[lab] : 0.f;  // per-row CE (summed in order)
  if (dlog) {
    const float coef = mask * gscale / (float)rows;
    T* dr = dlog + r * ldd;
    for (int j = threadIdx.x; j < v; j += 256) {
      float p = expf(x[j] - m) / s;
      if (j == lab) p -= 1.f;
      dr[j] = from_f32<T>(p * coef);
    }
  }
}

}  // namespace fpnmt

using namespace fpnmt;

#define DT_DISPATCH(dtype, FN, ...)                                         \
  ((dtype) == FPNMT_BF16 ? FN<bf16>(__VA_ARGS__)                            \
   : (dtype) == FPNMT_F32 ? FN<float>(__VA_ARGS__)                          \
                          : fail(FPNMT_E_ARG, "unknown dtype"))

extern "C" {

long long fpnmt_act_bwd_ws_bytes(int dtype, long long rows, int c) {
  if (rows <= 0 || c <= 0) return 0;
  // worst case over alignment (the unvectorised grid has the most chunks)
  const ActBwdGrid a = dtype == FPNMT_BF16 ? act_bwd_grid<bf16>(rows, c, true, true)
                                           : act_bwd_grid<float>(rows, c, true, true);
  const ActBwdGrid b = dtype == FPNMT_BF16 ? act_bwd_grid<bf16>(rows, c, false, true)
                                           : act_bwd_grid<float>(rows, c, false, true);
  return (long long)std::max(a.gy, b.gy) * c * (long long)sizeof(float);
}

int fpnmt_act_bwd(int dtype, long long rows, int c, int act, float act_alpha, const void* dy,
                  const void* y, void* dz, float* db, float* ws, float drop_p, unsigned long long drop_seed,
                  const long long* drop_seed_dev, fpnmt_stream_t stream) {
  if (rows <= 0 || c <= 0) return 0;
  if (!dy || !dz || (act != FPNMT_ACT_NONE && !y)) return fail(FPNMT_E_ARG, "act_bwd: null pointer");
  if (drop_p >= 1.f) return fail(FPNMT_E_ARG, "act_bwd: drop_p must be < 1");
  return DT_DISPATCH(dtype, act_bwd_t, rows, c, act, act_alpha, dy, y, dz, db, ws, drop_p, drop_seed,
                     drop_seed_dev, S(stream));
}

int fpnmt_bias_grad(int dtype, long long rows, int c, const void* dy, float* db, fpnmt_stream_t stream) {
  if (rows <= 0 || c <= 0 || !db) return 0;
  if (!dy) return fail(FPNMT_E_ARG, "bias_grad: null pointer");
  if (dtype != FPNMT_BF16 && dtype != FPNMT_F32) return fail(FPNMT_E_ARG, "bias_grad: bad dtype");
  hipStream_t s = S(stream);
  if (!defer_active())
    return dtype == FPNMT_BF16
               ? act_bwd_t<bf16>(rows, c, FPNMT_ACT_NONE, 0.f, dy, nullptr, (void*)dy, db, nullptr, 0.f, 0ull, nullptr, s)
               : act_bwd_t<float>(rows, c, FPNMT_ACT_NONE, 0.f, dy, nullptr, (void*)dy, db, nullptr, 0.f, 0ull, nullptr, s);
  const bool aligned = ((uintptr_t)dy % 16) == 0;
  const ActBwdGrid G = dtype == FPNMT_BF16 ? act_bwd_grid<bf16>(rows, c, aligned, true)
                                           : act_bwd_grid<float>(rows, c, aligned, true);
  DefDirect J{};
  J.dy = dy;
  J.db = db;
  J.rows = rows;
  J.c = c;
  J.rpc = G.rpc;
  J.gt = G.gt;
  J.gx = G.gx;
  J.gy = G.gy;
  J.vec = G.vec ? 1 : 0;
  J.dtype = dtype;
  {
    // partials + a queued colsum even for one chunk (the colsum of one chunk
    // adds exactly the block's sum, as the direct add would): consecutive
    // sums into one db (a shared conv's levels) then extend one colsum job
    // instead of flushing the queue at each level
    J.ws = defer_alloc((long long)G.gy * c);
    if (!J.ws)  // deferred arena full: the immediate launches
      return dtype == FPNMT_BF16 ? act_bwd_t<bf16>(rows, c, FPNMT_ACT_NONE, 0.f, dy, nullptr, (void*)dy, db, nullptr,
                                                   0.f, 0ull, nullptr, s)
                                 : act_bwd_t<float>(rows, c, FPNMT_ACT_NONE, 0.f, dy, nullptr, (void*)dy, db, nullptr,
                                                    0.f, 0ull, nullptr, s);
  }
  int st = defer_direct(J, s);
  if (!st) colsum_launch(G.gy, c, J.ws, db, s);  // queued behind the partials
  return st;
}

int fpnmt_cast(int in_dtype, int out_dtype, long long n, const void* in, void* out,
               fpnmt_stream_t stream) {
  if (n <= 0) return 0;
  const int g = grid_for(n, 256);
  hipStream_t s = S(stream);
  if (in_dtype == FPNMT_F32 && out_dtype == FPNMT_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(g), dim3(256), 0, s, n, (const float*)in, (bf16*)out);
  else if (in_dtype == FPNMT_BF16 && out_dtype == FPNMT_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(g), dim3(256), 0, s, n, (const bf16*)in, (float*)out);
  else if (in_dtype == FPNMT_F32 && out_dtype == FPNMT_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(g), dim3(256), 0, s, n, (const float*)in, (float*)out);
  else if (in_dtype == FPNMT_BF16 && out_dtype == FPNMT_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(g), dim3(256), 0, s, n, (const bf16*)in, (bf16*)out);
  else
    return fail(FPNMT_E_ARG, "cast: bad dtype");
  return check_launch("cast");
}

int fpnmt_dropout(int dtype, long long n, float p, unsigned long long seed, const long long* seed_dev,
                  const void* x, void* y, fpnmt_stream_t stream) {
  if (n <= 0) return 0;
  if (!(p >= 0.f && p < 1.f)) return fail(FPNMT_E_ARG, "dropout: p must be in [0,1)");
  const int g = grid_for(n, 256);
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((dropout_kernel<bf16>), dim3(g), dim3(256), 0, S(stream), n, p, seed, seed_dev,
                       (const bf16*)x, (bf16*)y);
  else
    hipLaunchKernelGGL((dropout_kernel<float>), dim3(g), dim3(256), 0, S(stream), n, p, seed, seed_dev,
                       (const float*)x, (float*)y);
  return check_launch("dropout");
}

int fpnmt_add(int dtype, long long n, const void* a, const void* b, void* out, fpnmt_stream_t stream) {
  if (n <= 0) return 0;
  const int g = grid_for(n, 256);
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((add_kernel<bf16>), dim3(g), dim3(256), 0, S(stream), n, (const bf16*)a,
                       (const bf16*)b, (bf16*)out);
  else
    hipLaunchKernelGGL((add_kernel<float>), dim3(g), dim3(256), 0, S(stream), n, (const float*)a,
                       (const float*)b, (float*)out);
  return check_launch("add");
}

int fpnmt_maxpool2d_fwd(int dtype, int n, int h, int w, int c, int kh, int kw, int sh, int sw, int pt,
                        int pl, int ho, int wo, const void* x, void* y, uint8_t* argmax, fpnmt_stream_t stream) {
  const long long total = (long long)n * ho * wo * c;
  if (total <= 0) return 0;
  if (argmax && kh * kw > 255) return fail(FPNMT_E_UNSUPPORTED, "maxpool: argmax needs kh*kw <= 255");
  if (dtype == FPNMT_BF16)
    maxpool_launch<bf16>(true, n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo, x, y, argmax, nullptr, nullptr, S(stream));
  else
    maxpool_launch<float>(true, n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo, x, y, argmax, nullptr, nullptr, S(stream));
  return check_launch("maxpool_fwd");
}

int fpnmt_maxpool2d_bwd(int dtype, int n, int h, int w, int c, int kh, int kw, int sh, int sw, int pt,
                        int pl, int ho, int wo, const void* x, const uint8_t* argmax, const void* dy, void* dx,
                        fpnmt_stream_t stream) {
  const long long total = (long long)n * h * w * c;
  if (total <= 0) return 0;
  if (ho <= 0 || wo <= 0) return zero_fill(dx, total * (dtype == FPNMT_BF16 ? 2 : 4), S(stream));
  if (!argmax && !x) return fail(FPNMT_E_ARG, "maxpool_bwd: need x or argmax");
  if (dtype == FPNMT_BF16)
    maxpool_launch<bf16>(false, n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo, x, nullptr, (uint8_t*)argmax, dy, dx, S(stream));
  else
    maxpool_launch<float>(false, n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo, x, nullptr, (uint8_t*)argmax, dy, dx, S(stream));
  return check_launch("maxpool_bwd");
}

int fpnmt_maxpool2d_bwd_act(int dtype, int n, int h, int w, int c, int kh, int kw, int sh, int sw, int pt, int pl,
                            int ho, int wo, const uint8_t* argmax, const void* dy, const void* x, int act,
                            float alpha, void* dx, fpnmt_stream_t stream) {
  const long long total = (long long)n * h * w * c;
  if (total <= 0) return 0;
  if (ho <= 0 || wo <= 0) return zero_fill(dx, total * (dtype == FPNMT_BF16 ? 2 : 4), S(stream));
  if (!argmax || !x || !dy || !dx) return fail(FPNMT_E_ARG, "maxpool_bwd_act: null argmax / x / dy / dx");
  if (act != FPNMT_ACT_RELU && act != FPNMT_ACT_RELU6 && act != FPNMT_ACT_LEAKY)
    return fail(FPNMT_E_ARG, "maxpool_bwd_act: act must be relu / relu6 / leaky");
  // a leaky factor after a sum of several windows' dy would round twice
  if (act == FPNMT_ACT_LEAKY && (kh > sh || kw > sw))
    return fail(FPNMT_E_UNSUPPORTED, "maxpool_bwd_act: leaky needs non-overlapping windows");
  if (dtype == FPNMT_BF16)
    maxpool_launch<bf16>(false, n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo, nullptr, nullptr, (uint8_t*)argmax, dy,
                         dx, S(stream), x, act, alpha);
  else
    maxpool_launch<float>(false, n, h, w, c, kh, kw, sh, sw, pt, pl, ho, wo, nullptr, nullptr, (uint8_t*)argmax, dy,
                          dx, S(stream), x, act, alpha);
  return check_launch("maxpool_bwd_act");
}

int fpnmt_fpn_topdown_fwd(int dtype, int n, int c, int h5, int w5, int h4, int w4, int h3, int w3,
                          const void* lat5, const void* lat4, const void* lat3, void* p4m, void* p3m,
                          fpnmt_stream_t stream) {
  const int vn = dtype == FPNMT_BF16 ? 8 : 4;
  if (c % vn) return fail(FPNMT_E_UNSUPPORTED, "fpn_topdown: channels must be a multiple of 8 (bf16) / 4 (f32)");
  const long long total = (long long)n * (h3 * w3 + h4 * w4) * (c / vn);
  if (total <= 0) return 0;
  const int g = grid_for(total, 256);
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((fpn_fwd_kernel<bf16>), dim3(g), dim3(256), 0, S(stream), n, c / vn, h5, w5, h4, w4,
                       h3, w3, (const bf16*)lat5, (const bf16*)lat4, (const bf16*)lat3, (bf16*)p4m, (bf16*)p3m);
  else
    hipLaunchKernelGGL((fpn_fwd_kernel<float>), dim3(g), dim3(256), 0, S(stream), n, c / vn, h5, w5, h4, w4,
                       h3, w3, (const float*)lat5, (const float*)lat4, (const float*)lat3, (float*)p4m,
                       (float*)p3m);
  return check_launch("fpn_topdown_fwd");
}

int fpnmt_fpn_topdown_bwd(int dtype, int n, int c, int h5, int w5, int h4, int w4, int h3, int w3,
                          const void* d_p4m, const void* d_p3m, void* d_lat4, void* d_lat5,
                          int accumulate_lat5, fpnmt_stream_t stream) {
  const int vn = dtype == FPNMT_BF16 ? 8 : 4;
  if (c % vn) return fail(FPNMT_E_UNSUPPORTED, "fpn_topdown: channels must be a multiple of 8 (bf16) / 4 (f32)");
  const long long total = (long long)n * (h4 * w4 + h5 * w5) * (c / vn);
  if (total <= 0) return 0;
  const int g = grid_for(total, 256);
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((fpn_bwd_kernel<bf16>), dim3(g), dim3(256), 0, S(stream), n, c / vn, h5, w5, h4, w4,
                       h3, w3, (const bf16*)d_p4m, (const bf16*)d_p3m, (bf16*)d_lat4, (bf16*)d_lat5,
                       accumulate_lat5);
  else
    hipLaunchKernelGGL((fpn_bwd_kernel<float>), dim3(g), dim3(256), 0, S(stream), n, c / vn, h5, w5, h4, w4,
                       h3, w3, (const float*)d_p4m, (const float*)d_p3m, (float*)d_lat4, (float*)d_lat5,
                       accumulate_lat5);
  return check_launch("fpn_topdown_bwd");
}

int fpnmt_spatial_softmax_fwd(int dtype, int n, int hw, int c, const void* score, const void* hs,
                              void* ctx, float* a_out, fpnmt_stream_t stream) {
  if (n <= 0 || hw <= 0) return 0;
  int chunks = (int)((long long)hw * c / 8192);
  if (chunks < 1) chunks = 1;
  if (chunks > hw) chunks = hw;
  const int chunk = cdiv(hw, chunks);
  chunks = cdiv(hw, chunk);
  dim3 grid(n, chunks);
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((ssm_fwd_kernel<bf16>), grid, dim3(256), 0, S(stream), hw, c, chunk,
                       (const bf16*)score, (const bf16*)hs, (bf16*)ctx, a_out);
  else
    hipLaunchKernelGGL((ssm_fwd_kernel<float>), grid, dim3(256), 0, S(stream), hw, c, chunk,
                       (const float*)score, (const float*)hs, (float*)ctx, a_out);
  return check_launch("spatial_softmax_fwd");
}

int fpnmt_spatial_softmax_bwd(int dtype, int n, int hw, int c, const float* a, const void* hs,
                              const void* d_ctx, void* d_score, void* d_hs, double* ws,
                              fpnmt_stream_t stream) {
  if (n <= 0 || hw <= 0) return 0;
  const long long npos = (long long)n * hw;
  const int g = grid_for(npos, 4, 8192);
  if (dtype == FPNMT_BF16) {
    hipLaunchKernelGGL((ssm_bwd1_kernel<bf16>), dim3(g), dim3(256), 0, S(stream), npos, c, a,
                       (const bf16*)hs, (const bf16*)d_ctx, (bf16*)d_hs, ws);
    hipLaunchKernelGGL((ssm_bwd2_kernel<bf16>), dim3(n), dim3(256), 0, S(stream), hw, a, ws, (bf16*)d_score);
  } else {
    hipLaunchKernelGGL((ssm_bwd1_kernel<float>), dim3(g), dim3(256), 0, S(stream), npos, c, a,
                       (const float*)hs, (const float*)d_ctx, (float*)d_hs, ws);
    hipLaunchKernelGGL((ssm_bwd2_kernel<float>), dim3(n), dim3(256), 0, S(stream), hw, a, ws, (float*)d_score);
  }
  return check_launch("spatial_softmax_bwd");
}

static bool ln_vec(int d, std::initializer_list<const void*> ptrs) {
  if (d % 8) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p & 15) return false;
  return true;
}

int fpnmt_layernorm_fwd(int dtype, long long rows, int d, float eps, const void* x, const void* res,
                        const float* gamma, const float* beta, const float* pe, int pe_rows, void* y,
                        float* mean, float* rstd, fpnmt_stream_t stream) {
  if (rows <= 0) return 0;
  if (d > 64 * LN_MAXE) return fail(FPNMT_E_UNSUPPORTED, "layernorm: d > 1024");
  if (pe && pe_rows <= 0) return fail(FPNMT_E_ARG, "layernorm: pe_rows");
  const int g = grid_for(rows, 4, 8192);
  if (dtype == FPNMT_BF16) {
    if (ln_vec(d, {x, res, y}))
      hipLaunchKernelGGL((ln_fwd_kernel<bf16, true>), dim3(g), dim3(256), 0, S(stream), rows, d, eps, (const bf16*)x,
                       (const bf16*)res, gamma, beta, pe, pe_rows, (bf16*)y, mean, rstd);
    else
      hipLaunchKernelGGL((ln_fwd_kernel<bf16>), dim3(g), dim3(256), 0, S(stream), rows, d, eps, (const bf16*)x,
                       (const bf16*)res, gamma, beta, pe, pe_rows, (bf16*)y, mean, rstd);
  } else {
    hipLaunchKernelGGL((ln_fwd_kernel<float>), dim3(g), dim3(256), 0, S(stream), rows, d, eps, (const float*)x,
                       (const float*)res, gamma, beta, pe, pe_rows, (float*)y, mean, rstd);
  }
  return check_launch("layernorm_fwd");
}

static int layernorm_bwd_impl(int dtype, long long rows, int d, const void* x, const void* res, const float* gamma,
                              const float* mean, const float* rstd, const void* dy, void* dx, float* dgamma,
                              float* dbeta, float dp, unsigned long long dseed, const long long* dseed_dev, void* dz,
                              hipStream_t s) {
  if (rows <= 0) return 0;
  if (d > 64 * LN_MAXE) return fail(FPNMT_E_UNSUPPORTED, "layernorm: d > 1024");
  if (dz && !(dp > 0.f && dp < 1.f)) return fail(FPNMT_E_ARG, "layernorm_bwd_drop: drop_p outside (0, 1)");
  // one row per wave, at most 1024 blocks (bounds the partial-sum rows)
  const int g = grid_for(rows, 4, 1024);
  float* part = nullptr;
  if (dgamma || dbeta) {
    part = partial_f32((long long)g * 2 * d);
    if (!part) return fail(FPNMT_E_ARG, "layernorm_bwd: dgamma / dbeta need the fpnmt workspace");
  }
  if (dtype == FPNMT_BF16) {
    if (ln_vec(d, {x, res, dy, dx, dz}))
      hipLaunchKernelGGL((ln_bwd_kernel<bf16, true>), dim3(g), dim3(256), 0, s, rows, d, (const bf16*)x,
                         (const bf16*)res, gamma, mean, rstd, (const bf16*)dy, (bf16*)dx, part, dp, dseed, dseed_dev,
                         (bf16*)dz);
    else
      hipLaunchKernelGGL((ln_bwd_kernel<bf16>), dim3(g), dim3(256), 0, s, rows, d, (const bf16*)x,
                         (const bf16*)res, gamma, mean, rstd, (const bf16*)dy, (bf16*)dx, part, dp, dseed, dseed_dev,
                         (bf16*)dz);
  } else {
    hipLaunchKernelGGL((ln_bwd_kernel<float>), dim3(g), dim3(256), 0, s, rows, d, (const float*)x,
                       (const float*)res, gamma, mean, rstd, (const float*)dy, (float*)dx, part, dp, dseed, dseed_dev,
                       (float*)dz);
  }
  if (part) colsum_launch(g, 2 * d, part, dgamma, s, d, dbeta);
  return check_launch("layernorm_bwd");
}

int fpnmt_layernorm_bwd(int dtype, long long rows, int d, const void* x, const void* res,
                        const float* gamma, const float* mean, const float* rstd, const void* dy, void* dx,
                        float* dgamma, float* dbeta, fpnmt_stream_t stream) {
  return layernorm_bwd_impl(dtype, rows, d, x, res, gamma, mean, rstd, dy, dx, dgamma, dbeta, 0.f, 0ull, nullptr,
                            nullptr, S(stream));
}

int fpnmt_layernorm_bwd_drop(int dtype, long long rows, int d, const void* x, const void* res, const float* gamma,
                             const float* mean, const float* rstd, const void* dy, void* dx, float* dgamma,
                             float* dbeta, float drop_p, unsigned long long drop_seed,
                             const long long* drop_seed_dev, void* dz, fpnmt_stream_t stream) {
  if (!dz) return fail(FPNMT_E_ARG, "layernorm_bwd_drop: null dz");
  return layernorm_bwd_impl(dtype, rows, d, x, res, gamma, mean, rstd, dy, dx, dgamma, dbeta, drop_p, drop_seed,
                            drop_seed_dev, dz, S(stream));
}

static bool ln_views_vec(int n, int d, const fpnmt_ln_view* v, bool bwd) {
  for (int i = 0; i < n; ++i)
    if (!(bwd ? ln_vec(d, {v[i].x, v[i].dy, v[i].y}) : ln_vec(d, {v[i].x, v[i].y}))) return false;
  return true;
}

int fpnmt_layernorm_views_fwd(int dtype, int n, int d, float eps, const fpnmt_ln_view* views, const float* gamma,
                              const float* beta, const float* pe, float drop_p, const long long* seed_dev,
                              fpnmt_stream_t stream) {
  if (n < 0 || n > FPNMT_MAX_LN_VIEWS) return fail(FPNMT_E_ARG, "layernorm_views_fwd: 0 <= n <= FPNMT_MAX_LN_VIEWS");
  if (d > 64 * LN_MAXE) return fail(FPNMT_E_UNSUPPORTED, "layernorm: d > 1024");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return fail(FPNMT_E_ARG, "layernorm_views_fwd: drop_p outside [0, 1)");
  LnViews A{};
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    const fpnmt_ln_view& v = views[i];
    if (v.rows <= 0) continue;
    if (!v.x || !v.y || !v.mean || !v.rstd || (pe && v.pe_rows <= 0))
      return fail(FPNMT_E_ARG, "layernorm_views_fwd: null pointer / pe_rows");
    LnView& a = A.v[A.n++];
    a.x = v.x; a.y = v.y; a.mean = v.mean; a.rstd = v.rstd; a.rows = v.rows; a.seed = v.seed;
    a.pe_rows = pe ? v.pe_rows : 1;
    a.blk0 = blocks;
    a.nblk = grid_for(v.rows, 4, 8192);  // fpnmt_layernorm_fwd's grid for this view
    blocks += a.nblk;
  }
  if (!A.n) return 0;
  hipStream_t s = S(stream);
  if (dtype == FPNMT_BF16) {
    if (ln_views_vec(n, d, views, false))
      hipLaunchKernelGGL((ln_views_fwd_kernel<bf16, true>), dim3(blocks), dim3(256), 0, s, A, d, eps, gamma, beta, pe,
                         drop_p, seed_dev);
    else
      hipLaunchKernelGGL((ln_views_fwd_kernel<bf16, false>), dim3(blocks), dim3(256), 0, s, A, d, eps, gamma, beta,
                         pe, drop_p, seed_dev);
  } else {
    hipLaunchKernelGGL((ln_views_fwd_kernel<float, false>), dim3(blocks), dim3(256), 0, s, A, d, eps, gamma, beta, pe,
                       drop_p, seed_dev);
  }
  return check_launch("layernorm_views_fwd");
}

int fpnmt_layernorm_views_bwd(int dtype, int n, int d, const fpnmt_ln_view* views, const float* gamma, float drop_p,
                              const long long* seed_dev, float* dgamma, float* dbeta, fpnmt_stream_t stream) {
  if (n < 0 || n > FPNMT_MAX_LN_VIEWS) return fail(FPNMT_E_ARG, "layernorm_views_bwd: 0 <= n <= FPNMT_MAX_LN_VIEWS");
  if (d > 64 * LN_MAXE) return fail(FPNMT_E_UNSUPPORTED, "layernorm: d > 1024");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return fail(FPNMT_E_ARG, "layernorm_views_bwd: drop_p outside [0, 1)");
  LnViews A{};
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    const fpnmt_ln_view& v = views[i];
    if (v.rows <= 0) continue;
    if (!v.x || !v.y || !v.dy || !v.mean || !v.rstd) return fail(FPNMT_E_ARG, "layernorm_views_bwd: null pointer");
    LnView& a = A.v[A.n++];
    a.x = v.x; a.y = v.y; a.dy = v.dy; a.mean = v.mean; a.rstd = v.rstd; a.rows = v.rows; a.seed = v.seed;
    a.blk0 = blocks;
    a.nblk = grid_for(v.rows, 4, 1024);  // fpnmt_layernorm_bwd's grid for this view
    blocks += a.nblk;
    a.part = nullptr;
  }
  if (!A.n) return 0;
  if (dgamma || dbeta) {  // one partial row per block, the views' rows back to back
    float* part = partial_f32((long long)blocks * 2 * d);
    if (!part) return fail(FPNMT_E_ARG, "layernorm_views_bwd: dgamma / dbeta need the fpnmt workspace");
    for (int i = 0; i < A.n; ++i) A.v[i].part = part + (long long)A.v[i].blk0 * 2 * d;
  }
  hipStream_t s = S(stream);
  if (dtype == FPNMT_BF16) {
    if (ln_views_vec(n, d, views, true))
      hipLaunchKernelGGL((ln_views_bwd_kernel<bf16, true>), dim3(blocks), dim3(256), 0, s, A, d, gamma, drop_p,
                         seed_dev);
    else
      hipLaunchKernelGGL((ln_views_bwd_kernel<bf16, false>), dim3(blocks), dim3(256), 0, s, A, d, gamma, drop_p,
                         seed_dev);
  } else {
    hipLaunchKernelGGL((ln_views_bwd_kernel<float, false>), dim3(blocks), dim3(256), 0, s, A, d, gamma, drop_p,
                       seed_dev);
  }
  const int st = check_launch("layernorm_views_bwd");
  if (st) return st;
  // the views' gamma / beta sums in view order (as separate launches would)
  for (int i = 0; i < A.n; ++i)
    if (A.v[i].part) colsum_launch(A.v[i].nblk, 2 * d, A.v[i].part, dgamma, s, d, dbeta);
  return check_launch("layernorm_views_bwd colsum");
}

static int embed_fwd_impl(int dtype, int b, int t, int d, const int32_t* tok, const float* emb, const float* pe,
                          void* y, float p, unsigned long long seed, const long long* seed_dev, hipStream_t s) {
  const long long total = (long long)b * t * d;
  if (total <= 0) return 0;
  const int g = grid_for(total, 256);
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((embed_fwd_kernel<bf16>), dim3(g), dim3(256), 0, s, b, t, d, tok, emb, pe, (bf16*)y, p, seed,
                       seed_dev);
  else
    hipLaunchKernelGGL((embed_fwd_kernel<float>), dim3(g), dim3(256), 0, s, b, t, d, tok, emb, pe, (float*)y, p,
                       seed, seed_dev);
  return check_launch("embed_fwd");
}

static int embed_bwd_impl(int dtype, int b, int t, int d, const int32_t* tok, const void* dy, float* d_emb,
                          float* sumsq, float p, unsigned long long seed, const long long* seed_dev,
                          hipStream_t s) {
  const long long rows = (long long)b * t;
  if (rows <= 0) return 0;
  if (rows >= (1LL << 31)) return fail(FPNMT_E_UNSUPPORTED, "embed_bwd: too many positions");
  float* part = scratch_f32(rows * d + rows);
  if (!part) return fail(FPNMT_E_ARG, "embed_bwd: needs the fpnmt workspace");
  float* rowsq = sumsq ? part + rows * d : nullptr;
  const unsigned nch = (unsigned)((rows + EMB_CHUNK - 1) / EMB_CHUNK);
  const unsigned lds = rows <= 8192 ? (unsigned)(rows * 4) : 0u;  // tokens in LDS when they fit
  if (dtype == FPNMT_BF16) {
    hipLaunchKernelGGL((embed_chunk_kernel<bf16>), dim3(nch), dim3(256), 0, s, rows, d, tok, (const bf16*)dy, part,
                       p, seed, seed_dev);
    hipLaunchKernelGGL((embed_leader_kernel<bf16>), dim3((unsigned)rows), dim3(64), lds, s, rows, d, tok,
                       (const bf16*)dy, (const float*)part, d_emb, rowsq, lds > 0, p, seed, seed_dev);
  } else {
    hipLaunchKernelGGL((embed_chunk_kernel<float>), dim3(nch), dim3(256), 0, s, rows, d, tok, (const float*)dy, part,
                       p, seed, seed_dev);
    hipLaunchKernelGGL((embed_leader_kernel<float>), dim3((unsigned)rows), dim3(64), lds, s, rows, d, tok,
                       (const float*)dy, (const float*)part, d_emb, rowsq, lds > 0, p, seed, seed_dev);
  }
  if (sumsq) hipLaunchKernelGGL(ordered_sum_kernel, dim3(1), dim3(256), 0, s, rows, rowsq, 1.f, sumsq, 1);
  return check_launch("embed_bwd");
}

int fpnmt_embed_posenc_fwd(int dtype, int b, int t, int d, const int32_t* tok, const float* emb,
                           const float* pe, void* y, fpnmt_stream_t stream) {
  return embed_fwd_impl(dtype, b, t, d, tok, emb, pe, y, 0.f, 0ull, nullptr, S(stream));
}

int fpnmt_embed_posenc_bwd(int dtype, int b, int t, int d, const int32_t* tok, const void* dy, float* d_emb,
                           float* sumsq, fpnmt_stream_t stream) {
  return embed_bwd_impl(dtype, b, t, d, tok, dy, d_emb, sumsq, 0.f, 0ull, nullptr, S(stream));
}

int fpnmt_embed_posenc_fwd_drop(int dtype, int b, int t, int d, const int32_t* tok, const float* emb,
                                const float* pe, void* y, float drop_p, unsigned long long seed,
                                const long long* seed_dev, fpnmt_stream_t stream) {
  if (!(drop_p >= 0.f && drop_p < 1.f)) return fail(FPNMT_E_ARG, "embed_posenc_fwd_drop: drop_p outside [0, 1)");
  return embed_fwd_impl(dtype, b, t, d, tok, emb, pe, y, drop_p, seed, seed_dev, S(stream));
}

int fpnmt_embed_posenc_bwd_drop(int dtype, int b, int t, int d, const int32_t* tok, const void* dy, float* d_emb,
                                float* sumsq, float drop_p, unsigned long long seed, const long long* seed_dev,
                                fpnmt_stream_t stream) {
  if (!(drop_p >= 0.f && drop_p < 1.f)) return fail(FPNMT_E_ARG, "embed_posenc_bwd_drop: drop_p outside [0, 1)");
  return embed_bwd_impl(dtype, b, t, d, tok, dy, d_emb, sumsq, drop_p, seed, seed_dev, S(stream));
}
int fpnmt_decoder_targets(int b, int t_full, const void* tok, int tok_bytes, long long ld_tok, int32_t* tar_inp,
                          int32_t* tar_real, float* mask, fpnmt_stream_t stream) {
  const int t = t_full - 1;
  if (b <= 0 || t <= 0) return 0;
  if (!tok || !tar_inp || !tar_real || !mask || ld_tok < t_full || (tok_bytes != 4 && tok_bytes != 8))
    return fail(FPNMT_E_ARG, "decoder_targets: null pointer / ld_tok < t_full / tok_bytes not 4 or 8");
  const long long total = (long long)b * t * t;
  if (tok_bytes == 8)
    hipLaunchKernelGGL(decoder_targets_kernel<long long>, dim3(grid_for(total, 256)), dim3(256), 0, S(stream), b, t,
                       (const long long*)tok, ld_tok, tar_inp, tar_real, mask);
  else
    hipLaunchKernelGGL(decoder_targets_kernel<int32_t>, dim3(grid_for(total, 256)), dim3(256), 0, S(stream), b, t,
                       (const int32_t*)tok, ld_tok, tar_inp, tar_real, mask);
  return check_launch("decoder_targets");
}

int fpnmt_xent_fwd_bwd(int dtype, long long rows, int v, const float* logits, long long ld,
                       const int32_t* labels, float* loss, void* dlogits, long long ldd, float dloss_scale,
                       fpnmt_stream_t stream) {
  if (!loss || !logits || !labels) return fail(FPNMT_E_ARG, "xent: null pointer");
  if (rows <= 0) return zero_fill(loss, sizeof(float), S(stream));
  float* row_loss = scratch_f32(rows);
  if (!row_loss) return fail(FPNMT_E_ARG, "xent: needs the fpnmt workspace");
  if (dtype == FPNMT_BF16)
    hipLaunchKernelGGL((xent_kernel<bf16>), dim3((unsigned)rows), dim3(256), 0, S(stream), rows, v, logits, ld,
                       labels, row_loss, (bf16*)dlogits, ldd, dloss_scale);
  else
    hipLaunchKernelGGL((xent_kernel<float>), dim3((unsigned)rows), dim3(256), 0, S(stream), rows, v, logits, ld,
                       labels, row_loss, (float*)dlogits, ldd, dloss_scale);
  // mean over ALL rows (utils/pipeline.py:57), summed in row order
  hipLaunchKernelGGL(ordered_sum_kernel, dim3(1), dim3(256), 0, S(stream), rows, (const float*)row_loss,
                     1.f / (float)rows, loss, 0);
  return check_launch("xent");
}

}  // extern "C"
