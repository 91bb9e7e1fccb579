// Deferred ordered reductions (fpnmt_defer_begin / fpnmt_defer_flush).
//
// A training step's backward issues ~150 small reduction launches besides
// its GEMMs: the split-K weight-gradient reduces (wgrad_reduce_kernel: slabs
// -> the fp32 gradient arena) and the column sums of bias / LayerNorm
// gradients (act_colsum_kernel: per-chunk partials -> db). Each is a latency-
// bound 4-7 us launch whose result only the optimizer reads. Between
// fpnmt_defer_begin and fpnmt_defer_flush their inputs (slabs, partials) are
// bump-allocated in a caller-provided arena instead of the shared workspace,
// the reductions are queued, and the flush runs them as a few batched
// launches (one block per job item, jobs found through a prefix table in the
// kernel arguments). Every job keeps exactly the summation order of its
// immediate kernel, so the results are bitwise those of immediate mode; a job
// whose destination overlaps a queued one's starts a new batch (two jobs of
// one launch never add into the same element).
#include <vector>

#include "gemm_impl.h"

namespace fpnmt {

namespace {

struct DefWgrad {
  float* C;
  const float* ws;
  const float* col_scale;
  long long c_so, c_si, ldc;
  int M, N, S, batch, batch_inner, G;
  float alpha;
  int blk0;  // first block of this job in its launch
};
// A colsum job sums `nseg` segments of per-chunk partials (segment i: seg[i]
// chunks at ws + seg_off[i]) and adds each segment's sum into db / db2 in
// segment order: exactly the sequence of the segments' immediate act_colsum
// launches. A later job into the same destinations with nothing else queued
// into them since (the per-level bias gradients of a shared head conv)
// extends the last job instead of flushing the queue.
constexpr int CS_MAX_SEG = 6;
struct DefColsum {
  const float* ws;
  float* db;
  float* db2;
  int c, c_split, CB;
  int blk0;
  int nseg;
  int seg[CS_MAX_SEG];
  int seg_off[CS_MAX_SEG];  // floats from ws
};

constexpr int WG_PER_LAUNCH = 20;
constexpr int CS_PER_LAUNCH = 24;  // the batch stays within 4 KB of kernel arguments
struct WgradBatch {
  DefWgrad j[WG_PER_LAUNCH];
  int n;
};
struct ColsumBatch {
  DefColsum j[CS_PER_LAUNCH];
  int n;
};

struct Range {
  uintptr_t lo, hi;
};

struct Deferred {
  char* base = nullptr;
  long long bytes = 0, used = 0, peak = 0;
  bool active = false;
  // queued jobs in issue order; a barrier index starts a new launch
  std::vector<DefDirect> dir;
  std::vector<DefGemmJob> gj;  // deferred weight-gradient GEMMs (launch_gemm_jobs)
  std::vector<DefWgrad> wg;
  std::vector<DefColsum> cs;
  std::vector<Range> dst;  // destinations queued since the last flush
};
Deferred g_def;

bool overlaps(const Range& r) {
  for (const Range& q : g_def.dst)
    if (r.lo < q.hi && q.lo < r.hi) return true;
  return false;
}

// ---- batched kernels: block -> job by a static-index scan of the table ----
template <int NJ, typename J>
__device__ __forceinline__ int job_of(const J (&j)[NJ], int n, int b) {
  int k = 0;
#pragma unroll
  for (int i = 1; i < NJ; ++i)
    if (i < n && b >= j[i].blk0) k = i;
  return k;
}

// wgrad_reduce_kernel<G> with G a job field: the same item mapping, split
// loop and lane-ordered LDS combine (bitwise its results)
__global__ __launch_bounds__(256) void defer_wgrad_kernel(const WgradBatch B) {
  __shared__ f32x4 red[256];
  const int k = job_of<WG_PER_LAUNCH>(B.j, B.n, blockIdx.x);
  DefWgrad J = B.j[0];
#pragma unroll
  for (int i = 1; i < WG_PER_LAUNCH; ++i)
    if (i == k) J = B.j[i];
  const int G = J.G, IT = 256 / G;
  const int c4 = (J.N + 3) / 4;
  const long long items = (long long)J.M * c4;
  const long long nbx = (items + IT - 1) / IT;
  const long long local = blockIdx.x - J.blk0;
  const int z = (int)(local / nbx);
  const long long bx = local - (long long)z * nbx;
  const int it = threadIdx.x % IT, g = threadIdx.x / IT;
  const long long q = bx * IT + it;
  const bool live = q < items;
  const int row = live ? (int)(q / c4) : 0, col = live ? (int)(q - (long long)row * c4) * 4 : 0;
  const long long per = (long long)J.M * J.N, slab = per * J.batch;
  const float* src = J.ws + z * per + (long long)row * J.N + col;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    if ((J.N & 3) == 0) {
      v = ordered_slab_sum4(src, slab, g, J.S, G);
    } else {
      for (int s = g; s < J.S; s += G)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (col + j < J.N) v[j] += src[s * slab + j];
    }
  }
  if (G > 1) {
    red[g * IT + it] = v;
    __syncthreads();
    if (g != 0) return;
    for (int s = 1; s < G; ++s) v += red[s * IT + it];
  }
  if (!live) return;
  const int zo = z / J.batch_inner, zi = z - zo * J.batch_inner;
  float* C = J.C + zo * J.c_so + zi * J.c_si + (long long)row * J.ldc + col;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (col + j < J.N) C[j] += v[j] * J.alpha * (J.col_scale ? J.col_scale[col + j] : 1.f);
}

// act_colsum_kernel<CB> with CB a job field (same lanes, same order), once
// per segment
__global__ __launch_bounds__(1024) void defer_colsum_kernel(const ColsumBatch B) {
  __shared__ float red[1024];
  const int k = job_of<CS_PER_LAUNCH>(B.j, B.n, blockIdx.x);
  DefColsum J = B.j[0];
#pragma unroll
  for (int i = 1; i < CS_PER_LAUNCH; ++i)
    if (i == k) J = B.j[i];
  const int CB = J.CB, KL = 1024 / CB;
  const int cl = threadIdx.x % CB, kl = threadIdx.x / CB;
  const int col = (blockIdx.x - J.blk0) * CB + cl;
#pragma unroll
  for (int sg = 0; sg < CS_MAX_SEG; ++sg) {
    if (sg >= J.nseg) break;  // uniform
    const int chunks = J.seg[sg];
    const float* ws = J.ws + J.seg_off[sg];
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (col < J.c) {
      int q = kl;
      for (; q + 3 * KL < chunks; q += 4 * KL) {
        s0 += ws[(long long)q * J.c + col];
        s1 += ws[(long long)(q + KL) * J.c + col];
        s2 += ws[(long long)(q + 2 * KL) * J.c + col];
        s3 += ws[(long long)(q + 3 * KL) * J.c + col];
      }
      for (; q < chunks; q += KL) s0 += ws[(long long)q * J.c + col];
    }
    if (sg > 0) __syncthreads();  // the previous segment's red reads are done
    red[kl * CB + cl] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (kl == 0 && col < J.c) {
      float s = red[cl];
      for (int r = 1; r < KL; ++r) s += red[r * CB + cl];
      if (col < J.c_split) {
        if (J.db) J.db[col] += s;
      } else if (J.db2) {
        J.db2[col - J.c_split] += s;
      }
    }
  }
}

int flush_colsum(hipStream_t s);

int flush_wgrad(hipStream_t s) {
  size_t i = 0;
  while (i < g_def.wg.size()) {
    WgradBatch B{};
    int blocks = 0;
    while (i < g_def.wg.size() && B.n < WG_PER_LAUNCH) {
      DefWgrad J = g_def.wg[i++];
      const int IT = 256 / J.G;
      const long long items = (long long)J.M * ((J.N + 3) / 4);
      J.blk0 = blocks;
      blocks += (int)(((items + IT - 1) / IT) * J.batch);
      B.j[B.n++] = J;
    }
    hipLaunchKernelGGL(defer_wgrad_kernel, dim3(blocks), dim3(256), 0, s, B);
    const int st = check_launch("defer_wgrad_kernel");
    if (st) return st;
  }
  g_def.wg.clear();
  return 0;
}

int flush_colsum(hipStream_t s) {
  size_t i = 0;
  while (i < g_def.cs.size()) {
    ColsumBatch B{};
    int blocks = 0;
    while (i < g_def.cs.size() && B.n < CS_PER_LAUNCH) {
      DefColsum J = g_def.cs[i++];
      J.blk0 = blocks;
      blocks += (J.c + J.CB - 1) / J.CB;
      B.j[B.n++] = J;
    }
    hipLaunchKernelGGL(defer_colsum_kernel, dim3(blocks), dim3(1024), 0, s, B);
    const int st = check_launch("defer_colsum_kernel");
    if (st) return st;
  }
  g_def.cs.clear();
  return 0;
}

// the queued bias-gradient column passes (before the colsum jobs that sum
// their partials)
int flush_direct(hipStream_t s) {
  size_t i = 0;
  while (i < g_def.dir.size()) {
    DirectBatch B{};
    int blocks = 0;
    while (i < g_def.dir.size() && B.n < DIRECT_PER_LAUNCH) {
      DefDirect J = g_def.dir[i++];
      J.blk0 = blocks;
      blocks += J.gx * J.gy;
      B.j[B.n++] = J;
    }
    const int st = direct_colsum_launch(B, blocks, s);
    if (st) return st;
  }
  g_def.dir.clear();
  return 0;
}

// the queued weight-gradient GEMMs: a few grouped launches
int flush_gemm_jobs(hipStream_t s) {
  if (g_def.gj.empty()) return 0;
  const int st = launch_gemm_jobs(g_def.gj.data(), (int)g_def.gj.size(), s);
  g_def.gj.clear();
  return st;
}

// every queued job, in phase order gemm -> direct -> wgrad -> colsum (jobs
// of one flush never share a destination: see overlaps())
int flush_queue(hipStream_t s) {
  int st = flush_gemm_jobs(s);
  if (!st) st = flush_direct(s);
  if (!st) st = flush_wgrad(s);
  if (!st) st = flush_colsum(s);
  return st;
}

// run the queue; the arena is free again for launches ordered after these
int flush_all(hipStream_t s) {
  int st = flush_queue(s);
  g_def.dst.clear();
  g_def.used = 0;
  return st;
}

}  // namespace

bool defer_active() { return g_def.active; }
static bool g_wgrad_queue_ok = false;
bool wgrad_queue_ok() { return g_wgrad_queue_ok; }
void set_wgrad_queue_ok(bool on) { g_wgrad_queue_ok = on; }

long long defer_room() { return g_def.active ? (g_def.bytes - g_def.used) / 4 : 0; }

float* defer_alloc(long long floats) {
  if (!g_def.active || floats <= 0) return nullptr;
  const long long b = ((floats * 4) + 255) & ~255LL;
  if (g_def.used + b > g_def.bytes) return nullptr;
  float* p = (float*)(g_def.base + g_def.used);
  g_def.used += b;
  g_def.peak = std::max(g_def.peak, g_def.used);
  return p;
}

float* partial_f32(long long n) {
  float* p = defer_alloc(n);
  return p ? p : scratch_f32(n);
}

bool defer_owns(const void* p) {
  return g_def.active && p && (const char*)p >= g_def.base && (const char*)p < g_def.base + g_def.bytes;
}

int defer_wgrad(const GemmParams& p, const float* ws, int batch, int G, hipStream_t s) {
  DefWgrad J{};
  J.C = (float*)p.C; J.ws = ws; J.col_scale = p.col_scale;
  J.c_so = p.c_so; J.c_si = p.c_si; J.ldc = p.ldc;
  J.M = p.M; J.N = p.N; J.S = p.split_k; J.batch = batch; J.batch_inner = p.batch_inner; J.G = G;
  J.alpha = p.alpha;
  long long hi = 0;
  for (int z = 0; z < batch; ++z) {
    const int zo = z / p.batch_inner, zi = z - zo * p.batch_inner;
    hi = std::max(hi, zo * p.c_so + zi * p.c_si);
  }
  const Range r{(uintptr_t)J.C, (uintptr_t)(J.C + hi + (long long)(p.M - 1) * p.ldc + p.N)};
  if (overlaps(r)) {  // an earlier queued job adds into the same gradient: keep the order
    // the new job's slabs were written by a launch already on the stream; the
    // flush runs before anything later overwrites the arena, but this job's
    // own slabs must survive it: run the queue without recycling the arena
    const long long keep = g_def.used;
    const int st = flush_queue(s);
    if (st) return st;
    g_def.dst.clear();
    g_def.used = keep;
  }
  g_def.dst.push_back(r);
  g_def.wg.push_back(J);
  return 0;
}

int defer_gemm_job(const DefGemmJob& J, hipStream_t s) {
  const Range r{(uintptr_t)J.C, (uintptr_t)(J.C + (long long)(J.M - 1) * J.ldc + J.N)};
  if (overlaps(r)) {  // a queued job adds into the same gradient: keep the order
    const long long keep = g_def.used;
    const int st = flush_queue(s);
    if (st) return st;
    g_def.dst.clear();
    g_def.used = keep;
  }
  g_def.dst.push_back(r);
  g_def.gj.push_back(J);
  return 0;
}

int defer_touch(const void* lo, const void* hi, hipStream_t s) {
  if (!g_def.active) return 0;
  if (!overlaps(Range{(uintptr_t)lo, (uintptr_t)hi})) return 0;
  // an immediate accumulation into a queued job's destination: run the queue
  // first so the sum order is the immediate mode's (the arena is kept: the
  // caller may be about to read slabs or partials written in it)
  const long long keep = g_def.used;
  const int st = flush_queue(s);
  g_def.dst.clear();
  g_def.used = keep;
  return st;
}

int defer_colsum(int chunks, int c, const float* ws, float* db, int c_split, float* db2, int CB, hipStream_t s) {
  DefColsum J{ws, db, db2, c, c_split, CB, 0, 1, {chunks}, {0}};
  const int n1 = std::min(c, c_split);
  std::vector<Range> rs;
  if (db && n1 > 0) rs.push_back({(uintptr_t)db, (uintptr_t)(db + n1)});
  if (db2 && c > c_split) rs.push_back({(uintptr_t)db2, (uintptr_t)(db2 + (c - c_split))});
  for (const Range& r : rs)
  // the next segment of the last queued colsum job: same destinations, and
  // nothing else queued into them since (its ranges are the last registered;
  // any other job into them would have flushed the queue)
  if (!g_def.cs.empty()) {
    DefColsum& L = g_def.cs.back();
    const size_t nr = rs.size();
    bool tail = nr > 0 && g_def.dst.size() >= nr;
    for (size_t i = 0; tail && i < nr; ++i) {
      const Range& q = g_def.dst[g_def.dst.size() - nr + i];
      tail = q.lo == rs[i].lo && q.hi == rs[i].hi;
    }
    const long long off = ws - L.ws;
    if (tail && L.db == db && L.db2 == db2 && L.c == c && L.c_split == c_split && L.CB == CB &&
        L.nseg < CS_MAX_SEG && off >= 0 && off < (1LL << 31)) {
      L.seg[L.nseg] = chunks;
      L.seg_off[L.nseg++] = (int)off;
      return 0;
    }
  }
  bool ov = false;
  for (const Range& r : rs) ov = ov || overlaps(r);
  if (ov) {
    const long long keep = g_def.used;
    const int st = flush_queue(s);
    if (st) return st;
    g_def.dst.clear();
    g_def.used = keep;
  }
  for (const Range& r : rs) g_def.dst.push_back(r);
  g_def.cs.push_back(J);
  return 0;
}

int defer_direct(const DefDirect& J, hipStream_t s) {
  // a one-chunk job without partials adds into db itself: after any queued job into db
  if (J.gy == 1 && !J.ws) {
    const Range r{(uintptr_t)J.db, (uintptr_t)(J.db + J.c)};
    if (overlaps(r)) {
      const long long keep = g_def.used;
      const int st = flush_queue(s);
      if (st) return st;
      g_def.dst.clear();
      g_def.used = keep;
    }
    g_def.dst.push_back(r);
  }
  g_def.dir.push_back(J);
  return 0;
}

}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

int fpnmt_defer_begin(void* arena, long long bytes) {
  if (g_def.active) return fail(FPNMT_E_ARG, "defer_begin: already active (flush first)");
  if (!arena || bytes <= 0 || ((uintptr_t)arena & 255)) return fail(FPNMT_E_ARG, "defer_begin: need a 256-B aligned arena");
  g_def.base = (char*)arena;
  g_def.bytes = bytes;
  g_def.used = 0;
  g_def.active = true;
  g_def.dir.clear();
  g_def.gj.clear();
  g_def.wg.clear();
  g_def.cs.clear();
  g_def.dst.clear();
  return 0;
}

int fpnmt_defer_flush(fpnmt_stream_t stream) {
  if (!g_def.active) return 0;
  const int st = flush_all((hipStream_t)stream);
  g_def.active = false;
  return st;
}

long long fpnmt_defer_peak_bytes(void) { return g_def.peak; }

}  // extern "C"
