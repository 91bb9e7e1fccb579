// bf16 instantiation set of the MFMA GEMM family (see gemm_impl.h).
#include <algorithm>
#include <cstring>
#include <vector>
#include "gemm_dispatch.h"
namespace fpnmt {
int gemm_bf16(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  return dispatch_gemm_impl<bf16>(p, batch, amode, bmode, vec, s);
}

static GemmParams slab_view(float* C, int M, int N, int ldc, int splits, const float* col_scale) {
  GemmParams p;
  std::memset(&p, 0, sizeof(p));
  p.M = M;
  p.N = N;
  p.C = C;
  p.ldc = ldc;
  p.batch_inner = 1;
  p.alpha = 1.f;
  p.col_scale = col_scale;
  p.accumulate = 2;
  p.c_f32 = 1;
  p.split_k = splits;
  return p;
}

float* wgrad_slabs(int M, int N, int splits) {
  const GemmParams p = slab_view(nullptr, M, N, N, splits, nullptr);
  return slab_fits(p, 1, splits) ? slab_alloc(p, 1, splits) : nullptr;
}

int wgrad_slabs_reduce(float* C, int M, int N, int ldc, int splits, const float* col_scale, const float* slabs,
                       hipStream_t s) {
  return launch_wgrad_reduce(slab_view(C, M, N, ldc, splits, col_scale), 1, slabs, s);
}

// the flush of the deferred weight-gradient GEMMs (deferred.hip): jobs laid
// out block by block, GEMM_JOBS_PER_LAUNCH per launch
#ifndef FPNMT_JOBS_STAGES
#define FPNMT_JOBS_STAGES 2  // two blocks per CU (64 KB of LDS each): measured 0.23 ms per C2 step faster than 4 stages at one block
#endif
int launch_gemm_jobs(const DefGemmJob* jobs_in, int n, hipStream_t s) {
  // longest reductions first (their tiles dispatch first and the short ones
  // fill in behind them); the jobs of one flush share no destination, so
  // their order is free
  std::vector<DefGemmJob> jobs(jobs_in, jobs_in + n);
  std::stable_sort(jobs.begin(), jobs.end(), [](const DefGemmJob& a, const DefGemmJob& b) { return a.K > b.K; });
  int i = 0;
  while (i < n) {
    GemmJobs J{};
    J.zero = g_split_ws.zero;
    int blocks = 0;
    while (i < n && J.n < GEMM_JOBS_PER_LAUNCH) {
      DefGemmJob q = jobs[i++];
      q.tiles_n = cdiv(q.N, 128);
      q.blk0 = blocks;
      blocks += cdiv(q.M, 128) * q.tiles_n;
      J.j[J.n++] = q;
    }
    hipLaunchKernelGGL((gemm_wg_jobs_kernel<128, 128, 2, 4, FPNMT_JOBS_STAGES>), dim3(blocks), dim3(512), 0, s, J);
    const int st = check_launch("gemm_wg_jobs_kernel");
    if (st) return st;
  }
  return 0;
}
}  // namespace fpnmt
