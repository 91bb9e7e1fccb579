// bf16 instantiation set of the MFMA GEMM family (see gemm_impl.h).
#include "gemm_dispatch.h"
namespace fpnmt {
int gemm_bf16(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  return dispatch_gemm_impl<bf16>(p, batch, amode, bmode, vec, s);
}

// the flush of the deferred weight-gradient GEMMs (deferred.hip): jobs laid
// out block by block, GEMM_JOBS_PER_LAUNCH per launch
int launch_gemm_jobs(const DefGemmJob* jobs, int n, hipStream_t s) {
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
    hipLaunchKernelGGL((gemm_wg_jobs_kernel<128, 128, 2, 4>), dim3(blocks), dim3(512), 0, s, J);
    const int st = check_launch("gemm_wg_jobs_kernel");
    if (st) return st;
  }
  return 0;
}
}  // namespace fpnmt
