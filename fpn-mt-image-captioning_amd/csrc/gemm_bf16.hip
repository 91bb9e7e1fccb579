// bf16 instantiation set of the MFMA GEMM family (see gemm_impl.h).
#include "gemm_dispatch.h"
namespace fpnmt {
int gemm_bf16(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  return dispatch_gemm_impl<bf16>(p, batch, amode, bmode, vec, s);
}
}  // namespace fpnmt
