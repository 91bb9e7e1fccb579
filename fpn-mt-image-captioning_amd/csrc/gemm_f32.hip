// f32 (exact f32 MFMA, parity mode) instantiation set of the GEMM family.
#include "gemm_dispatch.h"
namespace fpnmt {
int gemm_f32(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  return dispatch_gemm_impl<float>(p, batch, amode, bmode, vec, s);
}
}  // namespace fpnmt
