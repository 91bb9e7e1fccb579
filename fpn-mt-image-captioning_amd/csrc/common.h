// Internal helpers shared by the libfpnmt HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "../../include/fpnmt.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace fpnmt {

// thread-local last-error message (fpnmt_last_error)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);
// Zero fills as kernels (api.hip). hipMemsetAsync / hipMemset2DAsync inside a
// captured hipGraph were measured NOT to re-zero on replay (tools/probes/
// conv_noise.py: the strided 1x1 bwd-data accumulated onto stale memory), so
// every zeroing on a capturable path is an ordinary kernel node.
int zero_fill(void* p, size_t bytes, hipStream_t s);
int zero_fill_2d(void* p, size_t pitch, size_t width_bytes, size_t rows, hipStream_t s);
// fp32 scratch from the process workspace (fpnmt_set_workspace) for the
// ordered two-pass reductions (per-block partials, then a fixed-order sum);
// nullptr when no workspace of n floats is attached. Stream-ordered use only.
float* scratch_f32(long long n);
// >= 256 B of zeros in device memory (the workspace's zero page; nullptr when
// no workspace is attached): a load source for out-of-range taps
const void* zero16_ptr();
// db[col] += sum_k ws[k][col] over `chunks` partial rows, in k order (one
// writer per column; columns >= c_split go to db2[col - c_split]) — elementwise.hip
void colsum_launch(int chunks, int c, const float* ws, float* db, hipStream_t s, int c_split = 1 << 30,
                   float* db2 = nullptr);
// deferred ordered reductions (deferred.hip; fpnmt_defer_begin / _flush):
// while active, slabs / partials go to the caller's arena (defer_alloc) and
// their reductions are queued (colsum_launch over an arena buffer queues
// itself). defer_touch: an immediate accumulation into [lo, hi) is about to
// be issued — runs the queue first if it holds a job for that range.
bool defer_active();
// set only for the duration of an fpnmt_gemm_wgrad call: the caller allows its
// Dense weight-gradient GEMM to be queued until the deferred flush
bool wgrad_queue_ok();
void set_wgrad_queue_ok(bool on);
long long defer_room();  // floats
float* defer_alloc(long long floats);
bool defer_owns(const void* p);
int defer_colsum(int chunks, int c, const float* ws, float* db, int c_split, float* db2, int CB, hipStream_t s);
int defer_touch(const void* lo, const void* hi, hipStream_t s);
// fp32 partial buffer of an ordered two-pass reduction: the deferred arena
// when active, else the process workspace (scratch_f32)
float* partial_f32(long long n);
// bias gradients queued by fpnmt_bias_grad inside a deferred region: the
// column-sum pass of act_bwd (act NONE, dz == dy) over dy, run at the flush
// with the immediate launch's grid (gx column tiles x gy row chunks of rpc
// rows, gt column groups per block): gy == 1 adds into db, else per-chunk
// partials into ws (summed by a queued colsum job)
struct DefDirect {
  const void* dy;
  float* ws;
  float* db;
  long long rows;
  int c, rpc, gt, gx, gy, vec, dtype, blk0;
};
constexpr int DIRECT_PER_LAUNCH = 24;
struct DirectBatch {
  DefDirect j[DIRECT_PER_LAUNCH];
  int n;
};
int direct_colsum_launch(const DirectBatch& B, int blocks, hipStream_t s);  // elementwise.hip
int defer_direct(const DefDirect& J, hipStream_t s);                         // deferred.hip (queues)
// single-filter (k = 1) convolutions as streaming kernels (conv_n1.hip);
// pass 0 fwd, 1 bwd-data (act_in: fused producer act', y_in per level in
// lv.residual), 2 bwd-filter (into dw). 1 launched, 0 not handled, < 0 error
int conv_n1(int pass, const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv, const void* w,
            const float* scale, const float* bias, int act_in, float* dw, hipStream_t s);
// ordered split-K partials for a kernel outside the GEMM family (gemm_bf16.hip):
// room for `splits` fp32 slabs of M x N (the deferred arena while one is
// active, else the workspace; null: no room), and C (fp32, ldc) += col_scale[n] *
// the slabs' split-ordered sum (queued in a deferred region, else launched)
float* wgrad_slabs(int M, int N, int splits);
int wgrad_slabs_reduce(float* C, int M, int N, int ldc, int splits, const float* col_scale, const float* slabs,
                       hipStream_t s);
// ResNet 7x7/2 stem weight gradient (conv_stem.hip): 1 launched, 0 not handled
int stem_conv_bwd_filter(const fpnmt_conv_desc* d, const void* x, const void* dz, const float* col_scale,
                         float* dw_hwio, hipStream_t s);
// ResNet 7x7/2 stem over 3 channels (conv_stem.hip): 1 launched, 0 not handled
int stem_conv_fwd(const fpnmt_conv_desc* d, const void* x, const void* w_ohwi, const float* scale,
                  const float* bias, const void* residual, void* y, hipStream_t s);

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float act_apply(float v, int act, float a) {
  if (act == FPNMT_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == FPNMT_ACT_LEAKY) return v > 0.f ? v : v * a;
  if (act == FPNMT_ACT_RELU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}
// derivative from the activation OUTPUT y (relu/leaky preserve the sign)
__device__ __forceinline__ float act_grad_from_y(float y, int act, float a) {
  if (act == FPNMT_ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == FPNMT_ACT_LEAKY) return y > 0.f ? 1.f : a;
  if (act == FPNMT_ACT_RELU6) return (y > 0.f && y < 6.f) ? 1.f : 0.f;
  return 1.f;
}
// the 0/1 derivative of relu / relu6 (fused act'-mask epilogues)
// act'(pre-activation) read back from the activation's OUTPUT y: ReLU /
// ReLU6 as 0/1 masks; LeakyReLU(alpha) as 1 / alpha (y > 0 iff the input was)
__device__ __forceinline__ float act_mask_from_y(float y, int act, float alpha = 0.f) {
  if (act == FPNMT_ACT_RELU6) return (y > 0.f && y < 6.f) ? 1.f : 0.f;
  if (act == FPNMT_ACT_LEAKY) return y > 0.f ? 1.f : alpha;
  return y > 0.f ? 1.f : 0.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// counter-based hash RNG for dropout (stateless, graph-replay safe when the
// seed/offset live in kernel args of a re-captured graph or device memory)
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t i) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 8);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  return (float)(hash_u32(seed, i) & 0xFFFFFF) * (1.0f / 16777216.0f);
}

inline hipStream_t S(fpnmt_stream_t s) { return (hipStream_t)s; }
inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace fpnmt
