// C-ABI entry points for the MFMA contractions: general batched GEMM,
// implicit-GEMM convolution (fwd / bwd-data / bwd-filter) and attention
// (QK^T -> masked row softmax -> PV, and its backward), plus error handling.
#include "gemm_impl.h"
#include <cstring>

namespace fpnmt {

static thread_local std::string g_last_error;
SplitWs g_split_ws = {nullptr, nullptr, nullptr, 0, 0};
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}
const void* zero16_ptr() { return g_split_ws.zero; }
float* scratch_f32(long long n) { return (g_split_ws.part && n <= g_split_ws.part_floats) ? g_split_ws.part : nullptr; }
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FPNMT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}

__global__ void zero2d_kernel(char* __restrict__ p, size_t pitch, size_t width, size_t rows) {
  // 16-B stores where the row start and width allow it, bytes otherwise
  const size_t r = blockIdx.y;
  char* row = p + r * pitch;
  const bool vec = (((uintptr_t)row | width) & 15) == 0;
  if (vec) {
    const size_t nv = width / 16;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
      ((uint4*)row)[i] = make_uint4(0u, 0u, 0u, 0u);
  } else {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < width; i += (size_t)gridDim.x * blockDim.x)
      row[i] = 0;
  }
}

int zero_fill_2d(void* p, size_t pitch, size_t width_bytes, size_t rows, hipStream_t s) {
  if (!width_bytes || !rows) return 0;
  if (!p) return fail(FPNMT_E_ARG, "zero_fill: null pointer");
  size_t per = (width_bytes + 15) / 16;
  unsigned gx = (unsigned)std::min<size_t>(4096, (per + 255) / 256);
  size_t ry = rows;
  char* base = (char*)p;
  while (ry > 0) {  // grid.y <= 65535 rows per launch
    const unsigned chunk = (unsigned)std::min<size_t>(ry, 65535);
    hipLaunchKernelGGL(zero2d_kernel, dim3(gx ? gx : 1, chunk), dim3(256), 0, s, base, pitch, width_bytes,
                       (size_t)chunk);
    base += (size_t)chunk * pitch;
    ry -= chunk;
  }
  return check_launch("zero_fill");
}

int zero_fill(void* p, size_t bytes, hipStream_t s) {
  if (!bytes) return 0;
  // one "row" per 256 MiB keeps the per-row index in size_t comfortably
  const size_t row = bytes < ((size_t)1 << 28) ? bytes : ((size_t)1 << 28);
  const size_t rows = bytes / row;
  int e = zero_fill_2d(p, row, row, rows, s);
  if (e || bytes == rows * row) return e;
  return zero_fill_2d((char*)p + rows * row, bytes - rows * row, bytes - rows * row, 1, s);
}

int gemm_bf16(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s);
int gemm_f32(GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s);

static void init_params(GemmParams& p) {
  std::memset(&p, 0, sizeof(p));
  p.batch_inner = 1;
  p.alpha = 1.f;
  p.fd_HoWo = p.fd_Wo = p.fd_C = p.fd_S = p.fd_sHoWo = p.fd_sWo = make_fastdiv(1);
  p.H = p.W = p.Cc = p.Ho = p.Wo = p.Rk = p.Sk = p.sh = p.sw = 1;
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

// one-query attention kernels (decode.hip)
bool attn_q1_ok(const fpnmt_attn_desc* d);
bool attn_small_ok(const fpnmt_attn_desc* d);
int attn_small_fwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const float* mask, void* out,
                   void* weights, hipStream_t s);
int attn_small_bwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const void* weights,
                   const void* dout, void* dq, void* dk, void* dv, hipStream_t s);
int attn_q1_fwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const float* mask, void* out,
                void* weights, hipStream_t s);
int attn_q1_bwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const void* weights,
                const void* dout, void* dq, void* dk, void* dv, hipStream_t s);
bool attn_q1_view_ok(const fpnmt_attn_desc* d, const void* k, const void* v, const void* o1, const void* o2,
                     const void* o3);
int attn_q1_views_fwd(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                      const void* const* v, void* const* out, void* const* w, hipStream_t s);
int attn_q1_views_bwd(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                      const void* const* v, const void* const* w, const void* const* dout, void* const* dq,
                      void* const* dk, void* const* dv, hipStream_t s);

static int run_gemm(int dtype, GemmParams& p, int batch, int amode, int bmode, bool vec, hipStream_t s) {
  if (p.accumulate == 2 && !(p.c_f32 || dtype == FPNMT_F32))
    return fail(FPNMT_E_ARG, "gemm: atomic accumulation needs an fp32 C");
  if (p.accumulate == 2 && dtype == FPNMT_F32) p.c_f32 = 1;
  if (p.split_k > 1 && p.accumulate != 2) return fail(FPNMT_E_ARG, "gemm: split_k > 1 needs accumulate == 2");
  if (p.accumulate == 2 && p.act != FPNMT_ACT_NONE) return fail(FPNMT_E_ARG, "gemm: no activation with atomic accumulation");
  if (p.M <= 0 || p.N <= 0 || batch <= 0) return 0;
  if (p.M >= (1 << 30) || p.N >= (1 << 30) || p.K >= (1 << 30)) return fail(FPNMT_E_UNSUPPORTED, "gemm: dimension too large");
  if (vec) {
    // the vector loaders need every 16-B vector wholly in or out of range:
    // the vectorised extent must divide the contiguous dimension
    const int V = dtype == FPNMT_BF16 ? 8 : 4;
    const bool a_ok = (amode == A_ROW || amode == A_IM2COL) ? p.K % V == 0
                      : amode == A_COL                       ? p.M % V == 0
                                                             : p.Cc % V == 0;  // A_IM2COL_T: features
    const bool b_ok = bmode == B_NK ? p.K % V == 0 : p.N % V == 0;
    vec = a_ok && b_ok;
  }
  if (dtype == FPNMT_BF16) return gemm_bf16(p, batch, amode, bmode, vec, s);
  if (dtype == FPNMT_F32) return gemm_f32(p, batch, amode, bmode, vec, s);
  return fail(FPNMT_E_ARG, "gemm: unknown dtype");
}

static int conv_out(int in, int pa, int pb, int k, int st) { return (in + pa + pb - k) / st + 1; }

// ---- attention helpers: masked row softmax fwd / bwd --------------------
// row = (b*H + h)*Lq + i ; S (fp32, ld lds) -> P (T, ld ldp); pad cols zeroed
template <typename T>
__global__ __launch_bounds__(256) void attn_softmax_kernel(long long rows, int H, int Lq, int Lk,
                                                           const float* __restrict__ Sm, long long lds,
                                                           const float* __restrict__ mask, long long msb,
                                                           long long msh, long long msi, long long msj,
                                                           T* __restrict__ P, long long ldp) {
  const int lane = threadIdx.x & 63;
  const long long r = (blockIdx.x * 256LL + threadIdx.x) >> 6;
  if (r >= rows) return;
  const int i = (int)(r % Lq);
  const long long bh = r / Lq;
  const int h = (int)(bh % H);
  const long long b = bh / H;
  const float* srow = Sm + r * lds;
  const float* mrow = mask ? mask + b * msb + h * msh + (long long)i * msi : nullptr;
  float mx = -INFINITY;
  for (int j = lane; j < Lk; j += 64) {
    float s = srow[j];
    if (mrow) s += mrow[(long long)j * msj] * -1e9f;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Lk; j += 64) {
    float s = srow[j];
    if (mrow) s += mrow[(long long)j * msj] * -1e9f;
    sum += expf(s - mx);
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  T* prow = P + r * ldp;
  for (int j = lane; j < (int)ldp; j += 64) {
    float o = 0.f;
    if (j < Lk) {
      float s = srow[j];
      if (mrow) s += mrow[(long long)j * msj] * -1e9f;
      o = expf(s - mx) * inv;
    }
    prow[j] = from_f32<T>(o);
  }
}

// dS = P * (dP - sum_j dP_j P_j)   (dP fp32 ld ldd; P, dS in T with ld ldp)
template <typename T>
__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(long long rows, int Lk, const T* __restrict__ P,
                                                               const float* __restrict__ dP, long long ldd,
                                                               T* __restrict__ dS, long long ldp) {
  const int lane = threadIdx.x & 63;
  const long long r = (blockIdx.x * 256LL + threadIdx.x) >> 6;
  if (r >= rows) return;
  const T* prow = P + r * ldp;
  const float* drow = dP + r * ldd;
  float dot = 0.f;
  for (int j = lane; j < Lk; j += 64) dot += to_f32(prow[j]) * drow[j];
  dot = wave_sum(dot);
  T* o = dS + r * ldp;
  for (int j = lane; j < (int)ldp; j += 64) o[j] = from_f32<T>(j < Lk ? to_f32(prow[j]) * (drow[j] - dot) : 0.f);
}

}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

const char* fpnmt_last_error(void) { return g_last_error.c_str(); }
int fpnmt_version(void) { return 100; }

int fpnmt_fill_zero(void* p, long long bytes, fpnmt_stream_t stream) {
  if (bytes < 0 || (bytes > 0 && !p)) return fail(FPNMT_E_ARG, "fill_zero: bad buffer");
  if (bytes == 0) return 0;
  return zero_fill(p, (size_t)bytes, S(stream)) ? fail(FPNMT_E_HIP, "fill_zero: launch") : 0;
}

int fpnmt_set_workspace(void* ws, long long bytes) {
  if (!ws || bytes <= 0) {
    g_split_ws = {nullptr, nullptr, nullptr, 0, 0};
    return 0;
  }
  if (((uintptr_t)ws & 255) != 0) return fail(FPNMT_E_ARG, "set_workspace: pointer must be 256-B aligned");
  const long long cnt_bytes = 64 * 1024;  // [0, 256): zero page; then tile counters
  if (bytes < cnt_bytes + 2048 * 4) return fail(FPNMT_E_ARG, "set_workspace: need >= 72 KiB");
  g_split_ws.zero = ws;
  g_split_ws.cnt = (unsigned*)((char*)ws + 256);
  g_split_ws.cnt_n = (int)((cnt_bytes - 256) / 4);
  g_split_ws.part = (float*)((char*)ws + cnt_bytes);
  g_split_ws.part_floats = (bytes - cnt_bytes) / 4;
  return 0;
}

static int gemm_impl_api(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, const float* col_scale,
                         const float* bias, const void* R, int r_mask, float mask_alpha, fpnmt_stream_t stream);

int fpnmt_gemm(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, const float* col_scale,
               const float* bias, const void* R, fpnmt_stream_t stream) {
  return gemm_impl_api(d, A, B, C, col_scale, bias, R, 0, 0.f, stream);
}

int fpnmt_gemm_wgrad(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, fpnmt_stream_t stream) {
  if (!d) return fail(FPNMT_E_ARG, "gemm_wgrad: null pointer");
  if (!d->a_trans || !d->b_trans || !d->c_f32 || (d->accumulate != 1 && d->accumulate != 2) || d->act != FPNMT_ACT_NONE ||
      d->drop_p > 0.f)
    return fail(FPNMT_E_UNSUPPORTED, "gemm_wgrad: a weight gradient is a_trans = b_trans = 1, fp32 C, accumulate 1 / 2, "
                                     "no act / dropout");
  set_wgrad_queue_ok(true);
  const int st = gemm_impl_api(d, A, B, C, nullptr, nullptr, nullptr, 0, 0.f, stream);
  set_wgrad_queue_ok(false);
  return st;
}

int fpnmt_gemm_act_in(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, const void* y_in, int act_in,
                      float act_alpha, fpnmt_stream_t stream) {
  if (!d || !y_in) return fail(FPNMT_E_ARG, "gemm_act_in: null pointer");
  if (act_in != FPNMT_ACT_RELU && act_in != FPNMT_ACT_RELU6 && act_in != FPNMT_ACT_LEAKY)
    return fail(FPNMT_E_ARG, "gemm_act_in: act_in must be relu / relu6 / leaky_relu");
  if (d->act != FPNMT_ACT_NONE || d->drop_p > 0.f || d->accumulate != 0 || d->batch != 1 || d->split_k > 1)
    return fail(FPNMT_E_UNSUPPORTED, "gemm_act_in: plain single GEMM only (no act, dropout, accumulate, batch)");
  return gemm_impl_api(d, A, B, C, nullptr, nullptr, y_in, act_in, act_alpha, stream);
}

static int gemm_impl_api(const fpnmt_gemm_desc* d, const void* A, const void* B, void* C, const float* col_scale,
                         const float* bias, const void* R, int r_mask, float mask_alpha, fpnmt_stream_t stream) {
  if (!d) return fail(FPNMT_E_ARG, "gemm: null pointer");
  if (d->m < 0 || d->n < 0 || d->k < 0 || d->batch < 0 || d->batch_inner <= 0)
    return fail(FPNMT_E_ARG, "gemm: negative size");
  if (d->m == 0 || d->n == 0 || d->batch == 0) return 0;
  if (!C || (d->k > 0 && (!A || !B))) return fail(FPNMT_E_ARG, "gemm: null pointer");
  GemmParams p;
  init_params(p);
  p.M = d->m;
  p.N = d->n;
  p.K = d->k;
  p.A = A;
  p.B = B;
  p.C = C;
  p.R = R;
  p.lda = d->lda;
  p.ldb = d->ldb;
  p.ldc = d->ldc;
  p.ldr = d->ldr;
  p.batch_inner = d->batch_inner;
  p.a_so = d->a_so; p.a_si = d->a_si; p.b_so = d->b_so; p.b_si = d->b_si;
  p.c_so = d->c_so; p.c_si = d->c_si; p.r_so = d->r_so; p.r_si = d->r_si;
  p.alpha = d->alpha;
  p.col_scale = col_scale;
  p.bias = bias;
  p.act = d->act;
  p.act_alpha = d->act_alpha;
  p.accumulate = d->accumulate;
  p.c_f32 = d->c_f32;
  p.split_k = d->split_k;
  if (r_mask) {  // C = (A B) * act_in'(R): the producing layer's activation backward
    p.r_mask = r_mask;
    p.act_alpha = mask_alpha;
  }
  if (d->drop_p > 0.f) {
    if (d->drop_p >= 1.f) return fail(FPNMT_E_ARG, "gemm: drop_p must be < 1");
    if (d->batch != 1 || d->accumulate == 2) return fail(FPNMT_E_UNSUPPORTED, "gemm: fused dropout needs batch 1, no atomics");
    p.drop_p = d->drop_p;
    p.drop_seed = d->drop_seed;
    p.drop_seed_dev = d->drop_seed_dev;
  }
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  const bool vec = aligned16(A) && aligned16(B) && d->lda % V == 0 && d->ldb % V == 0 &&
                   d->a_so % V == 0 && d->a_si % V == 0 && d->b_so % V == 0 && d->b_si % V == 0;
  const int amode = d->a_trans ? A_COL : A_ROW;
  const int bmode = d->b_trans ? B_KN : B_NK;
  return run_gemm(d->dtype, p, d->batch, amode, bmode, vec, S(stream));
}

int fpnmt_conv2d_fwd(const fpnmt_conv_desc* d, const void* x, const void* w_ohwi, const float* scale,
                     const float* bias, const void* residual, void* y, fpnmt_stream_t stream) {
  if (!d) return fail(FPNMT_E_ARG, "conv2d_fwd: null descriptor");
  const int ho = conv_out(d->h, d->pad_t, d->pad_b, d->r, d->stride_h);
  const int wo = conv_out(d->w, d->pad_l, d->pad_r, d->s, d->stride_w);
  if (ho <= 0 || wo <= 0 || d->n <= 0 || d->k <= 0) return 0;  // empty output (e.g. the 0x0 P7 level)
  if (!x || !w_ohwi || !y) return fail(FPNMT_E_ARG, "conv2d_fwd: null pointer");
  {
    const int st = stem_conv_fwd(d, x, w_ohwi, scale, bias, residual, y, S(stream));
    if (st) return st < 0 ? st : 0;
  }
  if (d->k == 1) {
    const fpnmt_conv_level one{d->n, d->h, d->w, x, nullptr, residual, y};
    const int st = conv_n1(0, d, 1, &one, w_ohwi, scale, bias, FPNMT_ACT_NONE, nullptr, S(stream));
    if (st) return st < 0 ? st : 0;
  }
  GemmParams p;
  init_params(p);
  p.M = d->n * ho * wo;
  p.N = d->k;
  p.K = d->r * d->s * d->c;
  p.A = x;
  p.B = w_ohwi;
  p.C = y;
  p.R = residual;
  p.lda = 0;
  p.ldb = p.K;
  p.ldc = d->k;
  p.ldr = d->k;
  p.H = d->h; p.W = d->w; p.Cc = d->c; p.Ho = ho; p.Wo = wo; p.Rk = d->r; p.Sk = d->s;
  p.sh = d->stride_h; p.sw = d->stride_w; p.pt = d->pad_t; p.pl = d->pad_l;
  p.fd_HoWo = make_fastdiv(ho * wo);
  p.fd_Wo = make_fastdiv(wo);
  p.fd_C = make_fastdiv(d->c);
  p.fd_S = make_fastdiv(d->s);
  p.col_scale = scale;
  p.bias = bias;
  p.act = d->act;
  p.act_alpha = d->act_alpha;
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  const bool vec = d->c % V == 0 && aligned16(x) && aligned16(w_ohwi);
  return run_gemm(d->dtype, p, 1, A_IM2COL, B_NK, vec, S(stream));
}

static bool mask_act_ok(int act) { return act == FPNMT_ACT_RELU || act == FPNMT_ACT_RELU6; }

static int conv2d_bwd_data_impl(const fpnmt_conv_desc* d, const void* dz, const void* w_flip, void* dx,
                                int accumulate, const void* y_in, int act_in, fpnmt_stream_t stream,
                                const void* res = nullptr, const void* y2 = nullptr, int act2 = 0,
                                const void* ym = nullptr, int actm = 0) {
  if (!d) return fail(FPNMT_E_ARG, "conv2d_bwd_data: null descriptor");
  if (res && (y_in || accumulate)) return fail(FPNMT_E_ARG, "conv2d_bwd_data_res: no act mask / accumulate");
  if (ym && (y_in || res || !mask_act_ok(actm)))
    return fail(FPNMT_E_ARG, "conv2d_bwd_data_mask: act must be relu / relu6, no other epilogue operand");
  if (y_in && (!mask_act_ok(act_in) || accumulate))
    return fail(FPNMT_E_ARG, "conv2d_bwd_data_act: act_in must be relu / relu6, no accumulate");
  const int ho = conv_out(d->h, d->pad_t, d->pad_b, d->r, d->stride_h);
  const int wo = conv_out(d->w, d->pad_l, d->pad_r, d->s, d->stride_w);
  if ((long long)d->n * d->h * d->w * d->c <= 0) return 0;  // empty dx
  if (!dx || ((ho > 0 && wo > 0) && (!dz || !w_flip))) return fail(FPNMT_E_ARG, "conv2d_bwd_data: null pointer");
  const int esz = d->dtype == FPNMT_BF16 ? 2 : 4;
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  GemmParams p;
  init_params(p);
  p.B = w_flip;
  p.C = dx;
  p.N = d->c;
  p.ldc = d->c;
  p.accumulate = accumulate ? 1 : 0;
  if (ho <= 0 || wo <= 0) {
    if (!accumulate) {
      if (zero_fill(dx, (size_t)d->n * d->h * d->w * d->c * esz, S(stream)))
        return fail(FPNMT_E_HIP, "conv2d_bwd_data: zero fill");
    }
    return 0;
  }
  if (d->k == 1 && !accumulate && !res && !ym) {
    const fpnmt_conv_level one{d->n, d->h, d->w, dz, nullptr, y_in, dx};
    const int st = conv_n1(1, d, 1, &one, w_flip, nullptr, nullptr, y_in ? act_in : FPNMT_ACT_NONE, nullptr,
                           S(stream));
    if (st) return st < 0 ? st : 0;
  }
  if (d->stride_h == 1 && d->stride_w == 1) {
    // dx = conv(dz, w_flip) with pads R-1-pt, S-1-pl over the (h, w) output grid
    p.M = d->n * d->h * d->w;
    p.K = d->r * d->s * d->k;
    p.A = dz;
    p.ldb = p.K;
    p.H = ho; p.W = wo; p.Cc = d->k; p.Ho = d->h; p.Wo = d->w; p.Rk = d->r; p.Sk = d->s;
    p.sh = 1; p.sw = 1; p.pt = d->r - 1 - d->pad_t; p.pl = d->s - 1 - d->pad_l;
    p.fd_HoWo = make_fastdiv(d->h * d->w);
    p.fd_Wo = make_fastdiv(d->w);
    p.fd_C = make_fastdiv(d->k);
    p.fd_S = make_fastdiv(d->s);
    if (y_in) {  // dx *= act_in'(y_in): the producing layer's act_bwd in the epilogue
      p.R = y_in;
      p.ldr = d->c;
      p.r_mask = act_in;
    } else if (res) {  // dx += res: the input's other gradient, added before the store
      p.R = res;
      p.ldr = d->c;
      p.r_mask = 0;
      if (y2) {  // then dx *= act2'(y2): the producer of the input's act_bwd
        p.M2 = y2;
        p.m2_act = act2;
      }
    }
    if (ym) {  // this launch's contribution times actm'(ym), ym in dx's layout
      p.M2 = ym;
      p.m2_act = actm;
      p.ldr = d->c;
    }
    const bool vec = d->k % V == 0 && aligned16(dz) && aligned16(w_flip);
    return run_gemm(d->dtype, p, 1, A_IM2COL, B_NK, vec, S(stream));
  }
  if (y_in || res) return fail(FPNMT_E_UNSUPPORTED, "conv2d_bwd_data_act / _res: stride 1 only");
  if (d->r == 1 && d->s == 1 && d->pad_t == 0 && d->pad_l == 0 && d->stride_h == d->stride_w) {
    if (!accumulate) {
      if (zero_fill(dx, (size_t)d->n * d->h * d->w * d->c * esz, S(stream)))
        return fail(FPNMT_E_HIP, "conv2d_bwd_data: zero fill");
      p.accumulate = 1;
    }
    p.M = d->n * ho * wo;
    p.K = d->k;
    p.A = dz;
    p.lda = d->k;
    p.ldb = d->k;
    p.c_mode = C_SCATTER;
    p.scat_Hd = d->h;
    p.scat_Wd = d->w;
    p.scat_s = d->stride_h;
    p.fd_sHoWo = make_fastdiv(ho * wo);
    p.fd_sWo = make_fastdiv(wo);
    if (ym) {  // masked at the scattered rows; the rows left zero stay zero
      p.M2 = ym;
      p.m2_act = actm;
      p.ldr = d->c;
    }
    const bool vec = d->k % V == 0 && aligned16(dz) && aligned16(w_flip);
    return run_gemm(d->dtype, p, 1, A_ROW, B_NK, vec, S(stream));
  }
  return fail(FPNMT_E_UNSUPPORTED, "conv2d_bwd_data: only stride 1, or 1x1 stride s pad 0");
}

int fpnmt_conv2d_bwd_data(const fpnmt_conv_desc* d, const void* dz, const void* w_flip, void* dx, int accumulate,
                          fpnmt_stream_t stream) {
  return conv2d_bwd_data_impl(d, dz, w_flip, dx, accumulate, nullptr, FPNMT_ACT_NONE, stream);
}

int fpnmt_conv2d_bwd_data_mask(const fpnmt_conv_desc* d, const void* dz, const void* w_flip, void* dx,
                               int accumulate, const void* y, int act, fpnmt_stream_t stream) {
  if (!y) return fail(FPNMT_E_ARG, "conv2d_bwd_data_mask: null y");
  return conv2d_bwd_data_impl(d, dz, w_flip, dx, accumulate, nullptr, FPNMT_ACT_NONE, stream, nullptr, nullptr, 0, y,
                              act);
}

int fpnmt_conv2d_bwd_data_act(const fpnmt_conv_desc* d, const void* dz, const void* w_flip, void* dx,
                              const void* y_in, int act_in, fpnmt_stream_t stream) {
  if (!y_in) return fail(FPNMT_E_ARG, "conv2d_bwd_data_act: null y_in");
  return conv2d_bwd_data_impl(d, dz, w_flip, dx, 0, y_in, act_in, stream);
}

int fpnmt_conv2d_bwd_data_res(const fpnmt_conv_desc* d, const void* dz, const void* w_flip, void* dx,
                              const void* res, fpnmt_stream_t stream) {
  if (!res) return fail(FPNMT_E_ARG, "conv2d_bwd_data_res: null res");
  return conv2d_bwd_data_impl(d, dz, w_flip, dx, 0, nullptr, FPNMT_ACT_NONE, stream, res);
}

int fpnmt_conv2d_bwd_data_res_act(const fpnmt_conv_desc* d, const void* dz, const void* w_flip, void* dx,
                                  const void* res, const void* y_in, int act_in, fpnmt_stream_t stream) {
  if (!res || !y_in) return fail(FPNMT_E_ARG, "conv2d_bwd_data_res_act: null res / y_in");
  if (!mask_act_ok(act_in)) return fail(FPNMT_E_ARG, "conv2d_bwd_data_res_act: act_in must be relu / relu6");
  return conv2d_bwd_data_impl(d, dz, w_flip, dx, 0, nullptr, FPNMT_ACT_NONE, stream, res, y_in, act_in);
}

// db (optional, fp32 [k]): db += the column sums of dz, folded into the
// LDS-DMA weight-gradient kernel where that kernel runs (it streams dz through
// LDS anyway), else the separate column pass of fpnmt_bias_grad
static int conv_bwd_filter(const fpnmt_conv_desc* d, const void* x, const void* dz, const float* col_scale,
                           float* dw_hwio, float* db, fpnmt_stream_t stream);

int fpnmt_conv2d_bwd_filter(const fpnmt_conv_desc* d, const void* x, const void* dz, const float* col_scale,
                            float* dw_hwio, fpnmt_stream_t stream) {
  return conv_bwd_filter(d, x, dz, col_scale, dw_hwio, nullptr, stream);
}

int fpnmt_conv2d_bwd_filter_bias(const fpnmt_conv_desc* d, const void* x, const void* dz, const float* col_scale,
                                 float* dw_hwio, float* db, fpnmt_stream_t stream) {
  return conv_bwd_filter(d, x, dz, col_scale, dw_hwio, db, stream);
}

static int conv_bwd_filter(const fpnmt_conv_desc* d, const void* x, const void* dz, const float* col_scale,
                           float* dw_hwio, float* db, fpnmt_stream_t stream) {
  if (!d) return fail(FPNMT_E_ARG, "conv2d_bwd_filter: null descriptor");
  const int ho = conv_out(d->h, d->pad_t, d->pad_b, d->r, d->stride_h);
  const int wo = conv_out(d->w, d->pad_l, d->pad_r, d->s, d->stride_w);
  if (ho <= 0 || wo <= 0 || d->n <= 0) return 0;  // no pixels: nothing to add
  if (!x || !dz || !dw_hwio) return fail(FPNMT_E_ARG, "conv2d_bwd_filter: null pointer");
  const long long pix = (long long)d->n * ho * wo;
  // the separate column pass (after the weight gradient, as the fold would add)
  auto bias_pass = [&](int st) {
    return (st || !db) ? st : fpnmt_bias_grad(d->dtype, pix, d->k, dz, db, stream);
  };
  if (d->k == 1) {
    const fpnmt_conv_level one{d->n, d->h, d->w, x, dz, nullptr, nullptr};
    const int st = conv_n1(2, d, 1, &one, nullptr, col_scale, nullptr, FPNMT_ACT_NONE, dw_hwio, S(stream));
    if (st) return bias_pass(st < 0 ? st : 0);
  }
  {
    const int st = stem_conv_bwd_filter(d, x, dz, col_scale, dw_hwio, S(stream));
    if (st) return bias_pass(st < 0 ? st : 0);
  }
  GemmParams p;
  init_params(p);
  p.M = d->r * d->s * d->c;
  p.N = d->k;
  p.K = d->n * ho * wo;
  p.A = x;
  p.B = dz;
  p.C = dw_hwio;
  p.ldb = d->k;
  p.ldc = d->k;
  p.H = d->h; p.W = d->w; p.Cc = d->c; p.Ho = ho; p.Wo = wo; p.Rk = d->r; p.Sk = d->s;
  p.sh = d->stride_h; p.sw = d->stride_w; p.pt = d->pad_t; p.pl = d->pad_l;
  p.fd_HoWo = make_fastdiv(ho * wo);
  p.fd_Wo = make_fastdiv(wo);
  p.fd_C = make_fastdiv(d->c);
  p.fd_S = make_fastdiv(d->s);
  p.col_scale = col_scale;
  p.accumulate = 2;
  p.c_f32 = 1;
  p.split_k = 0;  // auto
  p.cs_db = db;
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  const bool vec = d->c % V == 0 && d->k % V == 0 && aligned16(x) && aligned16(dz);
  const int st = run_gemm(d->dtype, p, 1, A_IM2COL_T, B_KN, vec, S(stream));
  if (st || !p.cs_db) return st;  // error, or the kernel folded the column sums
  return fpnmt_bias_grad(d->dtype, pix, d->k, dz, db, stream);
}

// ---- grouped (multi-level) convolution --------------------------------
static void set_group_geom(GemmGroup& g, int H, int W, int Ho, int Wo) {
  g.H = H; g.W = W; g.Ho = Ho; g.Wo = Wo;
  g.fd_HoWo = make_fastdiv(Ho * Wo);
  g.fd_Wo = make_fastdiv(Wo);
}

// Grouped launches that go to the pipelined kernel (one 128x256 tile per CU):
// a level whose tiles would spill a few past a multiple of the CU count goes
// to the next launch instead. P3 + P4 of the batch-32 step fill 245 of 256
// CUs; adding P5..P7 made 260 tiles, i.e. a second full tile time for 4 tiles
// (100 us per subnet conv instead of ~55).
static int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}
static bool pipe_tail_break(int dtype, int n_out, int k_red, int c_in, long long tiles_now, long long m_level) {
  if (dtype != FPNMT_BF16 || n_out < 256 || k_red % 64 || c_in % 64 || tiles_now == 0) return false;
  const long long cus = cu_count();
  const long long after = tiles_now + ((m_level + 127) / 128) * ((n_out + 255) / 256);
  return (after + cus - 1) / cus > (tiles_now + cus - 1) / cus && after % cus != 0 && after % cus <= cus / 4;
}

int fpnmt_conv2d_fwd_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                             const void* w_ohwi, const float* scale, const float* bias,
                             fpnmt_stream_t stream) {
  if (!d || (n_levels > 0 && !lv)) return fail(FPNMT_E_ARG, "conv2d_fwd_grouped: null descriptor");
  if (d->k == 1) {
    const int st = conv_n1(0, d, n_levels, lv, w_ohwi, scale, bias, FPNMT_ACT_NONE, nullptr, S(stream));
    if (st) return st < 0 ? st : 0;
  }
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  int i = 0;
  while (i < n_levels) {
    GemmParams p;
    init_params(p);
    p.N = d->k;
    p.K = d->r * d->s * d->c;
    p.B = w_ohwi;
    p.ldb = p.K;
    p.ldc = d->k;
    p.ldr = d->k;
    p.Cc = d->c; p.Rk = d->r; p.Sk = d->s;
    p.sh = d->stride_h; p.sw = d->stride_w; p.pt = d->pad_t; p.pl = d->pad_l;
    p.fd_C = make_fastdiv(d->c);
    p.fd_S = make_fastdiv(d->s);
    p.col_scale = scale;
    p.bias = bias;
    p.act = d->act;
    p.act_alpha = d->act_alpha;
    bool vec = d->c % V == 0 && aligned16(w_ohwi);
    int any_res = -1;
    long long tiles_now = 0;
    for (; i < n_levels && p.ngroups < MAX_GROUPS; ++i) {
      const fpnmt_conv_level& L = lv[i];
      const int ho = conv_out(L.h, d->pad_t, d->pad_b, d->r, d->stride_h);
      const int wo = conv_out(L.w, d->pad_l, d->pad_r, d->s, d->stride_w);
      if (ho <= 0 || wo <= 0 || L.n <= 0 || d->k <= 0) continue;
      const long long m_level = (long long)L.n * ho * wo;
      if (pipe_tail_break(d->dtype, d->k, p.K, d->c, tiles_now, m_level)) break;
      tiles_now += ((m_level + 127) / 128) * ((d->k + 255) / 256);
      if (!L.x || !L.y || !w_ohwi) return fail(FPNMT_E_ARG, "conv2d_fwd_grouped: null pointer");
      const int has_res = L.residual != nullptr;
      if (any_res >= 0 && any_res != has_res) return fail(FPNMT_E_ARG, "conv2d_fwd_grouped: residual on some levels only");
      any_res = has_res;
      GemmGroup& g = p.groups[p.ngroups++];
      g.A = L.x; g.B = w_ohwi; g.C = L.y; g.R = L.residual;
      g.M = L.n * ho * wo;
      g.K = p.K;
      set_group_geom(g, L.h, L.w, ho, wo);
      p.M += g.M;
      vec = vec && aligned16(L.x);
    }
    if (p.ngroups == 0) continue;
    // the first group's values double as the plain-problem fields
    p.A = p.groups[0].A; p.C = p.groups[0].C; p.R = p.groups[0].R;
    p.H = p.groups[0].H; p.W = p.groups[0].W; p.Ho = p.groups[0].Ho; p.Wo = p.groups[0].Wo;
    p.fd_HoWo = p.groups[0].fd_HoWo; p.fd_Wo = p.groups[0].fd_Wo;
    const int st = run_gemm(d->dtype, p, 1, A_IM2COL, B_NK, vec, S(stream));
    if (st) return st;
  }
  return 0;
}

// masked: fpnmt_conv2d_bwd_data_grouped_mask (the act mask on this launch's
// contribution, accumulating too; a level without lv.residual gets none)
static int conv2d_bwd_data_grouped_impl(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                        const void* w_flip, int accumulate, int act_in, fpnmt_stream_t stream,
                                        bool masked = false) {
  if (!d || (n_levels > 0 && !lv)) return fail(FPNMT_E_ARG, "conv2d_bwd_data_grouped: null descriptor");
  if (act_in != FPNMT_ACT_NONE && (!mask_act_ok(act_in) || (accumulate && !masked)))
    return fail(FPNMT_E_ARG, "conv2d_bwd_data_grouped_act: act_in must be relu / relu6, no accumulate");
  if (d->stride_h != 1 || d->stride_w != 1) return fail(FPNMT_E_UNSUPPORTED, "conv2d_bwd_data_grouped: stride 1 only");
  if (d->k == 1 && !accumulate && !masked) {
    bool all_out = true;  // levels without output pixels need the zero fill below
    for (int i = 0; i < n_levels; ++i)
      if ((long long)lv[i].n * lv[i].h * lv[i].w > 0 &&
          (lv[i].h + d->pad_t + d->pad_b - d->r < 0 || lv[i].w + d->pad_l + d->pad_r - d->s < 0))
        all_out = false;
    const int st = all_out ? conv_n1(1, d, n_levels, lv, w_flip, nullptr, nullptr, act_in, nullptr, S(stream)) : 0;
    if (st) return st < 0 ? st : 0;
  }
  const int esz = d->dtype == FPNMT_BF16 ? 2 : 4;
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  int i = 0;
  while (i < n_levels) {
    GemmParams p;
    init_params(p);
    p.N = d->c;
    p.K = d->r * d->s * d->k;
    p.B = w_flip;
    p.ldb = p.K;
    p.ldc = d->c;
    p.accumulate = accumulate ? 1 : 0;
    p.Cc = d->k; p.Rk = d->r; p.Sk = d->s;
    p.sh = 1; p.sw = 1; p.pt = d->r - 1 - d->pad_t; p.pl = d->s - 1 - d->pad_l;
    p.fd_C = make_fastdiv(d->k);
    p.fd_S = make_fastdiv(d->s);
    if (act_in != FPNMT_ACT_NONE) {
      p.ldr = d->c;
      p.r_mask = act_in;
    }
    bool vec = d->k % V == 0 && aligned16(w_flip);
    long long tiles_now = 0;
    for (; i < n_levels && p.ngroups < MAX_GROUPS; ++i) {
      const fpnmt_conv_level& L = lv[i];
      if ((long long)L.n * L.h * L.w * d->c <= 0) continue;
      const int ho = conv_out(L.h, d->pad_t, d->pad_b, d->r, 1);
      const int wo = conv_out(L.w, d->pad_l, d->pad_r, d->s, 1);
      if (ho > 0 && wo > 0) {
        const long long m_level = (long long)L.n * L.h * L.w;
        if (pipe_tail_break(d->dtype, d->c, p.K, d->k, tiles_now, m_level)) break;
        tiles_now += ((m_level + 127) / 128) * ((d->c + 255) / 256);
      }
      if (!L.y) return fail(FPNMT_E_ARG, "conv2d_bwd_data_grouped: null dx");
      if (ho <= 0 || wo <= 0) {
        if (!accumulate && zero_fill(L.y, (size_t)L.n * L.h * L.w * d->c * esz, S(stream)))
          return fail(FPNMT_E_HIP, "conv2d_bwd_data_grouped: zero fill");
        continue;
      }
      if (!L.x || !w_flip || (act_in != FPNMT_ACT_NONE && !L.residual && !masked))
        return fail(FPNMT_E_ARG, "conv2d_bwd_data_grouped: null pointer");
      GemmGroup& g = p.groups[p.ngroups++];
      g.A = L.x; g.B = w_flip; g.C = L.y; g.R = act_in != FPNMT_ACT_NONE ? L.residual : nullptr;
      g.M = L.n * L.h * L.w;
      g.K = p.K;
      // implicit GEMM over the dz grid (ho, wo) producing the (h, w) grid
      set_group_geom(g, ho, wo, L.h, L.w);
      p.M += g.M;
      vec = vec && aligned16(L.x);
    }
    if (p.ngroups == 0) continue;
    p.A = p.groups[0].A; p.C = p.groups[0].C; p.R = p.groups[0].R;
    p.H = p.groups[0].H; p.W = p.groups[0].W; p.Ho = p.groups[0].Ho; p.Wo = p.groups[0].Wo;
    p.fd_HoWo = p.groups[0].fd_HoWo; p.fd_Wo = p.groups[0].fd_Wo;
    const int st = run_gemm(d->dtype, p, 1, A_IM2COL, B_NK, vec, S(stream));
    if (st) return st;
  }
  return 0;
}

int fpnmt_conv2d_bwd_data_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                  const void* w_flip, int accumulate, fpnmt_stream_t stream) {
  return conv2d_bwd_data_grouped_impl(d, n_levels, lv, w_flip, accumulate, FPNMT_ACT_NONE, stream);
}

int fpnmt_conv2d_bwd_data_grouped_act(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                      const void* w_flip, int act_in, fpnmt_stream_t stream) {
  return conv2d_bwd_data_grouped_impl(d, n_levels, lv, w_flip, 0, act_in, stream);
}

int fpnmt_conv2d_bwd_data_grouped_mask(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                       const void* w_flip, int accumulate, int act, fpnmt_stream_t stream) {
  if (!mask_act_ok(act)) return fail(FPNMT_E_ARG, "conv2d_bwd_data_grouped_mask: act must be relu / relu6");
  return conv2d_bwd_data_grouped_impl(d, n_levels, lv, w_flip, accumulate, act, stream, true);
}

int fpnmt_fill_zero_grid(void* p, long long bytes, int max_blocks, fpnmt_stream_t stream) {
  if (bytes <= 0) return bytes < 0 ? fail(FPNMT_E_ARG, "fill_zero_grid: negative size") : 0;
  if (!p) return fail(FPNMT_E_ARG, "fill_zero_grid: null pointer");
  if (((uintptr_t)p | (uintptr_t)bytes) & 15) return fpnmt_fill_zero(p, bytes, stream);
  const size_t nv = (size_t)bytes / 16;
  const unsigned g = (unsigned)std::max<size_t>(1, std::min<size_t>(max_blocks > 0 ? max_blocks : 4096, (nv + 255) / 256));
  // one row of `bytes` (the kernel's per-row index is size_t)
  hipLaunchKernelGGL(zero2d_kernel, dim3(g, 1), dim3(256), 0, S(stream), (char*)p, (size_t)bytes, (size_t)bytes,
                     (size_t)1);
  return check_launch("fill_zero_grid");
}

static int conv_bwd_filter_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                   const float* col_scale, float* dw_hwio, float* db, fpnmt_stream_t stream);

int fpnmt_conv2d_bwd_filter_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                    const float* col_scale, float* dw_hwio, fpnmt_stream_t stream) {
  return conv_bwd_filter_grouped(d, n_levels, lv, col_scale, dw_hwio, nullptr, stream);
}

int fpnmt_conv2d_bwd_filter_grouped_bias(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                         const float* col_scale, float* dw_hwio, float* db, fpnmt_stream_t stream) {
  return conv_bwd_filter_grouped(d, n_levels, lv, col_scale, dw_hwio, db, stream);
}

static int conv_bwd_filter_grouped(const fpnmt_conv_desc* d, int n_levels, const fpnmt_conv_level* lv,
                                   const float* col_scale, float* dw_hwio, float* db, fpnmt_stream_t stream) {
  if (!d || (n_levels > 0 && !lv)) return fail(FPNMT_E_ARG, "conv2d_bwd_filter_grouped: null descriptor");
  // the separate column pass of levels [lo, hi) (the ones whose launch did not fold it)
  auto bias_pass = [&](int lo, int hi) {
    for (int j = lo; j < hi && db; ++j) {
      const int ho = conv_out(lv[j].h, d->pad_t, d->pad_b, d->r, d->stride_h);
      const int wo = conv_out(lv[j].w, d->pad_l, d->pad_r, d->s, d->stride_w);
      if (ho <= 0 || wo <= 0 || lv[j].n <= 0 || !lv[j].dz) continue;
      const int st = fpnmt_bias_grad(d->dtype, (long long)lv[j].n * ho * wo, d->k, lv[j].dz, db, stream);
      if (st) return st;
    }
    return 0;
  };
  if (d->k == 1) {
    const int st = conv_n1(2, d, n_levels, lv, nullptr, col_scale, nullptr, FPNMT_ACT_NONE, dw_hwio, S(stream));
    if (st) return st < 0 ? st : bias_pass(0, n_levels);
  }
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  int i = 0;
  while (i < n_levels) {
    const int i0 = i;
    GemmParams p;
    init_params(p);
    p.M = d->r * d->s * d->c;
    p.N = d->k;
    p.C = dw_hwio;
    p.ldb = d->k;
    p.ldc = d->k;
    p.Cc = d->c; p.Rk = d->r; p.Sk = d->s;
    p.sh = d->stride_h; p.sw = d->stride_w; p.pt = d->pad_t; p.pl = d->pad_l;
    p.fd_C = make_fastdiv(d->c);
    p.fd_S = make_fastdiv(d->s);
    p.col_scale = col_scale;
    p.accumulate = 2;
    p.c_f32 = 1;
    p.group_k = 1;
    bool vec = d->c % V == 0 && d->k % V == 0;
    for (; i < n_levels && p.ngroups < MAX_GROUPS; ++i) {
      const fpnmt_conv_level& L = lv[i];
      const int ho = conv_out(L.h, d->pad_t, d->pad_b, d->r, d->stride_h);
      const int wo = conv_out(L.w, d->pad_l, d->pad_r, d->s, d->stride_w);
      if (ho <= 0 || wo <= 0 || L.n <= 0) continue;
      if (!L.x || !L.dz || !dw_hwio) return fail(FPNMT_E_ARG, "conv2d_bwd_filter_grouped: null pointer");
      GemmGroup& g = p.groups[p.ngroups++];
      g.A = L.x; g.B = L.dz; g.C = dw_hwio; g.R = nullptr;
      g.M = p.M;
      g.K = L.n * ho * wo;
      set_group_geom(g, L.h, L.w, ho, wo);
      p.K += g.K;
      vec = vec && aligned16(L.x) && aligned16(L.dz);
    }
    if (p.ngroups == 0) continue;
    p.A = p.groups[0].A; p.B = p.groups[0].B;
    p.H = p.groups[0].H; p.W = p.groups[0].W; p.Ho = p.groups[0].Ho; p.Wo = p.groups[0].Wo;
    p.fd_HoWo = p.groups[0].fd_HoWo; p.fd_Wo = p.groups[0].fd_Wo;
    p.cs_db = db;
    int st = run_gemm(d->dtype, p, 1, A_IM2COL_T, B_KN, vec, S(stream));
    if (!st && p.cs_db) st = bias_pass(i0, i);  // not folded by the launch
    if (st) return st;
  }
  return 0;
}

size_t fpnmt_attention_ws_bytes(const fpnmt_attn_desc* d) {
  if (!d) return 0;
  const size_t rows = (size_t)d->b * d->h * d->lq;
  const size_t esz = d->dtype == FPNMT_BF16 ? 2 : 4;
  return rows * (size_t)d->ldw * (4 + esz) + 256;
}

static int attn_check(const fpnmt_attn_desc* d) {
  if (!d) return fail(FPNMT_E_ARG, "attention: null desc");
  if (d->b < 0 || d->h <= 0 || d->lq < 0 || d->lk < 0 || d->d <= 0) return fail(FPNMT_E_ARG, "attention: bad sizes");
  if (d->ldw < d->lk || d->ldw % 8 != 0) return fail(FPNMT_E_ARG, "attention: ldw must be >= lk and a multiple of 8");
  return 0;
}

int fpnmt_attention_fwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const float* mask,
                        void* out, void* weights, void* ws, fpnmt_stream_t stream) {
  int e = attn_check(d);
  if (e) return e;
  if (d->b == 0 || d->lq == 0) return 0;
  hipStream_t s = S(stream);
  if (attn_q1_ok(d)) return attn_q1_fwd(d, q, k, v, mask, out, weights, s);
  if (attn_small_ok(d)) return attn_small_fwd(d, q, k, v, mask, out, weights, s);
  const int B = d->b, H = d->h, Lq = d->lq, Lk = d->lk, D = d->d;
  const long long ldw = d->ldw;
  float* Sbuf = (float*)ws;
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  // 1) S = scale * Q K^T  (fp32)
  if (Lk > 0) {
    GemmParams p;
    init_params(p);
    p.M = Lq; p.N = Lk; p.K = D;
    p.A = q; p.B = k; p.C = Sbuf;
    p.lda = d->ldq; p.ldb = d->ldk; p.ldc = ldw;
    p.batch_inner = H;
    p.a_so = (long long)Lq * d->ldq; p.a_si = D;
    p.b_so = (long long)Lk * d->ldk; p.b_si = D;
    p.c_so = (long long)H * Lq * ldw; p.c_si = (long long)Lq * ldw;
    p.alpha = d->scale;
    p.c_f32 = 1;
    const bool vec = aligned16(q) && aligned16(k) && d->ldq % V == 0 && d->ldk % V == 0 && D % V == 0;
    e = run_gemm(d->dtype, p, B * H, A_ROW, B_NK, vec, s);
    if (e) return e;
  }
  // 2) P = softmax(S + mask * -1e9)
  const long long rows = (long long)B * H * Lq;
  const int grid = (int)((rows * 64 + 255) / 256);
  if (d->dtype == FPNMT_BF16)
    hipLaunchKernelGGL((attn_softmax_kernel<bf16>), dim3(grid), dim3(256), 0, s, rows, H, Lq, Lk, Sbuf, ldw, mask,
                       d->m_sb, d->m_sh, d->m_si, d->m_sj, (bf16*)weights, ldw);
  else
    hipLaunchKernelGGL((attn_softmax_kernel<float>), dim3(grid), dim3(256), 0, s, rows, H, Lq, Lk, Sbuf, ldw, mask,
                       d->m_sb, d->m_sh, d->m_si, d->m_sj, (float*)weights, ldw);
  e = check_launch("attn_softmax");
  if (e) return e;
  // 3) O = P V
  GemmParams p;
  init_params(p);
  p.M = Lq; p.N = D; p.K = Lk;
  p.A = weights; p.B = v; p.C = out;
  p.lda = ldw; p.ldb = d->ldv; p.ldc = d->ldo;
  p.batch_inner = H;
  p.a_so = (long long)H * Lq * ldw; p.a_si = (long long)Lq * ldw;
  p.b_so = (long long)Lk * d->ldv; p.b_si = D;
  p.c_so = (long long)Lq * d->ldo; p.c_si = D;
  const bool vec = aligned16(weights) && aligned16(v) && d->ldv % V == 0 && D % V == 0;
  return run_gemm(d->dtype, p, B * H, A_ROW, B_KN, vec, s);
}

// n views sharing b / h / scale, all one-query bf16 D = 64 without a mask:
// one grouped launch; anything else: the views one by one
static bool views_grouped(int n, const fpnmt_attn_desc* d, const float* const* mask) {
  if (n <= 0) return false;
  for (int i = 0; i < n; ++i)
    if ((mask && mask[i]) || d[i].b != d[0].b || d[i].h != d[0].h || d[i].scale != d[0].scale) return false;
  return true;
}

// a view without images or queries has nothing to compute (the single-view
// entries return at once); the grouped launch takes the others
static bool view_empty(const fpnmt_attn_desc& d) { return d.b == 0 || d.lq == 0; }

int fpnmt_attention_fwd_views(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                              const void* const* v, const float* const* mask, void* const* out,
                              void* const* weights, void* const* ws, fpnmt_stream_t stream) {
  if (n < 0 || n > FPNMT_MAX_VIEWS) return fail(FPNMT_E_ARG, "attention_fwd_views: 0 <= n <= FPNMT_MAX_VIEWS");
  if (n > 0 && (!d || !q || !k || !v || !out || !weights || !ws))
    return fail(FPNMT_E_ARG, "attention_fwd_views: null table");
  bool grouped = views_grouped(n, d, mask);
  fpnmt_attn_desc gd[FPNMT_MAX_VIEWS];
  const void *gq[FPNMT_MAX_VIEWS], *gk[FPNMT_MAX_VIEWS], *gv[FPNMT_MAX_VIEWS];
  void *go[FPNMT_MAX_VIEWS], *gw[FPNMT_MAX_VIEWS];
  int ng = 0;
  for (int i = 0; i < n; ++i) {
    const int e = attn_check(&d[i]);
    if (e) return e;
    if (view_empty(d[i])) continue;
    grouped = grouped && attn_q1_view_ok(&d[i], k[i], v[i], out[i], nullptr, nullptr) && q[i] && weights[i];
    gd[ng] = d[i]; gq[ng] = q[i]; gk[ng] = k[i]; gv[ng] = v[i]; go[ng] = out[i]; gw[ng] = weights[i];
    ++ng;
  }
  if (grouped && ng > 0) {
    const int e = attn_q1_views_fwd(ng, gd, gq, gk, gv, go, gw, S(stream));
    if (e) return e;
  }
  for (int i = 0; i < n; ++i) {
    if (grouped && ng > 0 && !view_empty(d[i])) continue;
    const int e = fpnmt_attention_fwd(&d[i], q[i], k[i], v[i], mask ? mask[i] : nullptr, out[i], weights[i], ws[i],
                                      stream);
    if (e) return e;
  }
  return 0;
}

int fpnmt_attention_bwd_views(int n, const fpnmt_attn_desc* d, const void* const* q, const void* const* k,
                              const void* const* v, const void* const* weights, const void* const* d_out,
                              void* const* dq, void* const* dk, void* const* dv, void* const* ws,
                              fpnmt_stream_t stream) {
  if (n < 0 || n > FPNMT_MAX_VIEWS) return fail(FPNMT_E_ARG, "attention_bwd_views: 0 <= n <= FPNMT_MAX_VIEWS");
  if (n > 0 && (!d || !q || !k || !v || !weights || !d_out || !dq || !dk || !dv || !ws))
    return fail(FPNMT_E_ARG, "attention_bwd_views: null table");
  bool grouped = views_grouped(n, d, nullptr);
  fpnmt_attn_desc gd[FPNMT_MAX_VIEWS];
  const void *gq[FPNMT_MAX_VIEWS], *gk[FPNMT_MAX_VIEWS], *gv[FPNMT_MAX_VIEWS], *gw[FPNMT_MAX_VIEWS],
      *gdo[FPNMT_MAX_VIEWS];
  void *gdq[FPNMT_MAX_VIEWS], *gdk[FPNMT_MAX_VIEWS], *gdv[FPNMT_MAX_VIEWS];
  int ng = 0;
  for (int i = 0; i < n; ++i) {
    const int e = attn_check(&d[i]);
    if (e) return e;
    if (view_empty(d[i])) continue;
    grouped = grouped && attn_q1_view_ok(&d[i], k[i], v[i], dq[i], dk[i], dv[i]) && q[i] && weights[i] && d_out[i];
    gd[ng] = d[i]; gq[ng] = q[i]; gk[ng] = k[i]; gv[ng] = v[i]; gw[ng] = weights[i]; gdo[ng] = d_out[i];
    gdq[ng] = dq[i]; gdk[ng] = dk[i]; gdv[ng] = dv[i];
    ++ng;
  }
  if (grouped && ng > 0) {
    const int e = attn_q1_views_bwd(ng, gd, gq, gk, gv, gw, gdo, gdq, gdk, gdv, S(stream));
    if (e) return e;
  }
  for (int i = 0; i < n; ++i) {
    if (grouped && ng > 0 && !view_empty(d[i])) continue;
    const int e = fpnmt_attention_bwd(&d[i], q[i], k[i], v[i], weights[i], d_out[i], dq[i], dk[i], dv[i], ws[i],
                                      stream);
    if (e) return e;
  }
  return 0;
}

int fpnmt_attention_bwd(const fpnmt_attn_desc* d, const void* q, const void* k, const void* v, const void* weights,
                        const void* d_out, void* dq, void* dk, void* dv, void* ws, fpnmt_stream_t stream) {
  int e = attn_check(d);
  if (e) return e;
  if (d->b == 0) return 0;
  hipStream_t s = S(stream);
  const int B = d->b, H = d->h, Lq = d->lq, Lk = d->lk, D = d->d;
  const long long ldw = d->ldw;
  const int V = d->dtype == FPNMT_BF16 ? 8 : 4;
  const size_t esz = d->dtype == FPNMT_BF16 ? 2 : 4;
  const long long rows = (long long)B * H * Lq;
  float* dP = (float*)ws;
  void* dS = (char*)ws + (((size_t)rows * ldw * 4 + 255) / 256) * 256;
  if (Lq == 0 || Lk == 0) {
    // no scores: dq = 0, dk/dv over empty key set or no queries -> zero
    // rows of all batches share one pitch (row b*L+i at base + (b*L+i)*ld): one 2D memset each
    if (Lq > 0 && zero_fill_2d(dq, d->ldq * esz, (size_t)H * D * esz, (size_t)B * Lq, s))
      return fail(FPNMT_E_HIP, "attention_bwd: zero dq");
    if (Lk > 0 && (zero_fill_2d(dk, d->ldk * esz, (size_t)H * D * esz, (size_t)B * Lk, s) ||
                   zero_fill_2d(dv, d->ldv * esz, (size_t)H * D * esz, (size_t)B * Lk, s)))
      return fail(FPNMT_E_HIP, "attention_bwd: zero dk/dv");
    return 0;
  }
  if (attn_q1_ok(d)) return attn_q1_bwd(d, q, k, v, weights, d_out, dq, dk, dv, s);
  if (attn_small_ok(d)) return attn_small_bwd(d, q, k, v, weights, d_out, dq, dk, dv, s);
  // 1) dP = dO V^T (fp32)
  {
    GemmParams p;
    init_params(p);
    p.M = Lq; p.N = Lk; p.K = D;
    p.A = d_out; p.B = v; p.C = dP;
    p.lda = d->ldo; p.ldb = d->ldv; p.ldc = ldw;
    p.batch_inner = H;
    p.a_so = (long long)Lq * d->ldo; p.a_si = D;
    p.b_so = (long long)Lk * d->ldv; p.b_si = D;
    p.c_so = (long long)H * Lq * ldw; p.c_si = (long long)Lq * ldw;
    p.c_f32 = 1;
    const bool vec = aligned16(d_out) && aligned16(v) && d->ldo % V == 0 && d->ldv % V == 0 && D % V == 0;
    e = run_gemm(d->dtype, p, B * H, A_ROW, B_NK, vec, s);
    if (e) return e;
  }
  // 2) dS = P (dP - rowsum(dP P))
  {
    const int grid = (int)((rows * 64 + 255) / 256);
    if (d->dtype == FPNMT_BF16)
      hipLaunchKernelGGL((attn_softmax_bwd_kernel<bf16>), dim3(grid), dim3(256), 0, s, rows, Lk,
                         (const bf16*)weights, dP, ldw, (bf16*)dS, ldw);
    else
      hipLaunchKernelGGL((attn_softmax_bwd_kernel<float>), dim3(grid), dim3(256), 0, s, rows, Lk,
                         (const float*)weights, dP, ldw, (float*)dS, ldw);
    e = check_launch("attn_softmax_bwd");
    if (e) return e;
  }
  const bool vws = aligned16(dS) && aligned16(weights);
  // 3) dQ = scale dS K
  {
    GemmParams p;
    init_params(p);
    p.M = Lq; p.N = D; p.K = Lk;
    p.A = dS; p.B = k; p.C = dq;
    p.lda = ldw; p.ldb = d->ldk; p.ldc = d->ldq;
    p.batch_inner = H;
    p.a_so = (long long)H * Lq * ldw; p.a_si = (long long)Lq * ldw;
    p.b_so = (long long)Lk * d->ldk; p.b_si = D;
    p.c_so = (long long)Lq * d->ldq; p.c_si = D;
    p.alpha = d->scale;
    const bool vec = vws && aligned16(k) && d->ldk % V == 0 && D % V == 0;
    e = run_gemm(d->dtype, p, B * H, A_ROW, B_KN, vec, s);
    if (e) return e;
  }
  // 4) dK = scale dS^T Q
  {
    GemmParams p;
    init_params(p);
    p.M = Lk; p.N = D; p.K = Lq;
    p.A = dS; p.B = q; p.C = dk;
    p.lda = ldw; p.ldb = d->ldq; p.ldc = d->ldk;
    p.batch_inner = H;
    p.a_so = (long long)H * Lq * ldw; p.a_si = (long long)Lq * ldw;
    p.b_so = (long long)Lq * d->ldq; p.b_si = D;
    p.c_so = (long long)Lk * d->ldk; p.c_si = D;
    p.alpha = d->scale;
    const bool vec = vws && aligned16(q) && d->ldq % V == 0 && D % V == 0;
    e = run_gemm(d->dtype, p, B * H, A_COL, B_KN, vec, s);
    if (e) return e;
  }
  // 5) dV = P^T dO
  {
    GemmParams p;
    init_params(p);
    p.M = Lk; p.N = D; p.K = Lq;
    p.A = weights; p.B = d_out; p.C = dv;
    p.lda = ldw; p.ldb = d->ldo; p.ldc = d->ldv;
    p.batch_inner = H;
    p.a_so = (long long)H * Lq * ldw; p.a_si = (long long)Lq * ldw;
    p.b_so = (long long)Lq * d->ldo; p.b_si = D;
    p.c_so = (long long)Lk * d->ldv; p.c_si = D;
    const bool vec = vws && aligned16(d_out) && d->ldo % V == 0 && D % V == 0;
    return run_gemm(d->dtype, p, B * H, A_COL, B_KN, vec, s);
  }
}

}  // extern "C"
