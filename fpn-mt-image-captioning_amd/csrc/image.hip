// Input pipeline (reference dataset.py:19-26 load_image):
//   img = tf.image.resize(decode_jpeg(file, channels=3), (S, S))   # bilinear
//   img = mobilenet_v2.preprocess_input(img)                       # x/127.5 - 1
// for a whole batch of decoded, ragged-size uint8 RGB images in ONE launch,
// writing the NHWC fp32 / bf16 model input directly.
//
// TF2 tf.image.resize (ResizeBilinear, half_pixel_centers=True,
// align_corners=False, antialias=False), per output coordinate i of an axis:
//   scale = float(in_size) / float(out_size)
//   in    = (float(i) + 0.5f) * scale - 0.5f
//   lower = max(int(floor(in)), 0), upper = min(int(ceil(in)), in_size - 1)
//   lerp  = in - floor(in)
//   top = tl + (tr - tl) * xlerp; bottom = bl + (br - bl) * xlerp
//   out = top + (bottom - top) * ylerp
// in fp32 with every multiply and add rounded separately (no FMA
// contraction: the pragma below), so the result is bit-identical to the
// restatement in oracle/image_ref.py. Then out / div - sub (an IEEE divide,
// as the Keras preprocessing's `x /= 127.5`, not a reciprocal multiply).
//
// One 256-thread block per (image, output row): the two source rows the row
// interpolates between are staged in LDS with coalesced dword loads (the
// decoded rows are byte-packed, 3 B per pixel, so a row starts at any byte;
// the staging window starts at the dword below), then each thread produces
// output pixels from LDS. Rows wider than the LDS window read global memory
// directly. HBM-bound: the output (12 B / pixel fp32) dominates.
#include "common.h"

namespace fpnmt {
namespace {

constexpr int IMG_THREADS = 256;
constexpr int IMG_LDS_MAX = 64 * 1024;  // dynamic LDS per block for the two staged rows

struct Axis {
  int lo, hi;
  float lerp;
};

__device__ __forceinline__ Axis axis_weights(int i, float scale, int in_size) {
#pragma clang fp contract(off)
  const float in = ((float)i + 0.5f) * scale - 0.5f;
  const float f = floorf(in);
  Axis a;
  a.lo = max((int)f, 0);
  a.hi = min((int)ceilf(in), in_size - 1);
  a.lerp = in - f;
  return a;
}

__device__ __forceinline__ float lerp2(float tl, float tr, float bl, float br, float xl, float yl) {
#pragma clang fp contract(off)
  const float top = tl + (tr - tl) * xl;
  const float bottom = bl + (br - bl) * xl;
  return top + (bottom - top) * yl;
}

// bytes [start, start + len) of the packed buffer into LDS in 16-B pieces,
// from the 16-B boundary at or below `start` (the packed buffer is 16-B
// aligned); returns the byte shift of `start` inside the window
__device__ __forceinline__ int stage_row(uint32_t* lds, const uint8_t* px, long long px_bytes, long long start,
                                         int len) {
  const long long base = start & ~15LL;
  const int nq = (int)((start + len - base + 15) >> 4);
  const uint4* g = (const uint4*)(px + base);
  for (int i = threadIdx.x; i < nq; i += IMG_THREADS) {
    const long long b = base + 16LL * i;
    uint4 v;
    if (b + 15 < px_bytes) {
      v = g[i];
    } else {  // the buffer's last partial piece: byte loads
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      for (int k = 0; k < 16; ++k)
        if (b + k < px_bytes) w[k >> 2] |= (uint32_t)px[b + k] << (8 * (k & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *(uint4*)(lds + 4 * i) = v;
  }
  return (int)(start - base);
}

// LDS words of one staged row window: the row's bytes + up to 15 leading
// bytes, rounded up to whole 16-B pieces
__host__ __device__ __forceinline__ int row_window_words(int row_bytes) { return ((row_bytes + 30) / 16) * 4; }

// One 256-thread block per (image, RB consecutive output rows): the 2*RB
// source rows are staged in LDS with coalesced dword loads, then the block
// writes the RB output rows as runs of 4 consecutive values (one 16-B fp32 /
// 8-B bf16 store per thread per run; a value's pixel and channel are v / 3,
// v % 3), so a block issues ~170 wide stores per row instead of 672 scalar
// ones and a grid of 56 blocks per 224-row image instead of 224.
template <typename T, int RB, bool USE_LDS>
__global__ __launch_bounds__(IMG_THREADS) void resize_normalize_kernel(const fpnmt_image_item* __restrict__ items,
                                                                        const uint8_t* __restrict__ px,
                                                                        long long px_bytes, int row_words,
                                                                        int out_h, int out_w, float div, float sub,
                                                                        T* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ uint32_t lds[];
  const int y0 = blockIdx.x * RB, img = blockIdx.y;
  const fpnmt_image_item it = items[img];
  const int rv = out_w * 3;  // values per output row
  if (it.h <= 0 || it.w <= 0) {  // the host loader rejects empty images; keep the output defined
    for (int r = 0; r < RB && y0 + r < out_h; ++r) {
      T* orow = out + ((long long)img * out_h + y0 + r) * rv;
      for (int x = threadIdx.x; x < rv; x += IMG_THREADS) orow[x] = from_f32<T>(0.f);
    }
    return;
  }
  const int rb = it.w * 3;
  const float yscale = (float)it.h / (float)out_h, xscale = (float)it.w / (float)out_w;
  const uint8_t* top[RB];
  const uint8_t* bot[RB];
  float ylerp[RB];
  const bool staged = USE_LDS && row_window_words(rb) <= row_words;
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const Axis ya = axis_weights(min(y0 + r, out_h - 1), yscale, it.h);
    ylerp[r] = ya.lerp;
    if (staged) {
      // (the item's row fits the window sized for max_w; a wider row than
      // the caller declared reads global memory instead of overrunning LDS)
      uint32_t* l0 = lds + (2 * r) * row_words;
      uint32_t* l1 = lds + (2 * r + 1) * row_words;
      const int s0 = stage_row(l0, px, px_bytes, it.offset + (long long)ya.lo * rb, rb);
      const int s1 = stage_row(l1, px, px_bytes, it.offset + (long long)ya.hi * rb, rb);
      top[r] = (const uint8_t*)l0 + s0;
      bot[r] = (const uint8_t*)l1 + s1;
    } else {
      top[r] = px + it.offset + (long long)ya.lo * rb;
      bot[r] = px + it.offset + (long long)ya.hi * rb;
    }
  }
  if (staged) __syncthreads();
  auto value = [&](int r, int v) {
    const int x = v / 3, ch = v - 3 * x;
    const Axis xa = axis_weights(x, xscale, it.w);
    const int a = xa.lo * 3 + ch, b = xa.hi * 3 + ch;
    const float f = lerp2((float)top[r][a], (float)top[r][b], (float)bot[r][a], (float)bot[r][b], xa.lerp, ylerp[r]);
    return f / div - sub;
  };
  const bool vec = (rv & 3) == 0;  // every row starts 4-value aligned
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    if (y0 + r >= out_h) break;
    T* orow = out + ((long long)img * out_h + y0 + r) * rv;
    if (vec) {
      typedef __attribute__((ext_vector_type(4))) T T4;
      for (int q = threadIdx.x; q < (rv >> 2); q += IMG_THREADS) {
        T4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = from_f32<T>(value(r, 4 * q + j));
        *(T4*)(orow + 4 * q) = o;
      }
    } else {
      for (int v = threadIdx.x; v < rv; v += IMG_THREADS) orow[v] = from_f32<T>(value(r, v));
    }
  }
}

template <typename T>
void resize_launch(const fpnmt_image_item* items, int n, const uint8_t* px, long long px_bytes, int max_w, int out_h,
                   int out_w, float div, float sub, void* out, hipStream_t s) {
  constexpr int RB = 4;
  const int row_words = row_window_words(max_w * 3);
  const size_t lds4 = 2ull * RB * row_words * 4, lds1 = 2ull * row_words * 4;
  const bool aligned = ((uintptr_t)px & 15) == 0;  // the staging reads 16-B pieces of the packed buffer
  if (aligned && lds4 <= (size_t)IMG_LDS_MAX)
    resize_normalize_kernel<T, RB, true><<<dim3(cdiv(out_h, RB), n), IMG_THREADS, lds4, s>>>(
        items, px, px_bytes, row_words, out_h, out_w, div, sub, (T*)out);
  else if (aligned && lds1 <= (size_t)IMG_LDS_MAX)
    resize_normalize_kernel<T, 1, true><<<dim3(out_h, n), IMG_THREADS, lds1, s>>>(items, px, px_bytes, row_words,
                                                                                   out_h, out_w, div, sub, (T*)out);
  else
    resize_normalize_kernel<T, 1, false><<<dim3(out_h, n), IMG_THREADS, 0, s>>>(items, px, px_bytes, 0, out_h, out_w,
                                                                                div, sub, (T*)out);
}

}  // namespace
}  // namespace fpnmt

using namespace fpnmt;

extern "C" {

int fpnmt_image_resize_normalize(const fpnmt_image_item* items_dev, int n, const uint8_t* pixels,
                                 long long pixel_bytes, int max_w, int out_h, int out_w, float div, float sub,
                                 int dtype, void* out, fpnmt_stream_t stream) {
  if (dtype != FPNMT_BF16 && dtype != FPNMT_F32) return fail(FPNMT_E_ARG, "image_resize_normalize: bad dtype");
  if (n < 0 || out_h <= 0 || out_w <= 0 || max_w <= 0 || pixel_bytes < 0)
    return fail(FPNMT_E_ARG, "image_resize_normalize: bad sizes");
  if (out_h > 65535 || n > 65535) return fail(FPNMT_E_UNSUPPORTED, "image_resize_normalize: grid too large");
  if (!(div != 0.f)) return fail(FPNMT_E_ARG, "image_resize_normalize: div must be non-zero");
  if (n == 0) return 0;
  if (!items_dev || !pixels || !out) return fail(FPNMT_E_ARG, "image_resize_normalize: null pointer");
  if (dtype == FPNMT_BF16)
    resize_launch<bf16>(items_dev, n, pixels, pixel_bytes, max_w, out_h, out_w, div, sub, out, (hipStream_t)stream);
  else
    resize_launch<float>(items_dev, n, pixels, pixel_bytes, max_w, out_h, out_w, div, sub, out, (hipStream_t)stream);
  return check_launch("image_resize_normalize");
}

}  // extern "C"
