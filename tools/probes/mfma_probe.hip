#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
// A[32][16] row-major, B[16][32] row-major (k,n), C[32][32]
__global__ void k_bf16(const __bf16* A, const __bf16* B, float* C) {
  int l = threadIdx.x; int r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = A[r*16 + 8*h + j]; b[j] = B[(8*h+j)*32 + r]; }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int i = 0; i < 16; ++i) { int row = (i&3) + 8*(i>>2) + 4*h; C[row*32 + r] = acc[i]; }
}
__global__ void k_f32(const float* A, const float* B, float* C) {
  int l = threadIdx.x; int r = l & 31, h = l >> 5;
  f32x16 acc = {};
  for (int i = 0; i < 8; ++i) {
    float a = A[r*16 + 8*h + i]; float b = B[(8*h+i)*32 + r];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int i = 0; i < 16; ++i) { int row = (i&3) + 8*(i>>2) + 4*h; C[row*32 + r] = acc[i]; }
}
int main() {
  float hA[32*16], hB[16*32], ref[32*32];
  __bf16 bA[32*16], bB[16*32];
  for (int i = 0; i < 32*16; ++i) { hA[i] = (float)((i*7)%13 - 6); bA[i] = (__bf16)hA[i]; }
  for (int i = 0; i < 16*32; ++i) { hB[i] = (float)((i*5)%11 - 5); bB[i] = (__bf16)hB[i]; }
  for (int m = 0; m < 32; ++m) for (int n = 0; n < 32; ++n) { float s = 0; for (int k = 0; k < 16; ++k) s += hA[m*16+k]*hB[k*32+n]; ref[m*32+n] = s; }
  __bf16 *dA, *dB; float *fA, *fB, *dC; float hC[32*32];
  hipMalloc(&dA, sizeof bA); hipMalloc(&dB, sizeof bB); hipMalloc(&fA, sizeof hA); hipMalloc(&fB, sizeof hB); hipMalloc(&dC, sizeof hC);
  hipMemcpy(dA, bA, sizeof bA, hipMemcpyHostToDevice); hipMemcpy(dB, bB, sizeof bB, hipMemcpyHostToDevice);
  hipMemcpy(fA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(fB, hB, sizeof hB, hipMemcpyHostToDevice);
  k_bf16<<<1,64>>>(dA, dB, dC); hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  double e = 0; for (int i = 0; i < 1024; ++i) e = fmax(e, fabs(hC[i]-ref[i])); printf("bf16 maxerr %g\n", e);
  k_f32<<<1,64>>>(fA, fB, dC); hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  e = 0; for (int i = 0; i < 1024; ++i) e = fmax(e, fabs(hC[i]-ref[i])); printf("f32 maxerr %g\n", e);
  return 0;
}
