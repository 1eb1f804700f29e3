// Checks the operand / result lane maps this repo assumes for the bf16 MFMAs
// (kernels/lstm_mb.hip) against a CPU product: A[16 x K] B[K x 16] with small
// integers (exact in bf16 and fp32).
//   16x16x32 bf16: lane l holds A[l & 15][8 (l >> 4) + j], B[8 (l >> 4) + j][l & 15]
//   16x16x16 bf16_1k: lane l holds A[l & 15][4 (l >> 4) + j], B[4 (l >> 4) + j][l & 15]
//   C: lane l, register r = C[4 (l >> 4) + r][l & 15]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ uint16_t bf(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }

__global__ void k32(const float* A, const float* B, float* C) {  // A [16][32], B [32][16]
  const int l = threadIdx.x;
  uint16_t a[8], b[8];
  for (int j = 0; j < 8; ++j) {
    a[j] = bf(A[(l & 15) * 32 + 8 * (l >> 4) + j]);
    b[j] = bf(B[(8 * (l >> 4) + j) * 16 + (l & 15)]);
  }
  bf16x8 av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}
__global__ void k16(const float* A, const float* B, float* C) {  // A [16][16], B [16][16]
  const int l = threadIdx.x;
  uint16_t a[4], b[4];
  for (int j = 0; j < 4; ++j) {
    a[j] = bf(A[(l & 15) * 16 + 4 * (l >> 4) + j]);
    b[j] = bf(B[(4 * (l >> 4) + j) * 16 + (l & 15)]);
  }
  s16x4 av, bv;
  __builtin_memcpy(&av, a, 8);
  __builtin_memcpy(&bv, b, 8);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

static int check(int K, bool big) {
  std::vector<float> A(16 * K), B(K * 16), C(256), R(256, 0.f);
  for (int i = 0; i < 16 * K; ++i) A[i] = (float)((i * 7 + 3) % 9 - 4);
  for (int i = 0; i < K * 16; ++i) B[i] = (float)((i * 5 + 1) % 7 - 3);
  for (int i = 0; i < 16; ++i)
    for (int n = 0; n < 16; ++n)
      for (int k = 0; k < K; ++k) R[i * 16 + n] += A[i * K + k] * B[k * 16 + n];
  float *dA, *dB, *dC;
  (void)hipMalloc(&dA, A.size() * 4); (void)hipMalloc(&dB, B.size() * 4); (void)hipMalloc(&dC, 1024);
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  if (big) hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  else hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += C[i] != R[i];
  printf("16x16x%d bf16: %d of 256 results differ (C[0] %g ref %g)\n", K, bad, C[0], R[0]);
  return bad;
}

int main() { return (check(32, true) + check(16, false)) ? 1 : 0; }
