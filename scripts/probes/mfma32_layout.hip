// Probe: operand / accumulator layout of v_mfma_f32_32x32x16_bf16 on gfx950.
// A[32][16], B[16][32] random; lane l supplies A[l%32][8*(l/32)+e], B[8*(l/32)+e][l%32];
// checks C[row][col] with row = 8*(r/4) + 4*(l/32) + r%4, col = l%32 against a host reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const __bf16* A, const __bf16* B, float* C) {
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = A[(l % 32) * 16 + 8 * (l / 32) + e];
    b[e] = B[(8 * (l / 32) + e) * 32 + (l % 32)];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) C[(8 * (r / 4) + 4 * (l / 32) + r % 4) * 32 + (l % 32)] = c[r];
}

int main() {
  std::vector<__bf16> A(512), B(512);
  std::vector<float> Af(512), Bf(512), C(1024), R(1024, 0.f);
  for (int i = 0; i < 512; ++i) {
    Af[i] = (float)((i * 37 % 17) - 8) / 8.f; A[i] = (__bf16)Af[i];
    Bf[i] = (float)((i * 11 % 13) - 6) / 4.f; B[i] = (__bf16)Bf[i];
  }
  for (int m = 0; m < 32; ++m) for (int n = 0; n < 32; ++n) for (int kk = 0; kk < 16; ++kk)
    R[m * 32 + n] += Af[m * 16 + kk] * Bf[kk * 32 + n];
  __bf16 *dA, *dB; float* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
  hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < 1024; ++i) err = fmax(err, fabs(C[i] - R[i]));
  printf("mfma32x32x16 layout max err %g -> %s\n", err, err < 1e-3 ? "OK" : "MISMATCH");
  return err < 1e-3 ? 0 : 1;
}
