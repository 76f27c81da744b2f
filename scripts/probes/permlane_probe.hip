// Probe: v_permlane32_swap as an xor-32 lane exchange (inline asm with two distinct registers;
// the builtin with the same value in both operands gets them coalesced into one register).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ float xor32_sum(float v) {
  unsigned a = __builtin_bit_cast(unsigned, v), b = a;
  asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);
}
__global__ void k(float* a) {
  int i = threadIdx.x;
  a[i] = xor32_sum(a[i] * 1000.f) - a[i] * 1000.f;  // = partner * 1000
}
int main() {
  float h[64], *d;
  for (int i = 0; i < 64; ++i) h[i] = (float)i;
  hipMalloc(&d, sizeof(h)); hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) if (h[i] != (float)(i ^ 32) * 1000.f) { bad = 1; printf("lane %d got %g\n", i, h[i]); }
  printf(bad ? "MISMATCH\n" : "permlane32_swap xor-32 OK\n");
  return bad;
}
