// Pure HBM read stream ceiling on this chip (is the paged decode at 6.35 TB/s near it?).
// Each thread reads UNROLL 16-byte pieces per iteration (plain or non-temporal), grid-stride over
// a 4 GiB buffer (> the 256 MB Infinity Cache), and folds them into one word so the loads stay.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_read scripts/probes/hbm_read_probe.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) read_kernel(const u32x4* __restrict__ p, size_t n,
                                                   unsigned* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x * UNROLL;
  size_t i = (size_t)blockIdx.x * blockDim.x * UNROLL + threadIdx.x;
  unsigned acc = 0;
  for (; i + (UNROLL - 1) * blockDim.x < n; i += stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      v[u] = NT ? __builtin_nontemporal_load(p + i + u * blockDim.x) : p[i + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int UNROLL, bool NT>
static void run(const u32x4* p, size_t n, unsigned* out, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) read_kernel<UNROLL, NT><<<blocks, 256>>>(p, n, out);
  hipEventRecord(a);
  const int it = 10;
  for (int w = 0; w < it; ++w) read_kernel<UNROLL, NT><<<blocks, 256>>>(p, n, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)n * 16;
  printf("{\"unroll\": %d, \"nt\": %d, \"blocks\": %d, \"TBps\": %.3f}\n", UNROLL, (int)NT, blocks,
         bytes * it / (ms * 1e-3) / 1e12);
}

int main() {
  const size_t bytes = 4ull << 30;
  const size_t n = bytes / 16;
  u32x4* p;
  unsigned* out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(p, 1, bytes);
  hipDeviceSynchronize();
  for (int blocks : {1024, 2048, 4096, 8192}) {
    run<4, false>(p, n, out, blocks);
    run<4, true>(p, n, out, blocks);
    run<8, false>(p, n, out, blocks);
    run<8, true>(p, n, out, blocks);
  }
  hipFree(p);
  hipFree(out);
  return 0;
}
