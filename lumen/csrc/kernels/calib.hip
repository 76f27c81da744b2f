// Fixed-work box calibration (bench.py extra.box; VERDICT r5 "Next" #3): a non-temporal HBM read
// stream over a buffer far larger than the 256 MB Infinity Cache, timed next to every bench record
// so a slow record can be told apart from a slow box (same process, same lease).  The loop is
// scripts/probes/hbm_read_probe.cpp's: 16-byte non-temporal loads, 8 in flight per lane,
// grid-stride, folded into one word so the loads stay.
#include "common.h"

namespace lumen {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) hbm_read_kernel(const u32x4* __restrict__ p, long long n,
                                                       unsigned* __restrict__ out) {
  constexpr int U = 8;
  const long long stride = (long long)gridDim.x * 256 * U;
  long long i = (long long)blockIdx.x * 256 * U + threadIdx.x;
  unsigned acc = 0;
  for (; i + (U - 1) * 256 < n; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

}  // namespace lumen

// reads `bytes` (a multiple of 16 * 8 * 256 * blocks) from p; returns after the launch
extern "C" hipError_t lumen_hbm_read(const void* p, long long bytes, unsigned* out, int blocks,
                                     hipStream_t st) {
  if (p == nullptr || out == nullptr || blocks < 1 || bytes <= 0 ||
      bytes % (16LL * 8 * 256 * blocks) != 0 || (reinterpret_cast<uintptr_t>(p) & 15) != 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(lumen::hbm_read_kernel, dim3(blocks), dim3(256), 0, st,
                     reinterpret_cast<const lumen::u32x4*>(p), bytes / 16, out);
  return hipGetLastError();
}
