// SwiGLU activation act = silu(gate) * up, forward and backward.
//
// Reference behaviour: transformers' LlamaMLP `down(act_fn(gate(x)) * up(x))` (eager
// silu + mul, two launches and an extra [T, F] round trip).  Here gate and up come from ONE fused
// GEMM whose output row is [gate(F) | up(F)]; the kernel reads both halves with 16-byte vectors
// and writes act, and the backward writes the fused [dgate | dup] row that feeds that GEMM's dX.
#include "common.h"

namespace lumen {

template <typename T, bool BWD>
__global__ void __launch_bounds__(256) swiglu_kernel(const T* __restrict__ gu,
                                                     const T* __restrict__ dact,
                                                     T* __restrict__ out, int rows, int F,
                                                     int c0, int nc) {
  // columns [c0, c0 + nc) of the F-wide activation (the whole row: c0 = 0, nc = F)
  const int vpr = nc / 8;  // vectors per row
  const long long tid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= static_cast<long long>(rows) * vpr) return;
  const int r = static_cast<int>(tid / vpr), c = c0 + static_cast<int>(tid % vpr) * 8;
  const T* g_p = gu + static_cast<size_t>(r) * 2 * F + c;
  float g[8], u[8];
  load8(g_p, g);
  load8(g_p + F, u);
  if (!BWD) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu(g[j]) * u[j];
    store8(out + static_cast<size_t>(r) * F + c, o);
  } else {
    float d[8], dg[8], du[8];
    load8(dact + static_cast<size_t>(r) * F + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-g[j]));
      const float sl = g[j] * sg;
      du[j] = d[j] * sl;
      dg[j] = d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    T* o = out + static_cast<size_t>(r) * 2 * F + c;
    store8(o, dg);
    store8(o + F, du);
  }
}

template <typename T>
static hipError_t launch(bool bwd, const void* gu, const void* dact, void* out, int rows, int F,
                         int c0, int nc, hipStream_t st) {
  const long long total = static_cast<long long>(rows) * (nc / 8);
  if (total == 0) return hipSuccess;
  dim3 grid(static_cast<unsigned>((total + 255) / 256)), block(256);
  if (bwd)
    hipLaunchKernelGGL((swiglu_kernel<T, true>), grid, block, 0, st, (const T*)gu,
                       (const T*)dact, (T*)out, rows, F, c0, nc);
  else
    hipLaunchKernelGGL((swiglu_kernel<T, false>), grid, block, 0, st, (const T*)gu, nullptr,
                       (T*)out, rows, F, c0, nc);
  return hipGetLastError();
}

}  // namespace lumen

// columns [c0, c1) of the activation only (c0 = 0, c1 = F: the whole row).  The column range
// lets the MLP run the activation of the columns a split gate|up GEMM (or down-projection dX)
// has already produced while the GEMM's last-wave tail computes the rest on a side stream.
extern "C" hipError_t lumen_swiglu(int dtype, int bwd, const void* gu, const void* dact, void* out,
                                   int rows, int F, int c0, int c1, hipStream_t st) {
  if (F % 8 != 0 || c0 % 8 != 0 || c1 % 8 != 0 || c0 < 0 || c1 > F || c0 > c1)
    return hipErrorInvalidValue;
  const int nc = c1 - c0;
  if (dtype == lumen::kBF16) return lumen::launch<lumen::bf16>(bwd, gu, dact, out, rows, F, c0, nc, st);
  if (dtype == lumen::kF16) return lumen::launch<lumen::fp16>(bwd, gu, dact, out, rows, F, c0, nc, st);
  if (dtype == lumen::kF32) return lumen::launch<float>(bwd, gu, dact, out, rows, F, c0, nc, st);
  return hipErrorInvalidValue;
}
