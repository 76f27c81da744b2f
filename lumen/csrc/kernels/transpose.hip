// 2-D transpose of a 16-bit matrix through LDS (out[c][r] = in[r][c]).
//
// Used for the transposed frozen-weight copies that turn the input-gradient GEMM dY @ W into the
// faster TN form (lumen/models/layers.py, Linear.weight_t_fn): persistent weights are transposed
// once, ZeRO-3-gathered ones on the fly each step, so this has to run at HBM speed -- torch's
// strided copy reaches ~0.5 TB/s on these shapes.  Tile = 64 x 64 elements: 16-byte global loads
// along the input rows, an LDS tile padded by one 16-bit element per row so that the transposed
// reads of 8 rows x 1 column hit distinct banks, and 16-byte global stores along output rows.
#include "common.h"

namespace lumen {

template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                        int R, int C, long long ldi, long long ldo) {
  constexpr int TS = 64, LD = TS + 2;
  __shared__ T tile[TS * LD];
  const int r0 = blockIdx.y * TS, c0 = blockIdx.x * TS;
  // load: 64 rows x 8 chunks of 8 columns, 2 chunks per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int rr = idx >> 3, cc = (idx & 7) * 8;
    const int r = r0 + rr, c = c0 + cc;
    Vec8<T> v;
    if (r < R && c + 7 < C) {
      v = *reinterpret_cast<const Vec8<T>*>(in + (long long)r * ldi + c);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v.v[j] = (r < R && c + j < C) ? in[(long long)r * ldi + c + j] : T();
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[rr * LD + cc + j] = v.v[j];
  }
  __syncthreads();
  // store: output rows = input columns; 64 x 8 chunks of 8 (input rows), 2 per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int oc = idx >> 3, orr = (idx & 7) * 8;   // output row (= input col), input row chunk
    const int c = c0 + oc, r = r0 + orr;
    if (c >= C) continue;
    Vec8<T> v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.v[j] = tile[(orr + j) * LD + oc];
    if (r + 7 < R) {
      *reinterpret_cast<Vec8<T>*>(out + (long long)c * ldo + r) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (r + j < R) out[(long long)c * ldo + r + j] = v.v[j];
    }
  }
}

}  // namespace lumen

// in [R][ldi] -> out [C][ldo]; 16-byte alignment of rows is required for the vector path
// (ldi, ldo multiples of 8), tails are handled element-wise.
extern "C" hipError_t lumen_transpose(int dtype, const void* in, void* out, int R, int C,
                                      long long ldi, long long ldo, hipStream_t st) {
  if (R <= 0 || C <= 0) return hipSuccess;
  if ((ldi & 7) || (ldo & 7)) return hipErrorInvalidValue;
  dim3 grid((C + 63) / 64, (R + 63) / 64), block(256);
  if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::transpose_kernel<lumen::bf16>, grid, block, 0, st,
                       static_cast<const lumen::bf16*>(in), static_cast<lumen::bf16*>(out), R, C, ldi, ldo);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::transpose_kernel<lumen::fp16>, grid, block, 0, st,
                       static_cast<const lumen::fp16*>(in), static_cast<lumen::fp16*>(out), R, C, ldi, ldo);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
