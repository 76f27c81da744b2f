// Fused softmax cross-entropy forward + backward.
//
// Reference behaviour: transformers' causal-LM loss -- logits `.float()` (a [T, V] f32 copy)
// then `CrossEntropyLoss(ignore_index=-100)` over shifted labels, i.e. log-softmax, gather, mean
// over non-ignored tokens, then a separate softmax-minus-onehot backward.
//
// Here one workgroup per row makes two passes over the 16-bit logits: pass 1 = online max/sum
// (f32, one running pair per lane, merged across the block), pass 2 = write the gradient
// (softmax - onehot) * scale IN PLACE over the logits (the logits are dead after the loss), so
// the [T, V] f32 copy and the separate backward launch disappear.  `scale` is 1/num_valid_tokens
// (known on the host from the collated labels); the upstream grad scalar is applied later to the
// [T, H] result of the LM-head dX GEMM, which is 8x smaller than the logits.
// fp16 with dynamic loss scaling: `gscale` (device f32, optional) multiplies the written gradient
// by the CURRENT loss scale, as the reference's upcast-logits graph does ((p - y) * S / n reaches
// the fp16 LM-head GEMM already scaled); without it p / n underflows fp16 for most of the vocab.
#include "common.h"

namespace lumen {

template <typename T, int NT>
__global__ void __launch_bounds__(NT) xent_kernel(T* __restrict__ logits, const int64_t* labels,
                                                  float* __restrict__ loss_sum,
                                                  float* __restrict__ row_loss, int V,
                                                  int ignore_index, float scale, int write_grad,
                                                  const float* __restrict__ gscale) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  T* lr = logits + static_cast<size_t>(row) * V;
  const int nvec = V / 8;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < nvec; i += NT) {
    float x[8];
    load8(lr + i * 8, x);
    float mx = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mx = fmaxf(mx, x[j]);
    const float mn = fmaxf(m, mx);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(x[j] - mn);
    m = mn;
    s = acc;
  }
  const float gm = block_max<NT>(m, red);
  const float gs = block_sum<NT>(s * (m == -INFINITY ? 0.f : __expf(m - gm)), red);
  const float lse = gm + __logf(gs);
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  if (threadIdx.x == 0) {
    float l = 0.f;
    if (valid) l = lse - to_f32(lr[lab]);
    if (row_loss) row_loss[row] = l;
    if (loss_sum && valid) atomicAdd(loss_sum, l);
  }
  if (!write_grad) return;
  __syncthreads();  // everyone has read lr[lab] before it is overwritten
  const float sc = valid ? scale * (gscale ? *gscale : 1.f) : 0.f;
  for (int i = threadIdx.x; i < nvec; i += NT) {
    float x[8];
    load8(lr + i * 8, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(x[j] - lse);
      if (i * 8 + j == lab) p -= 1.f;
      x[j] = p * sc;
    }
    store8(lr + i * 8, x);
  }
}

// x *= num[0] / den[0] (den optional), f32 math on 16-bit rows, 16 bytes per thread: the LM
// head's dH times the upstream device scalar (as torch's mixed-dtype in-place mul it ran the
// generic unrolled elementwise kernel: 53 us for 32 MiB at Llama-2-7B's 8 x 512 tokens)
template <typename T>
__global__ void __launch_bounds__(256) scale_dev_kernel(T* __restrict__ x, long long n8,
                                                        const float* __restrict__ num,
                                                        const float* __restrict__ den) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  const float s = den ? num[0] / den[0] : num[0];
  float v[8];
  load8(x + i * 8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= s;
  store8(x + i * 8, v);
}

}  // namespace lumen

extern "C" hipError_t lumen_scale_dev(int dtype, void* x, long long n, const float* num,
                                      const float* den, hipStream_t st) {
  if (n % 8 != 0) return hipErrorInvalidValue;
  const long long n8 = n / 8;
  if (n8 == 0) return hipSuccess;
  dim3 grid(static_cast<unsigned>((n8 + 255) / 256)), block(256);
  if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::scale_dev_kernel<lumen::bf16>, grid, block, 0, st, (lumen::bf16*)x, n8, num, den);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::scale_dev_kernel<lumen::fp16>, grid, block, 0, st, (lumen::fp16*)x, n8, num, den);
  else if (dtype == lumen::kF32)
    hipLaunchKernelGGL(lumen::scale_dev_kernel<float>, grid, block, 0, st, (float*)x, n8, num, den);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t lumen_cross_entropy(int dtype, void* logits, const int64_t* labels,
                                          float* loss_sum, float* row_loss, int rows, int V,
                                          int ignore_index, float scale, int write_grad,
                                          const float* gscale, hipStream_t st) {
  if (V % 8 != 0) return hipErrorInvalidValue;
  if (rows == 0) return hipSuccess;
  dim3 grid(rows), block(512);
  if (dtype == lumen::kBF16)
    hipLaunchKernelGGL((lumen::xent_kernel<lumen::bf16, 512>), grid, block, 0, st,
                       (lumen::bf16*)logits, labels, loss_sum, row_loss, V, ignore_index, scale,
                       write_grad, gscale);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL((lumen::xent_kernel<lumen::fp16, 512>), grid, block, 0, st,
                       (lumen::fp16*)logits, labels, loss_sum, row_loss, V, ignore_index, scale,
                       write_grad, gscale);
  else if (dtype == lumen::kF32)
    hipLaunchKernelGGL((lumen::xent_kernel<float, 512>), grid, block, 0, st, (float*)logits,
                       labels, loss_sum, row_loss, V, ignore_index, scale, write_grad, gscale);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
