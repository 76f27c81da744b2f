// Token sampling: greedy / temperature / top-k / top-p in one kernel.
//
// Reference behaviour: vLLM 0.6.0's Sampler (declared serving stack, requirements.txt:17-18):
// temperature scaling, sort-based top-k/top-p masking, softmax, multinomial draw.
//
// Sort-free formulation, one 512-thread workgroup per row (logits row stays L2-resident):
//   z = logit / T;  m = max z;  Z = sum exp(z - m)
//   top-k:  tau_k = largest threshold with count(z >= tau_k) >= k    (bisection on the value)
//   top-p:  tau_p = largest threshold with mass(z >= tau_p) >= p     (bisection on the value)
//   token = argmax_{z_j >= max(tau_k, tau_p)} z_j + Gumbel(hash(seed, offset, row, j))
// Gumbel-max over the kept set is an exact draw from the renormalised truncated distribution.
// temperature == 0 -> greedy argmax.  Also returns the chosen token's log-prob under the
// temperature-scaled (untruncated) distribution.
#include "common.h"

namespace lumen {

constexpr int kSampNT = 512;

template <typename T>
__device__ __forceinline__ float ld_logit(const T* row, int j, float invT) {
  return to_f32(row[j]) * invT;
}

template <typename T>
__global__ void __launch_bounds__(kSampNT) sample_kernel(
    const T* __restrict__ logits, const float* __restrict__ temperature,
    const float* __restrict__ top_p, const int* __restrict__ top_k, unsigned long long seed,
    long long offset, long long* __restrict__ out_tok, float* __restrict__ out_lp, int V) {
  __shared__ float red[kSampNT / 64];
  __shared__ int redi[kSampNT / 64];
  const int row = blockIdx.x;
  const T* lr = logits + static_cast<size_t>(row) * V;
  const float temp = temperature[row];
  const bool greedy = !(temp > 0.f);
  const float invT = greedy ? 1.f : 1.f / temp;
  // max
  float m = -INFINITY;
  for (int j = threadIdx.x; j < V; j += kSampNT) m = fmaxf(m, ld_logit(lr, j, invT));
  m = block_max<kSampNT>(m, red);
  float s = 0.f;
  for (int j = threadIdx.x; j < V; j += kSampNT) s += __expf(ld_logit(lr, j, invT) - m);
  const float Z = block_sum<kSampNT>(s, red);
  float tau = -INFINITY;
  if (!greedy) {
    const int k = top_k[row];
    if (k > 0 && k < V) {
      float lo = m - 80.f, hi = m;  // count(z >= lo) >= k assumed (exp underflow region)
      for (int it = 0; it < 30; ++it) {
        const float mid = 0.5f * (lo + hi);
        float c = 0.f;
        for (int j = threadIdx.x; j < V; j += kSampNT) c += ld_logit(lr, j, invT) >= mid ? 1.f : 0.f;
        c = block_sum<kSampNT>(c, red);
        if (c >= static_cast<float>(k)) lo = mid; else hi = mid;
      }
      tau = lo;
    }
    const float p = top_p[row];
    if (p < 1.f) {
      float lo = m - 80.f, hi = m;
      for (int it = 0; it < 30; ++it) {
        const float mid = 0.5f * (lo + hi);
        float c = 0.f;
        for (int j = threadIdx.x; j < V; j += kSampNT) {
          const float z = ld_logit(lr, j, invT);
          c += z >= mid ? __expf(z - m) : 0.f;
        }
        c = block_sum<kSampNT>(c, red) / Z;
        if (c >= p) lo = mid; else hi = mid;
      }
      tau = fmaxf(tau, lo);
    }
  }
  // argmax over kept set (with Gumbel noise unless greedy)
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = threadIdx.x; j < V; j += kSampNT) {
    const float z = ld_logit(lr, j, invT);
    if (z < tau) continue;
    float key = z;
    if (!greedy) {
      const uint32_t sd = static_cast<uint32_t>(seed) ^
                          (static_cast<uint32_t>(offset) * 0x9E3779B9u + 0x7F4A7C15u);
      const uint32_t r = rng_u32(sd, static_cast<uint64_t>(row) * static_cast<uint64_t>(V) + j);
      const float u = (static_cast<float>(r >> 8) + 0.5f) * (1.f / 16777216.f);
      key = z - __logf(-__logf(u));
    }
    if (key > best || (key == best && j < bi)) { best = key; bi = j; }
  }
  // block argmax
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[wid] = best; redi[wid] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = red[0];
    int idx = redi[0];
    for (int w = 1; w < kSampNT / 64; ++w)
      if (red[w] > b || (red[w] == b && redi[w] < idx)) { b = red[w]; idx = redi[w]; }
    if (idx >= V) idx = 0;
    out_tok[row] = idx;
    if (out_lp) out_lp[row] = ld_logit(lr, idx, invT) - m - __logf(Z);
  }
}

}  // namespace lumen

extern "C" hipError_t lumen_sample(int dtype, const void* logits, const float* temperature,
                                   const float* top_p, const int* top_k, unsigned long long seed,
                                   long long offset, long long* out_tok, float* out_lp, int rows,
                                   int V, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  dim3 grid(rows), block(lumen::kSampNT);
  if (dtype == lumen::kF32)
    hipLaunchKernelGGL(lumen::sample_kernel<float>, grid, block, 0, st, (const float*)logits,
                       temperature, top_p, top_k, seed, offset, out_tok, out_lp, V);
  else if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::sample_kernel<lumen::bf16>, grid, block, 0, st,
                       (const lumen::bf16*)logits, temperature, top_p, top_k, seed, offset,
                       out_tok, out_lp, V);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::sample_kernel<lumen::fp16>, grid, block, 0, st,
                       (const lumen::fp16*)logits, temperature, top_p, top_k, seed, offset,
                       out_tok, out_lp, V);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
