// Token sampling: greedy / temperature / top-k / top-p in one kernel.
//
// Reference behaviour: vLLM 0.6.0's Sampler (the declared serving stack, requirements.txt:17-18),
// `_apply_top_k_top_p`: temperature scaling; top-k keeps every logit >= the k-th largest VALUE
// (ties kept); top-p then works on the softmax of the top-k-truncated logits and keeps the
// smallest head of the sorted distribution whose mass reaches p (at least one token); softmax,
// multinomial draw.
//
// Sort-free, one 512-thread workgroup per row, the row's scaled logits z cached in LDS
// (V <= 32768; larger vocabularies re-read the L2-resident row every pass):
//   keys: the f32 bits of z mapped to an order-preserving uint32
//   top-k: tau_k = the k-th largest key, by RADIX SELECT -- four 8-bit digit levels, each one
//          pass building a 256-bin count histogram of the keys under the prefix fixed so far,
//          then one wave's parallel suffix scan picks the digit (exact, 4 passes instead of the
//          previous 30-step bisection over the values)
//   top-p: fixed-point masses W = exp(z - m) * 2^32 (integer sums: order-independent, so the
//          kept set is deterministic); target = p * sum(W over key >= tau_k); tau_p = the largest
//          key whose suffix mass reaches the target, by the same radix select on mass histograms
//   token = argmax over key >= max(tau_k, tau_p) of z + Gumbel(hash(seed, offset, row, j)):
//          an exact draw from the renormalised truncated distribution
// temperature == 0 -> greedy argmax.  Also returns the chosen token's log-prob under the
// temperature-scaled (untruncated) distribution, and optionally the kept threshold (as a
// value of z) for tests.
#include "common.h"

namespace lumen {

constexpr int kSampNT = 512;

__device__ __forceinline__ uint32_t fkey(float z) {
  const uint32_t u = __float_as_uint(z);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float keyf(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// NPT = 1: the row's scaled logits cached in LDS (V <= kSampLdsV); NPT = 0: re-read from the
// (L2-resident) logits every pass
constexpr int kSampLdsV = 32768;

template <typename T, int NPT>
struct Row {
  const float* zl;  // LDS copy (NPT = 1)
  const T* p;
  int V;
  float invT;
  __device__ __forceinline__ float ld(int j) const { return to_f32(p[j]) * invT; }
  // f(j, z) for every element this thread owns, 8 at a time: the 8 loads are issued before any
  // f runs (f's LDS histogram atomics would otherwise order each load behind the previous
  // element's atomic -- one LDS / L2 round trip per element, ~7 us per pass over V = 32000)
  template <typename F>
  __device__ __forceinline__ void each(F&& f) const {
    constexpr int U = 8;
    int j0 = threadIdx.x;
    // full batches: no per-element bounds test (each one cost an exec-mask branch)
    for (; j0 + (U - 1) * kSampNT < V; j0 += U * kSampNT) {
      float zz[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (NPT > 0) zz[u] = zl[j0 + u * kSampNT];
        else zz[u] = ld(j0 + u * kSampNT);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) f(j0 + u * kSampNT, zz[u]);
    }
    for (; j0 < V; j0 += U * kSampNT) {
      float zz[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * kSampNT;
        const int jc = j < V ? j : V - 1;  // clamped: unconditional loads
        if constexpr (NPT > 0) zz[u] = zl[jc];
        else zz[u] = ld(jc);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * kSampNT;
        if (j < V) f(j, zz[u]);
      }
    }
  }
};

// Wave 0 picks the digit: bins descend from 255; lane l owns bins 255-4l .. 252-4l.  Finds the
// bin b where the suffix sum (from 255 down, inclusive) first reaches `need`, writes b and the
// need left inside b to sel[0] / sel64[0].
template <typename C>
__device__ __forceinline__ void pick_digit(const C* hist, unsigned long long need, int* sel_b,
                                           unsigned long long* sel_need) {
  const int lane = threadIdx.x;  // wave 0 only
  unsigned long long v[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = hist[255 - 4 * lane - q];
    s += v[q];
  }
  // inclusive prefix over lanes (lane 0 = the top bins); counts fit 32 bits: one shuffle a step
  unsigned long long pre = s;
  if constexpr (sizeof(C) == 4) {
    unsigned p32 = static_cast<unsigned>(s);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned t = __shfl_up(p32, o, 64);
      if (lane >= o) p32 += t;
    }
    pre = p32;
  } else {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned lo = __shfl_up(static_cast<unsigned>(pre), o, 64);
      const unsigned hi = __shfl_up(static_cast<unsigned>(pre >> 32), o, 64);
      if (lane >= o) pre += (static_cast<unsigned long long>(hi) << 32) | lo;
    }
  }
  const unsigned long long hit = __ballot(pre >= need);
  const int first = hit ? __builtin_ctzll(hit) : 63;
  if (lane == first) {
    unsigned long long base = pre - s;
    int b = 255 - 4 * lane - 3;
    unsigned long long left = need - base;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (base + v[q] >= need || q == 3) {
        b = 255 - 4 * lane - q;
        left = need - base;
        break;
      }
      base += v[q];
    }
    *sel_b = b;
    *sel_need = left;
  }
}

// Largest key t with  sum_{key >= t, key >= lo} weight >= need  (need >= 1), weight = 1
// (MASS = false) or the fixed-point mass (MASS = true).  Four 8-bit levels, MSB first.
template <typename T, int NPT, bool MASS>
__device__ __forceinline__ uint32_t radix_select(const Row<T, NPT>& row, float m, uint32_t lo,
                                 unsigned long long need, unsigned* hc, unsigned long long* hm,
                                 int* sel_b, unsigned long long* sel_need) {
  uint32_t prefix = 0, mask = 0;
#pragma unroll 1
  for (int lvl = 0; lvl < 4; ++lvl) {
    const int shift = 24 - 8 * lvl;
    for (int b = threadIdx.x; b < 256; b += kSampNT) {
      if (MASS) hm[b] = 0; else hc[b] = 0;
    }
    __syncthreads();
    row.each([&](int, float z) {
      const uint32_t k = fkey(z);
      if ((k & mask) == prefix && k >= lo) {
        const int d = (k >> shift) & 255;
        if constexpr (MASS) {
          const unsigned long long w =
              static_cast<unsigned long long>(__expf(z - m) * 4294967296.f);
          if (w) atomicAdd(hm + d, w);
        } else {
          atomicAdd(hc + d, 1u);
        }
      }
    });
    __syncthreads();
    if (threadIdx.x < 64) {
      if constexpr (MASS) pick_digit(hm, need, sel_b, sel_need);
      else pick_digit(hc, need, sel_b, sel_need);
    }
    __syncthreads();
    prefix |= static_cast<uint32_t>(*sel_b) << shift;
    mask |= 255u << shift;
    need = *sel_need;
    __syncthreads();
  }
  return prefix;
}

template <typename T, int NPT>
__global__ void __launch_bounds__(kSampNT) sample_kernel(
    const T* __restrict__ logits, const float* __restrict__ temperature,
    const float* __restrict__ top_p, const int* __restrict__ top_k, unsigned long long seed,
    long long offset, long long* __restrict__ out_tok, float* __restrict__ out_lp,
    float* __restrict__ out_tau, int V) {
  __shared__ float red[kSampNT / 64];
  __shared__ int redi[kSampNT / 64];
  __shared__ unsigned hc[256];
  __shared__ unsigned long long hm[256];
  __shared__ unsigned long long red64[kSampNT / 64];
  __shared__ int sel_b;
  __shared__ unsigned long long sel_need;
  extern __shared__ __attribute__((aligned(16))) float zlds[];
  const int row_i = blockIdx.x;
  const float temp = temperature[row_i];
  const bool greedy = !(temp > 0.f);
  Row<T, NPT> row;
  row.p = logits + static_cast<size_t>(row_i) * V;
  row.V = V;
  row.invT = greedy ? 1.f : 1.f / temp;
  row.zl = zlds;
  if constexpr (NPT > 0) {
    // 16-byte loads, 4 per thread in flight (one 2-byte load per element, a few in flight, left
    // the row copy latency-bound: ~20 us of a greedy step), then the scalar tail
    constexpr int E = 16 / static_cast<int>(sizeof(T));
    const bool al = (reinterpret_cast<uintptr_t>(row.p) & 15) == 0;
    const int nv = al ? V / E : 0;
    for (int i0 = threadIdx.x; i0 < nv; i0 += 4 * kSampNT) {
      uint4 u[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = min(i0 + q * kSampNT, nv - 1);  // clamped: unconditional loads
        u[q] = reinterpret_cast<const uint4*>(row.p)[i];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = i0 + q * kSampNT;
        if (i < nv) {
          const T* e = reinterpret_cast<const T*>(&u[q]);
#pragma unroll
          for (int t = 0; t < E; ++t) zlds[i * E + t] = to_f32(e[t]) * row.invT;
        }
      }
    }
    for (int j = nv * E + threadIdx.x; j < V; j += kSampNT) zlds[j] = row.ld(j);
    __syncthreads();
  }
  float m = -INFINITY;
  row.each([&](int, float z) { m = fmaxf(m, z); });
  const float tmax = m;  // this thread's own maximum (every thread owns >= 1 element: V >= 512)
  m = block_max<kSampNT>(m, red);
  float s = 0.f;
  row.each([&](int, float z) { s += __expf(z - m); });
  const float Z = block_sum<kSampNT>(s, red);
  uint32_t tau = 0;  // keep key >= tau (0: everything)
  if (!greedy) {
    const int k = top_k[row_i];
    if (k > 0 && k < V) {
      // lower bound for the k-th largest key: the smallest of the 512 per-thread maxima (512
      // distinct elements are >= it, so for k <= 512 the k-th largest is too).  Only keys >= it
      // enter the histograms: the first level's LDS atomics drop from V to the upper tail
      uint32_t lo = 0;
      if (k <= kSampNT && V >= kSampNT) lo = fkey(-block_max<kSampNT>(-tmax, red));
      tau = radix_select<T, NPT, false>(row, m, lo, static_cast<unsigned long long>(k), hc, hm,
                                        &sel_b, &sel_need);
    }
    const float p = top_p[row_i];
    if (p < 1.f) {
      // mass of the top-k-kept set, fixed point (exact integer sum)
      unsigned long long zk = 0;
      row.each([&](int, float z) {
        if (fkey(z) >= tau) zk += static_cast<unsigned long long>(__expf(z - m) * 4294967296.f);
      });
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned lo = __shfl_xor(static_cast<unsigned>(zk), o, 64);
        const unsigned hi = __shfl_xor(static_cast<unsigned>(zk >> 32), o, 64);
        zk += (static_cast<unsigned long long>(hi) << 32) | lo;
      }
      if ((threadIdx.x & 63) == 0) red64[threadIdx.x >> 6] = zk;
      __syncthreads();
      zk = 0;
#pragma unroll
      for (int w = 0; w < kSampNT / 64; ++w) zk += red64[w];
      __syncthreads();
      const double tgt = static_cast<double>(fmaxf(p, 0.f)) * static_cast<double>(zk);
      unsigned long long need = static_cast<unsigned long long>(ceil(tgt));
      if (need < 1) need = 1;
      if (need > zk) need = zk;
      const uint32_t tp =
          radix_select<T, NPT, true>(row, m, tau, need, hc, hm, &sel_b, &sel_need);
      tau = tp > tau ? tp : tau;
    }
  }
  // argmax over the kept set (with Gumbel noise unless greedy)
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const uint32_t sd = static_cast<uint32_t>(seed) ^
                      (static_cast<uint32_t>(offset) * 0x9E3779B9u + 0x7F4A7C15u);
  row.each([&](int j, float z) {
    if (fkey(z) < tau) return;
    float key = z;
    if (!greedy) {
      const uint32_t r = rng_u32(sd, static_cast<uint64_t>(row_i) * static_cast<uint64_t>(V) + j);
      const float u = (static_cast<float>(r >> 8) + 0.5f) * (1.f / 16777216.f);
      key = z - __logf(-__logf(u));
    }
    if (key > best || (key == best && j < bi)) { best = key; bi = j; }
  });
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
    out_tok[row_i] = idx;
    if (out_lp) out_lp[row_i] = row.ld(idx) - m - __logf(Z);
    if (out_tau) out_tau[row_i] = tau ? keyf(tau) : -INFINITY;
  }
}

template <typename T>
hipError_t launch_sample(const void* logits, const float* temperature, const float* top_p,
                         const int* top_k, unsigned long long seed, long long offset,
                         long long* out_tok, float* out_lp, float* out_tau, int rows, int V,
                         hipStream_t st) {
  dim3 grid(rows), block(kSampNT);
  const T* lg = static_cast<const T*>(logits);
  if (V <= kSampLdsV) {
    // the LDS row copy goes past the 64 KiB dynamic default (gfx950 has 160 KiB per CU)
    static bool attr_set = false;
    if (!attr_set) {
      const hipError_t e = hipFuncSetAttribute(
          reinterpret_cast<const void*>(&sample_kernel<T, 1>),
          hipFuncAttributeMaxDynamicSharedMemorySize, kSampLdsV * static_cast<int>(sizeof(float)));
      if (e != hipSuccess) return e;
      attr_set = true;
    }
    hipLaunchKernelGGL((sample_kernel<T, 1>), grid, block, V * sizeof(float), st, lg, temperature,
                       top_p, top_k, seed, offset, out_tok, out_lp, out_tau, V);
  } else {
    hipLaunchKernelGGL((sample_kernel<T, 0>), grid, block, 0, st, lg, temperature, top_p, top_k,
                       seed, offset, out_tok, out_lp, out_tau, V);
  }
  return hipGetLastError();
}

}  // namespace lumen

// out_tau (optional): per row the smallest kept scaled logit (-inf when nothing is truncated)
extern "C" hipError_t lumen_sample(int dtype, const void* logits, const float* temperature,
                                   const float* top_p, const int* top_k, unsigned long long seed,
                                   long long offset, long long* out_tok, float* out_lp,
                                   float* out_tau, int rows, int V, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  if (V < 1) return hipErrorInvalidValue;
  if (dtype == lumen::kF32)
    return lumen::launch_sample<float>(logits, temperature, top_p, top_k, seed, offset, out_tok,
                                       out_lp, out_tau, rows, V, st);
  if (dtype == lumen::kBF16)
    return lumen::launch_sample<lumen::bf16>(logits, temperature, top_p, top_k, seed, offset,
                                             out_tok, out_lp, out_tau, rows, V, st);
  if (dtype == lumen::kF16)
    return lumen::launch_sample<lumen::fp16>(logits, temperature, top_p, top_k, seed, offset,
                                             out_tok, out_lp, out_tau, rows, V, st);
  return hipErrorInvalidValue;
}
