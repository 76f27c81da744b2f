// Deterministic cross-workgroup sums (VERDICT r5 "Next" #4).
//
// The LoRA adapter gradients and the gradient norm used to be summed over workgroups with f32
// global atomics, whose order -- and so whose rounding -- changed from run to run.  Here every
// contributing workgroup writes its f32 partial with WRITE-THROUGH (sc1) stores, every storing
// wave drains them (vmcnt(0)), the workgroup meets at a barrier, ONE lane takes a ticket on an
// agent-scope counter, and the workgroup whose ticket is the last one sums all partials in a FIXED
// order with sc1 loads.  No fences: this is the hand-off form "one lane of each storing workgroup,
// an agent-scope atomic add; the last by the value its add returned; 4-/8-byte sc1 stores, sc1
// loads" of MI355X_MICROARCH.md (inter-workgroup visibility, Valid forms).  The last arriver
// re-zeroes the counter, so counters stay zero between launches.
#pragma once
#include "common.h"

namespace lumen {
namespace det {

typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store((gf32*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load((const gf32*)(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// two consecutive floats (8-byte aligned) in one sc1 load
__device__ __forceinline__ float2 ld_wt2(const float* p) {
  const unsigned long long u = __hip_atomic_load((const gu64*)(p),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float(static_cast<unsigned>(u)),
                     __uint_as_float(static_cast<unsigned>(u >> 32)));
}

// sum over q = 0 .. n-1 of the float pair at base + q * stride, added in q order: the loads are
// issued 16 at a time (independent, so they are in flight together; a dependent one-at-a-time loop
// left every slab's memory latency exposed: dy3 104.5 vs 28.9 us per call)
__device__ __forceinline__ float2 sum_pairs(const float* base, long long stride, int n) {
  float2 v = make_float2(0.f, 0.f);
  for (int q0 = 0; q0 < n; q0 += 16) {
    float2 u[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = q0 + k < n ? q0 + k : n - 1;  // clamped: unconditional loads
      u[k] = ld_wt2(base + q * stride);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (q0 + k < n) {
        v.x += u[k].x;
        v.y += u[k].y;
      }
    }
  }
  return v;
}

// Call from EVERY thread of the workgroup after its sc1 partial stores.  Returns true in every
// thread of the workgroup that arrived last of `n` (flag: an int in the kernel's LDS).
__device__ __forceinline__ bool last_arriver(unsigned* cnt, unsigned n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == n - 1;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

}  // namespace det
}  // namespace lumen
