// Common helpers for lumen's gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave64: every lane-count constant is 64, block sizes are multiples of 64.
//  * 16-bit activations (bf16 / fp16) are moved as 16-byte vectors (8 elements per lane),
//    converted to f32 in registers and accumulated in f32.
//  * launchers are `extern "C"` functions that take raw pointers + a hipStream_t and never
//    allocate or synchronise (safe under hipGraph capture).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace lumen {

constexpr int kWave = 64;

using bf16 = __hip_bfloat16;
using fp16 = __half;

// dtype codes shared with the Python binding
enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2 };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return __bfloat162float(x); }
__device__ __forceinline__ float to_f32(fp16 x) { return __half2float(x); }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return __float2bfloat16(x); }
template <> __device__ __forceinline__ fp16 from_f32<fp16>(float x) { return __float2half(x); }

// two f32 -> one packed 16-bit pair (element 0 in the low half), round to nearest even.  For
// bf16 this is ONE v_cvt_pk_bf16_f32; converting the elements one at a time compiles to two
// conversions plus a shift and an or per pair (4x the VALU in the attention / LoRA inner loops).
// fp16 likewise: ONE v_cvt_pk_f16_f32 (gfx950).  __floats2half2_rn compiled to two
// v_cvt_f16_f32 + v_perm per pair, and the compiler then waited for each feeding load on its
// own (lora3_dy: 116 vs 39 s_waitcnt, 58 vs 36 us per call; profiles/r3d/fp16).
typedef float lumen_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 lumen_bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 lumen_f16x2 __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ unsigned pk2(float a, float b);
template <> __device__ __forceinline__ unsigned pk2<bf16>(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(lumen_f32x2{a, b}, lumen_bf16x2));
}
template <> __device__ __forceinline__ unsigned pk2<fp16>(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(lumen_f32x2{a, b}, lumen_f16x2));
}

// 16-byte vector of 8 half-precision elements.
template <typename T> struct alignas(16) Vec8 { T v[8]; };

template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ p, float (&out)[8]) {
  const uint4 raw = *reinterpret_cast<const uint4*>(p);
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = to_f32(e[j]);
}

template <>
__device__ __forceinline__ void load8<float>(const float* __restrict__ p, float (&out)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
  out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
}

template <typename T>
__device__ __forceinline__ void store8(T* __restrict__ p, const float (&in)[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pk2<T>(in[0], in[1]), pk2<T>(in[2], in[3]),
                                            pk2<T>(in[4], in[5]), pk2<T>(in[6], in[7]));
}

template <>
__device__ __forceinline__ void store8<float>(float* __restrict__ p, const float (&in)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(in[4], in[5], in[6], in[7]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `scratch` holds NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

// Counter-based RNG for LoRA dropout: the backward regenerates the forward's keep-mask from
// (seed, element index) instead of storing it.  One multiply-mix of the 64-bit index with the
// host-premixed 32-bit seed, then the "lowbias32" finaliser (2 multiplies): ~10 VALU ops per
// element, so mask regeneration stays cheap inside memory-bound staging loops.
__device__ __forceinline__ uint32_t rng_u32(uint32_t seed32, uint64_t idx) {
  uint32_t h = static_cast<uint32_t>(idx) * 0x9E3779B1u +
               static_cast<uint32_t>(idx >> 32) * 0x85EBCA77u + seed32;
  h ^= h >> 16; h *= 0x7feb352dU;
  h ^= h >> 15; h *= 0x846ca68bU;
  h ^= h >> 16;
  return h;
}

// keep-probability test with a 16-bit threshold (p * 65536): one 32-bit hash of the pair index
// idx >> 1 serves two consecutive elements (low half for the even one, high half for the odd),
// halving the hashing work of the mask-regenerating kernels.
__device__ __forceinline__ bool dropout_keep(uint32_t seed32, uint64_t idx, uint32_t thresh16) {
  const uint32_t h = rng_u32(seed32, idx >> 1);
  return ((h >> ((idx & 1) * 16)) & 0xFFFFu) >= thresh16;
}

// masks of 8 consecutive elements starting at an even index: bit e set = element e kept
__device__ __forceinline__ uint32_t dropout_keep8(uint32_t seed32, uint64_t idx0, uint32_t thresh16) {
  uint32_t m = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t h = rng_u32(seed32, (idx0 >> 1) + e);
    m |= ((h & 0xFFFFu) >= thresh16 ? 1u : 0u) << (2 * e);
    m |= ((h >> 16) >= thresh16 ? 1u : 0u) << (2 * e + 1);
  }
  return m;
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

}  // namespace lumen
