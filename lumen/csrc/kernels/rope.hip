// Rotary position embedding, fused with the QKV split/transposition.
//
// Reference behaviour: transformers' Llama `apply_rotary_pos_emb` with `rotate_half`
// (theta = 1e4), applied to q and k of every layer of the model loaded at
// training/train_baseline.py:122-126 -- eager PyTorch runs it as slice/neg/cat/mul/add launches
// plus the `transpose(1, 2)` copies around SDPA.
//
// Here ONE pass reads the fused QKV GEMM output [T, (nh + 2*nkv) * D] (token-major) and writes
// q/k/v in the head-major [B, heads, S, D] layout attention consumes, rotating q and k on the way
// (rotate_half convention: pair (i, i + D/2)).  The backward pass applies the inverse rotation and
// writes the token-major dQKV that feeds the QKV GEMM's dX.  cos/sin come from an f32 table
// [max_pos, D/2] built once on the host (on-device sincosf would make this VALU-bound).
//
// Thread mapping: one thread = 8 rotation pairs (16 elements, two 16-byte vectors) of one
// (token, head); v heads are plain 16-element copies.
#include "common.h"

namespace lumen {

template <typename T, bool BWD>
__global__ void __launch_bounds__(256) qkv_rope_kernel(
    // fwd: src = qkv [T, nh+2nkv, D] ; dst q/k/v [B, heads, S, D]
    // bwd: src = dq/dk/dv [B, heads, S, D] ; dst dqkv [T, nh+2nkv, D]
    T* __restrict__ qkv, T* __restrict__ q, T* __restrict__ k, T* __restrict__ v,
    const int* __restrict__ pos, const float* __restrict__ cos_t, const float* __restrict__ sin_t,
    int T_tokens, int S, int nh, int nkv, int D) {
  const int chunks = D / 16;  // threads per head row
  const int heads = nh + 2 * nkv;
  const long long tid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long total = static_cast<long long>(T_tokens) * heads * chunks;
  if (tid >= total) return;
  const int c = static_cast<int>(tid % chunks);
  const int hs = static_cast<int>((tid / chunks) % heads);
  const int t = static_cast<int>(tid / (static_cast<long long>(chunks) * heads));
  const int b = t / S, s = t % S;
  const int half = D / 2;
  T* tok = qkv + (static_cast<size_t>(t) * heads + hs) * D;
  T* hm;  // head-major row
  if (hs < nh) hm = q + ((static_cast<size_t>(b) * nh + hs) * S + s) * D;
  else if (hs < nh + nkv) hm = k + ((static_cast<size_t>(b) * nkv + (hs - nh)) * S + s) * D;
  else hm = v + ((static_cast<size_t>(b) * nkv + (hs - nh - nkv)) * S + s) * D;

  if (hs >= nh + nkv) {  // v: copy 16 elements (32 bytes for 16-bit T, 64 for f32)
    const T* src = BWD ? hm : tok;
    T* dst = BWD ? tok : hm;
    constexpr int U = 16 * sizeof(T) / sizeof(uint4);
    const uint4* sp = reinterpret_cast<const uint4*>(src + c * 16);
    uint4* dp = reinterpret_cast<uint4*>(dst + c * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) dp[u] = sp[u];
    return;
  }
  const int p = pos ? pos[t] : s;
  const int i0 = c * 8;  // first of 8 pairs (i, i + half)
  const float* cp = cos_t + static_cast<size_t>(p) * half + i0;
  const float* sp = sin_t + static_cast<size_t>(p) * half + i0;
  float cs[8], sn[8], a[8], bb[8], oa[8], ob[8];
  load8(cp, cs);
  load8(sp, sn);
  const T* src = BWD ? hm : tok;
  T* dst = BWD ? tok : hm;
  load8(src + i0, a);
  load8(src + i0 + half, bb);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // fwd:  a' = a cos - b sin ;  b' = b cos + a sin
    // bwd (transpose of the rotation): da = da' cos + db' sin ; db = db' cos - da' sin
    const float sgn = BWD ? -1.f : 1.f;
    oa[j] = a[j] * cs[j] - sgn * bb[j] * sn[j];
    ob[j] = bb[j] * cs[j] + sgn * a[j] * sn[j];
  }
  store8(dst + i0, oa);
  store8(dst + i0 + half, ob);
}

// In-place RoPE on a token-major buffer x[T, row_stride] holding `nheads` heads of D starting at
// column offset 0 (serving path: q and k inside the fused QKV output, arbitrary positions).
template <typename T>
__global__ void __launch_bounds__(256) rope_inplace_kernel(
    T* __restrict__ x, const int* __restrict__ pos, const float* __restrict__ cos_t,
    const float* __restrict__ sin_t, int T_tokens, int row_stride, int nheads, int D) {
  const int chunks = D / 16;
  const long long tid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long total = static_cast<long long>(T_tokens) * nheads * chunks;
  if (tid >= total) return;
  const int c = static_cast<int>(tid % chunks);
  const int h = static_cast<int>((tid / chunks) % nheads);
  const int t = static_cast<int>(tid / (static_cast<long long>(chunks) * nheads));
  const int half = D / 2, i0 = c * 8;
  T* row = x + static_cast<size_t>(t) * row_stride + static_cast<size_t>(h) * D;
  float cs[8], sn[8], a[8], bb[8], oa[8], ob[8];
  // the row loads go out first: they do not depend on the position, whose load the cos / sin
  // loads wait for
  load8(row + i0, a);
  load8(row + i0 + half, bb);
  const int p = pos[t];
  load8(cos_t + static_cast<size_t>(p) * half + i0, cs);
  load8(sin_t + static_cast<size_t>(p) * half + i0, sn);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // explicit fmas: bit-identical to the fused RoPE + KV-cache write (rope_cache_kernel)
    // whatever the compiler contracts.  (8 heads per thread, one table load for all: 27.6 vs
    // 23.8 us per training call, gpurun r5_46 -- fewer rows in flight per CU; removed.)
    oa[j] = fmaf(a[j], cs[j], -(bb[j] * sn[j]));
    ob[j] = fmaf(bb[j], cs[j], a[j] * sn[j]);
  }
  store8(row + i0, oa);
  store8(row + i0 + half, ob);
}

template <typename T>
static hipError_t launch_qkv(bool bwd, void* qkv, void* q, void* k, void* v, const int* pos,
                             const float* cs, const float* sn, int T_tokens, int S, int nh,
                             int nkv, int D, hipStream_t st) {
  const long long total = static_cast<long long>(T_tokens) * (nh + 2 * nkv) * (D / 16);
  dim3 grid(static_cast<unsigned>((total + 255) / 256)), block(256);
  if (bwd)
    hipLaunchKernelGGL((qkv_rope_kernel<T, true>), grid, block, 0, st, (T*)qkv, (T*)q, (T*)k,
                       (T*)v, pos, cs, sn, T_tokens, S, nh, nkv, D);
  else
    hipLaunchKernelGGL((qkv_rope_kernel<T, false>), grid, block, 0, st, (T*)qkv, (T*)q, (T*)k,
                       (T*)v, pos, cs, sn, T_tokens, S, nh, nkv, D);
  return hipGetLastError();
}

}  // namespace lumen

extern "C" hipError_t lumen_qkv_rope(int dtype, int bwd, void* qkv, void* q, void* k, void* v,
                                     const int* pos, const float* cos_t, const float* sin_t,
                                     int T_tokens, int S, int nh, int nkv, int D, hipStream_t st) {
  if (D % 16 != 0) return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::launch_qkv<lumen::bf16>(bwd, qkv, q, k, v, pos, cos_t, sin_t, T_tokens, S, nh,
                                          nkv, D, st);
  if (dtype == lumen::kF16)
    return lumen::launch_qkv<lumen::fp16>(bwd, qkv, q, k, v, pos, cos_t, sin_t, T_tokens, S, nh,
                                          nkv, D, st);
  if (dtype == lumen::kF32)
    return lumen::launch_qkv<float>(bwd, qkv, q, k, v, pos, cos_t, sin_t, T_tokens, S, nh, nkv,
                                    D, st);
  return hipErrorInvalidValue;
}

extern "C" hipError_t lumen_rope_inplace(int dtype, void* x, const int* pos, const float* cos_t,
                                         const float* sin_t, int T_tokens, int row_stride,
                                         int nheads, int D, hipStream_t st) {
  if (D % 16 != 0) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(T_tokens) * nheads * (D / 16);
  dim3 grid(static_cast<unsigned>((total + 255) / 256)), block(256);
  if (total == 0) return hipSuccess;
  if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::rope_inplace_kernel<lumen::bf16>, grid, block, 0, st,
                       (lumen::bf16*)x, pos, cos_t, sin_t, T_tokens, row_stride, nheads, D);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::rope_inplace_kernel<lumen::fp16>, grid, block, 0, st,
                       (lumen::fp16*)x, pos, cos_t, sin_t, T_tokens, row_stride, nheads, D);
  else if (dtype == lumen::kF32)
    hipLaunchKernelGGL(lumen::rope_inplace_kernel<float>, grid, block, 0, st, (float*)x, pos,
                       cos_t, sin_t, T_tokens, row_stride, nheads, D);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
