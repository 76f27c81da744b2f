// Weight-streaming GEMM for low-batch decode: y[M, N] = x[M, K] @ W[N, K]^T, M <= 16.
//
// Reference behaviour: vLLM's decode projections (the serving stack the reference declares,
// SURVEY D11 / CS6) run these as library GEMMs.  At M <= 16 the op is a pure stream of the
// weight matrix (Llama-2-7B: 420 MB per layer, 2 FLOP per byte), and hipBLASLt's small-M tiles
// reach 50-80 % of HBM bandwidth (o_proj 12.1 us for 33.5 MB, profiles/r02_serve).
//
// Design (gfx950, wave64, v_mfma_f32_16x16x32_bf16):
//  * one workgroup = 4 waves = 16 output columns; the 4 waves split K four ways, each streaming
//    its 16 weight rows with 16-byte loads (lane: row n0 + (lane & 15), k offset 8 * (lane >> 4));
//  * the weight fragment IS the MFMA B operand (k-contiguous rows, no LDS staging); x (tiny,
//    L2-resident) is the A operand, rows >= M zero without a load;
//  * software pipelined: the next U k-steps' loads are in flight while the current ones feed
//    the MFMAs (U * 1 KiB per wave, 2U in flight), which is what keeps ~10 B/cycle/CU of HBM
//    traffic going at one workgroup per CU;
//  * the four K partials meet in LDS; wave 0 writes the M x 16 output tile.
#include "common.h"

namespace lumen {
namespace sk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
  static __device__ __forceinline__ f32x4 run(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mfma<fp16> {
  static __device__ __forceinline__ f32x4 run(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

constexpr int U = 8;  // k-steps (of 32) per pipeline stage

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// weights are read exactly once per decode step: non-temporal, so they do not evict x / y
template <typename T>
__device__ __forceinline__ uint4 ntload(const T* p) {
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
}

template <typename T>
__global__ void __launch_bounds__(256) skinny_kernel(const T* __restrict__ x,
                                                     const T* __restrict__ W, T* __restrict__ y,
                                                     int M, int N, int K, long long ldx,
                                                     long long ldy) {
  __shared__ float red[4][16][17];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kq = K >> 2;  // this wave's K range (host guarantees K % 128 == 0)
  const int kb = wid * kq;
  const bool arow = lr < M;
  const T* xp = x + (long long)(arow ? lr : 0) * ldx + kb + 8 * lg;
  const T* wp = W + (long long)(n0 + lr) * K + kb + 8 * lg;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int steps = kq >> 5;  // k-steps of 32
  const int full = steps / U;
  uint4 bcur[U], acur[U];
  const uint4 z = make_uint4(0, 0, 0, 0);
  if (full > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bcur[u] = ntload(wp + 32 * u);
      acur[u] = arow ? *reinterpret_cast<const uint4*>(xp + 32 * u) : z;
    }
  }
  for (int s = 0; s < full; ++s) {
    uint4 bnext[U], anext[U];
    const int kn = (s + 1) * 32 * U;
    if (s + 1 < full) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        bnext[u] = ntload(wp + kn + 32 * u);
        anext[u] = arow ? *reinterpret_cast<const uint4*>(xp + kn + 32 * u) : z;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = Mfma<T>::run(acur[u], bcur[u], acc);
    if (s + 1 < full) {
#pragma unroll
      for (int u = 0; u < U; ++u) { bcur[u] = bnext[u]; acur[u] = anext[u]; }
    }
  }
  for (int st = full * U; st < steps; ++st) {  // tail (K / 4 not a multiple of 32 U)
    const uint4 b = *reinterpret_cast<const uint4*>(wp + 32 * st);
    const uint4 a = arow ? *reinterpret_cast<const uint4*>(xp + 32 * st) : z;
    acc = Mfma<T>::run(a, b, acc);
  }
  // C tile: lane holds column lr, rows 4 lg + i
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wid][4 * lg + i][lr] = acc[i];
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * lg + i;
      if (m < M) {
        const float v = red[0][m][lr] + red[1][m][lr] + red[2][m][lr] + red[3][m][lr];
        y[(long long)m * ldy + n0 + lr] = from_f32<T>(v);
      }
    }
  }
}

// ---- M <= 4: VALU dot products on fully coalesced weight rows -------------------------------
// The MFMA form above reads each weight row in 64-byte pieces (16 rows per wave-instruction),
// which measured 2.3-3.4 TB/s.  Here a wave-instruction reads 4 rows x 256 contiguous bytes
// (lane: row L >> 4, 16-byte chunk L & 15), the full-rate access shape, and v_dot2c_f32_bf16
// does the (at most 4 rows x 2 FLOP/byte) arithmetic.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <typename T> __device__ __forceinline__ float dot2(unsigned a, unsigned b, float c);
template <> __device__ __forceinline__ float dot2<bf16>(unsigned a, unsigned b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a),
                                         __builtin_bit_cast(bf16x2, b), c, false);
}
template <> __device__ __forceinline__ float dot2<fp16>(unsigned a, unsigned b, float c) {
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b), c,
                                false);
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
__device__ __forceinline__ float sum16(float v) {  // over the 16 lanes of a DPP row
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return v;
}

constexpr int GU = 8;  // 128-element steps in flight per wave

// SWIGLU: x is the fused gate|up GEMM output [M, 2K] and the operand is act = silu(gate) * up,
// formed in registers and rounded to T exactly as kernels/swiglu.hip rounds it, so the batch-1
// down projection needs no separate activation launch.
template <typename T>
__device__ __forceinline__ uint4 swiglu8(uint4 g, uint4 u) {
  const T* ge = reinterpret_cast<const T*>(&g);
  const T* ue = reinterpret_cast<const T*>(&u);
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = silu(to_f32(ge[j])) * to_f32(ue[j]);
  return make_uint4(pk2<T>(a[0], a[1]), pk2<T>(a[2], a[3]), pk2<T>(a[4], a[5]),
                    pk2<T>(a[6], a[7]));
}

// One workgroup = 4 rows; its 4 waves split K in 128-element steps (weights AND x issued up
// front for the whole slice) and meet in LDS.  (A variant with one wave per 4 rows over the
// whole of K, prefetching weights but loading x inside the loop, measured 2.96 vs 3.73 TB/s.)
template <typename T, int MM, bool SWIGLU = false>
__global__ void __launch_bounds__(256) gemv_kernel(const T* __restrict__ x,
                                                   const T* __restrict__ W, T* __restrict__ y,
                                                   int M, int N, int K, long long ldx,
                                                   long long ldy) {
  __shared__ float red[4][MM][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane >> 4, c = lane & 15;
  const int n = blockIdx.x * 4 + r;
  const int S = (K + 127) >> 7;  // 128-element steps
  const int s0 = (wid * S) >> 2, s1 = ((wid + 1) * S) >> 2;
  const T* wp = W + (long long)n * K + 8 * c;
  const T* xp = x + 8 * c;
  float acc[MM];
#pragma unroll
  for (int m = 0; m < MM; ++m) acc[m] = 0.f;
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int s = s0; s < s1; s += GU) {
    uint4 wv[GU], xv[GU][MM];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int k = (s + u) * 128 + 8 * c;
      const bool ok = (s + u < s1) && (k < K);
      wv[u] = ok ? ntload(wp + (s + u) * 128) : z;
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const T* xr = xp + m * ldx + (s + u) * 128;
        xv[u][m] = (ok && m < M) ? *reinterpret_cast<const uint4*>(xr) : z;
        if constexpr (SWIGLU)  // up half at +K; zero pairs give silu(0) * 0 = 0
          xv[u][m] = swiglu8<T>(xv[u][m],
                                (ok && m < M) ? *reinterpret_cast<const uint4*>(xr + K) : z);
      }
    }
#pragma unroll
    for (int u = 0; u < GU; ++u)
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        acc[m] = dot2<T>(wv[u].x, xv[u][m].x, acc[m]);
        acc[m] = dot2<T>(wv[u].y, xv[u][m].y, acc[m]);
        acc[m] = dot2<T>(wv[u].z, xv[u][m].z, acc[m]);
        acc[m] = dot2<T>(wv[u].w, xv[u][m].w, acc[m]);
      }
  }
#pragma unroll
  for (int m = 0; m < MM; ++m) {
    const float v = sum16(acc[m]);
    if (c == 0) red[wid][m][r] = v;
  }
  __syncthreads();
  if (threadIdx.x < MM * 4) {
    const int m = threadIdx.x >> 2, rr = threadIdx.x & 3;
    if (m < M) {
      const float v = red[0][m][rr] + red[1][m][rr] + red[2][m][rr] + red[3][m][rr];
      y[(long long)m * ldy + blockIdx.x * 4 + rr] = from_f32<T>(v);
    }
  }
}

// ---- M == 1, rows-per-lane form ---------------------------------------------------------------
// lane = one 16-byte chunk of K, 4 weight rows per lane: a wave instruction reads 1 KiB of ONE
// row (fully contiguous), and the x chunk is loaded -- and with SWIGLU activated -- once per 4
// rows instead of once per row (the form above repeats both for each of its 4 row groups).
constexpr int GS = 4;  // 512-element steps in flight per wave (x 4 rows = 16 loads per lane)

template <typename T, bool SWIGLU, int MM = 1>
__global__ void __launch_bounds__(256) gemv_r4_kernel(const T* __restrict__ x,
                                                      const T* __restrict__ W, T* __restrict__ y,
                                                      int N, int K, int M, long long ldx,
                                                      long long ldy) {
  // MM > 1 (decode batches 2..4): the 4 weight rows of a lane meet MM x chunks (one per batch
  // row, x rows at stride ldx) -- the weight stream is unchanged, x traffic grows to MM : 4
  __shared__ float red[4][MM][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 4;
  const int S = (K + 511) >> 9;  // 512-element steps
  const int s0 = (wid * S) >> 2, s1 = ((wid + 1) * S) >> 2;
  const T* wp = W + (long long)n0 * K + 8 * lane;
  const T* xp = x + 8 * lane;
  float acc[MM][4];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[m][r] = 0.f;
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int s = s0; s < s1; s += GS) {
    uint4 wv[GS][4], xv[GS][MM];
#pragma unroll
    for (int u = 0; u < GS; ++u) {
      const int k = (s + u) * 512;
      const bool ok = (s + u < s1) && (k + 8 * lane < K);
#pragma unroll
      for (int r = 0; r < 4; ++r) wv[u][r] = ok ? ntload(wp + (long long)r * K + k) : z;
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const T* xr = xp + (long long)m * ldx + k;
        xv[u][m] = (ok && m < M) ? *reinterpret_cast<const uint4*>(xr) : z;
        if constexpr (SWIGLU)
          xv[u][m] = swiglu8<T>(xv[u][m], (ok && m < M) ? *reinterpret_cast<const uint4*>(xr + K) : z);
      }
    }
#pragma unroll
    for (int u = 0; u < GS; ++u)
#pragma unroll
      for (int m = 0; m < MM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[m][r] = dot2<T>(wv[u][r].x, xv[u][m].x, acc[m][r]);
          acc[m][r] = dot2<T>(wv[u][r].y, xv[u][m].y, acc[m][r]);
          acc[m][r] = dot2<T>(wv[u][r].z, xv[u][m].z, acc[m][r]);
          acc[m][r] = dot2<T>(wv[u][r].w, xv[u][m].w, acc[m][r]);
        }
  }
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = sum16(acc[m][r]);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane == 0) red[wid][m][r] = v;
    }
  __syncthreads();
  if (threadIdx.x < 4 * MM) {
    const int m = threadIdx.x >> 2, r = threadIdx.x & 3;
    if (m < M)
      y[(long long)m * ldy + n0 + r] =
          from_f32<T>(red[0][m][r] + red[1][m][r] + red[2][m][r] + red[3][m][r]);
  }
}

}  // namespace sk
}  // namespace lumen

// y[M, N] = x[M, K] @ W[N, K]^T with M <= 16, N % 16 == 0, K % 128 == 0; x rows at stride ldx,
// W contiguous, y rows at stride ldy.
namespace {
int g_gemv_form = 1;

template <typename T>
hipError_t launch_gemv(const void* x, const void* W, void* y, int M, int N, int K, long long ldx,
                       long long ldy, hipStream_t st) {
  dim3 grid(N / 4), block(256);
#define LUMEN_GEMV(MM)                                                                          \
  hipLaunchKernelGGL((lumen::sk::gemv_kernel<T, MM>), grid, block, 0, st, (const T*)x,        \
                     (const T*)W, (T*)y, M, N, K, ldx, ldy)
  if (M == 1 && g_gemv_form == 1)
    hipLaunchKernelGGL((lumen::sk::gemv_r4_kernel<T, false, 1>), grid, block, 0, st, (const T*)x,
                       (const T*)W, (T*)y, N, K, 1, ldx, ldy);
  else if (M == 2 && g_gemv_form == 1)
    hipLaunchKernelGGL((lumen::sk::gemv_r4_kernel<T, false, 2>), grid, block, 0, st, (const T*)x,
                       (const T*)W, (T*)y, N, K, 2, ldx, ldy);
  else if (M <= 4 && g_gemv_form == 1)
    hipLaunchKernelGGL((lumen::sk::gemv_r4_kernel<T, false, 4>), grid, block, 0, st, (const T*)x,
                       (const T*)W, (T*)y, N, K, M, ldx, ldy);
  else if (M == 1) LUMEN_GEMV(1);
  else if (M == 2) LUMEN_GEMV(2);
  else LUMEN_GEMV(4);
#undef LUMEN_GEMV
  return hipGetLastError();
}
}  // namespace

// y[1, N] = (silu(gu[:, :K]) * gu[:, K:]) @ W[N, K]^T: the batch-1 down projection with the
// SwiGLU activation formed on the fly (gu row stride ldgu >= 2K).
// M == 1 kernel form: 1 = rows-per-lane (gemv_r4_kernel), 0 = row-group form (gemv_kernel)
extern "C" void lumen_set_gemv_form(int form) { g_gemv_form = form; }

// y[M, N] = (silu(gu[:, :K]) * gu[:, K:]) @ W[N, K]^T for M <= 4 (decode batches): the SwiGLU
// activation formed in registers inside the rows-per-lane weight stream (gu rows at stride ldgu
// >= 2K), so the batch-1 down projection needs no separate activation launch.
extern "C" hipError_t lumen_skinny_swiglu_gemm(int dtype, const void* gu, const void* W, void* y,
                                               int M, int N, int K, long long ldgu,
                                               long long ldy, hipStream_t st) {
  if (M < 1 || M > 4 || N % 4 != 0 || K % 8 != 0 || ldgu < 2LL * K || ldgu % 8 != 0)
    return hipErrorInvalidValue;
  dim3 grid(N / 4), block(256);
#define LUMEN_SWG(TT, MM)                                                                       \
  hipLaunchKernelGGL((lumen::sk::gemv_r4_kernel<TT, true, MM>), grid, block, 0, st,            \
                     (const TT*)gu, (const TT*)W, (TT*)y, N, K, M, ldgu, ldy)
  if (dtype == lumen::kBF16) {
    if (M == 1) LUMEN_SWG(lumen::bf16, 1);
    else if (M == 2) LUMEN_SWG(lumen::bf16, 2);
    else LUMEN_SWG(lumen::bf16, 4);
  } else if (dtype == lumen::kF16) {
    if (M == 1) LUMEN_SWG(lumen::fp16, 1);
    else if (M == 2) LUMEN_SWG(lumen::fp16, 2);
    else LUMEN_SWG(lumen::fp16, 4);
  } else {
    return hipErrorInvalidValue;
  }
#undef LUMEN_SWG
  return hipGetLastError();
}

extern "C" hipError_t lumen_skinny_gemm(int dtype, const void* x, const void* W, void* y, int M,
                                        int N, int K, long long ldx, long long ldy,
                                        hipStream_t st) {
  if (M >= 1 && M <= 4 && N % 4 == 0 && K % 8 == 0) {  // VALU weight-streaming form
    if (dtype == lumen::kBF16) return launch_gemv<lumen::bf16>(x, W, y, M, N, K, ldx, ldy, st);
    if (dtype == lumen::kF16) return launch_gemv<lumen::fp16>(x, W, y, M, N, K, ldx, ldy, st);
    return hipErrorInvalidValue;
  }
  if (M < 1 || M > 16 || N % 16 != 0 || K % 128 != 0) return hipErrorInvalidValue;
  dim3 grid(N / 16), block(256);
  if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::sk::skinny_kernel<lumen::bf16>, grid, block, 0, st,
                       (const lumen::bf16*)x, (const lumen::bf16*)W, (lumen::bf16*)y, M, N, K,
                       ldx, ldy);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::sk::skinny_kernel<lumen::fp16>, grid, block, 0, st,
                       (const lumen::fp16*)x, (const lumen::fp16*)W, (lumen::fp16*)y, M, N, K,
                       ldx, ldy);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
