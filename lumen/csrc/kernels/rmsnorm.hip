// Fused residual-add + RMSNorm, forward and backward.
//
// Reference behaviour: transformers' LlamaRMSNorm (upcast to f32, x * rsqrt(mean(x^2) + eps),
// cast back, multiply by weight), invoked 65x per forward of Llama-2-7B
// (reference training/train_baseline.py:122 loads the model that runs it).  Eager PyTorch runs it
// as ~7 launches; here it is one memory-bound pass.
//
// Layout: one wave64 per row, each lane owns VPL 16-byte vectors (8 elements each) so a row of
// up to VPL*512 elements stays in registers between the reduction and the write-back.  The block
// holds 4 waves = 4 rows (256 threads), so a 1024-token micro-batch launches 256 blocks and larger
// batches scale past the 256 CUs.
//
// fwd:  s = x (+ residual)           -> written to `s_out` when residual is fused
//       y = s * rsqrt(mean(s^2)+eps) * w
//       rstd[row] saved (f32) for backward
// bwd:  g = dy * w;  ds = rstd * (g - s*rstd * mean(g * s*rstd)) (+ ds_residual)
//       dw (optional) += sum_rows(dy * s * rstd)  (f32, per-block partials then atomics)
#include "common.h"

#include <cstdlib>

namespace lumen {

// 8 elements of T kept packed in registers as 16-byte words: one for 16-bit T, two for f32.
// (Declared as uint4 words and loaded word by word: a struct of T[8] compiled to per-element
// flat loads plus scratch on the bf16 path, 26 -> 39 us per training-shape call.)
template <typename T> struct Pack8 {
  static constexpr int W = 8 * sizeof(T) / 16;
  uint4 w[W];
  __device__ __forceinline__ void load(const T* p, bool ok) {
#pragma unroll
    for (int i = 0; i < W; ++i)
      w[i] = ok ? reinterpret_cast<const uint4*>(p)[i] : make_uint4(0, 0, 0, 0);
  }
  __device__ __forceinline__ const T* v() const { return reinterpret_cast<const T*>(w); }
};

template <typename T, int VPL, int WPR = 1>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ residual, const T* __restrict__ w,
    T* __restrict__ y, T* __restrict__ s_out, float* __restrict__ rstd_out, int rows, int H,
    float eps, long long ldy) {
  // WPR waves per row (2 at H > 2048: half the row registers per lane, more waves in flight);
  // their partial sums of squares meet in LDS
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ws = wid % WPR;
  const int row = blockIdx.x * (4 / WPR) + wid / WPR;
  const bool rok = row < rows;  // no early return: the waves of a block meet at a barrier
  const size_t base = static_cast<size_t>(rok ? row : 0) * H;
  // every row load (x, residual, weight) is issued up front, packed, from a clamped address and
  // zeroed afterwards when out of range: loads guarded by `if (rok && c < H)` (and the residual
  // load behind its own branch) compiled to a vmcnt(0) per 16-byte load, serial round trips
  Pack8<T> xr[VPL], rr[VPL], wr[VPL];
  const T* rp = residual ? residual : x;  // a valid row either way; added only with a residual
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int cc = min(((i * WPR + ws) * 64 + lane) * 8, H - 8);
    xr[i].load(x + base + cc, true);
    rr[i].load(rp + base + cc, true);
    wr[i].load(w + cc, true);
  }
  float v[VPL][8], wv[VPL][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = ((i * WPR + ws) * 64 + lane) * 8;
    const bool ok = rok && c < H;
    const T* xe = xr[i].v();
    const T* re = rr[i].v();
    const T* we = wr[i].v();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = to_f32(xe[j]);
      if (residual) t += to_f32(re[j]);
      v[i][j] = ok ? t : 0.f;
      wv[i][j] = to_f32(we[j]);
      ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  if (WPR > 1) {
    if (lane == 0) part[wid] = ss;
    __syncthreads();
    ss = 0.f;
#pragma unroll
    for (int k = 0; k < WPR; ++k) ss += part[(wid / WPR) * WPR + k];
  }
  const float rs = rsqrtf(ss / static_cast<float>(H) + eps);
  if (rok && lane == 0 && ws == 0 && rstd_out) rstd_out[row] = rs;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = ((i * WPR + ws) * 64 + lane) * 8;
    if (rok && c < H) {
      if (s_out) {
        // round the residual stream to the activation dtype first: the normalisation below
        // must see exactly the value the next layer reads back.
        float sr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sr[j] = to_f32(from_f32<T>(v[i][j]));
        store8(s_out + base + c, sr);
      }
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rs * wv[i][j];
      store8(y + static_cast<size_t>((rok ? row : 0)) * ldy + c, o);
    }
  }
}

// Few rows (decode: 1..512 tokens): a whole 256-thread workgroup per row, so each lane issues
// VPT (= H / 2048) loads instead of H / 512 and the row reaches HBM / L2 with 4x the parallelism
// (batch-1 decode: 10 -> a few us per call, 65 calls per token).
template <typename T, int VPT>
__global__ void __launch_bounds__(256) rmsnorm_fwd_row_kernel(
    const T* __restrict__ x, const T* __restrict__ residual, const T* __restrict__ w,
    T* __restrict__ y, T* __restrict__ s_out, float* __restrict__ rstd_out, int rows, int H,
    float eps, long long ldy) {
  __shared__ float part[4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row = blockIdx.x;
  const size_t base = static_cast<size_t>(row) * H;
  // all loads up front, unconditional from clamped addresses (see rmsnorm_fwd_kernel)
  Pack8<T> xr[VPT], rr[VPT], wr[VPT];
  const T* rp = residual ? residual : x;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int cc = min((tid + i * 256) * 8, H - 8);
    xr[i].load(x + base + cc, true);
    rr[i].load(rp + base + cc, true);
    wr[i].load(w + cc, true);
  }
  float v[VPT][8], wv[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const bool ok = (tid + i * 256) * 8 < H;
    const T* xe = xr[i].v();
    const T* re = rr[i].v();
    const T* we = wr[i].v();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = to_f32(xe[j]);
      if (residual) t += to_f32(re[j]);
      v[i][j] = ok ? t : 0.f;
      wv[i][j] = to_f32(we[j]);
      ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) part[wid] = ss;
  __syncthreads();
  ss = part[0] + part[1] + part[2] + part[3];
  const float rs = rsqrtf(ss / static_cast<float>(H) + eps);
  if (tid == 0 && rstd_out) rstd_out[row] = rs;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (tid + i * 256) * 8;
    if (c < H) {
      if (s_out) {
        float sr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sr[j] = to_f32(from_f32<T>(v[i][j]));
        store8(s_out + base + c, sr);
      }
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rs * wv[i][j];
      store8(y + static_cast<size_t>(row) * ldy + c, o);
    }
  }
}

template <typename T, int VPL, int WPR>
__global__ void __launch_bounds__(256) rmsnorm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ s, const T* __restrict__ w,
    const float* __restrict__ rstd, const T* __restrict__ ds_res, T* __restrict__ dx,
    float* __restrict__ dw, int rows, int H) {
  // All row loads (dy, s and the residual-stream gradient) are issued up front and kept packed
  // (16-bit) in registers, so the reduction and the write-back never wait on a second round of
  // HBM latency.  WPR waves share a row (WPR = 2 at H = 4096: 48 instead of 96 VGPRs of row
  // data per lane, twice the waves in flight -- one wave per row measured 4.3 TB/s against the
  // forward's 5.4); their partial dot products meet in LDS.
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ws = wid % WPR;
  const int row = blockIdx.x * (4 / WPR) + wid / WPR;
  const bool rok = row < rows;  // no early return: the waves of a block meet at a barrier
  const size_t base = static_cast<size_t>(rok ? row : 0) * H;
  const float rs = rok ? rstd[row] : 0.f;
  // the norm weight is loaded with the rows (it was a guarded load8 in both passes below: four
  // serial L2 round trips per wave after the rows had landed)
  Pack8<T> dyr[VPL], sr[VPL], rr[VPL], wr[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = ((i * WPR + ws) * 64 + lane) * 8;
    const bool ok = rok && c < H;
    dyr[i].load(dy + base + c, ok);
    sr[i].load(s + base + c, ok);
    rr[i].load(ds_res + base + c, ok && ds_res);
    wr[i].load(w + min(c, H - 8), true);
  }
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = ((i * WPR + ws) * 64 + lane) * 8;
    if (rok && c < H) {
      const T* dyv = dyr[i].v();
      const T* sv = sr[i].v();
      const T* wv = wr[i].v();
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += to_f32(dyv[j]) * to_f32(wv[j]) * (to_f32(sv[j]) * rs);
      if (dw) {
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(dw + c + j, to_f32(dyv[j]) * to_f32(sv[j]) * rs);
      }
    }
  }
  dot = wave_sum(dot);
  if (WPR > 1) {
    if (lane == 0) part[wid] = dot;
    __syncthreads();
    dot = 0.f;
#pragma unroll
    for (int k = 0; k < WPR; ++k) dot += part[(wid / WPR) * WPR + k];
  }
  dot /= static_cast<float>(H);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = ((i * WPR + ws) * 64 + lane) * 8;
    if (rok && c < H) {
      const T* dyv = dyr[i].v();
      const T* sv = sr[i].v();
      const T* rv = rr[i].v();
      const T* wv = wr[i].v();
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = rs * (to_f32(dyv[j]) * to_f32(wv[j]) - to_f32(sv[j]) * rs * dot);
        if (ds_res) o[j] += to_f32(rv[j]);
      }
      store8(dx + base + c, o);
    }
  }
}

// Occupancy caps (dynamic LDS bytes reserved per workgroup, 0 = none).  At the training shape
// (4096 rows x 4096) the backward grid is 2048 workgroups = 8 per CU, all resident at once:
// every workgroup loads, reduces and stores in the same phase, so HBM reads and writes do not
// overlap.  Capping residency gives a second round whose loads run under the first's stores.
static int g_rms_lds[2] = {0, 0};  // [fwd, bwd]

template <typename T>
static hipError_t launch_fwd(const void* x, const void* res, const void* w, void* y, void* s_out,
                             float* rstd, int rows, int H, float eps, long long ldy,
                             hipStream_t st) {
  dim3 block(256);
  // LUMEN_RMS_FWD_WPR=4: the workgroup-per-row kernel at every row count (A/B switch; slower at
  // the training shape, profiles/r3d/rmsnorm)
  static const bool env_row = [] {
    const char* e = getenv("LUMEN_RMS_FWD_WPR");
    return e && atoi(e) == 4;
  }();
  if ((rows < 1024 || env_row) && H <= 8192) {  // under ~4 waves per CU: one workgroup per row
    dim3 grid(rows);
    const int vpt = (H + 2047) / 2048;
#define LUMEN_RMS_ROW(V)                                                                          \
  hipLaunchKernelGGL((rmsnorm_fwd_row_kernel<T, V>), grid, block, 0, st, (const T*)x,            \
                     (const T*)res, (const T*)w, (T*)y, (T*)s_out, rstd, rows, H, eps, ldy)
    if (vpt <= 1) LUMEN_RMS_ROW(1);
    else if (vpt <= 2) LUMEN_RMS_ROW(2);
    else LUMEN_RMS_ROW(4);
#undef LUMEN_RMS_ROW
    return hipGetLastError();
  }
  // two waves per row above H = 2048 (LUMEN_RMS_FWD_WPR=1: one)
  static const int env_wpr = [] {
    const char* e = getenv("LUMEN_RMS_FWD_WPR");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  const int wpr = H > 2048 ? env_wpr : 1;
  dim3 grid((rows + 4 / wpr - 1) / (4 / wpr));
  const int vpl = (H + 512 * wpr - 1) / (512 * wpr);
#define LUMEN_RMS_FWD(V, W)                                                                       \
  hipLaunchKernelGGL((rmsnorm_fwd_kernel<T, V, W>), grid, block, g_rms_lds[0], st, (const T*)x,  \
                     (const T*)res, (const T*)w, (T*)y, (T*)s_out, rstd, rows, H, eps, ldy)
  if (wpr == 1) {
    if (vpl <= 1) LUMEN_RMS_FWD(1, 1);
    else if (vpl <= 2) LUMEN_RMS_FWD(2, 1);
    else if (vpl <= 4) LUMEN_RMS_FWD(4, 1);
    else if (vpl <= 8) LUMEN_RMS_FWD(8, 1);
    else if (vpl <= 16) LUMEN_RMS_FWD(16, 1);
    else return hipErrorInvalidValue;
  } else {
    if (vpl <= 4) LUMEN_RMS_FWD(4, 2);
    else if (vpl <= 8) LUMEN_RMS_FWD(8, 2);
    else return hipErrorInvalidValue;
  }
#undef LUMEN_RMS_FWD
  return hipGetLastError();
}


template <typename T>
static hipError_t launch_bwd(const void* dy, const void* s, const void* w, const float* rstd,
                             const void* ds_res, void* dx, float* dw, int rows, int H,
                             hipStream_t st) {
  dim3 block(256);
  // four waves per row (one row per workgroup) once a row needs more than 4 vectors per lane
  // (H > 2048): Llama-2-7B training rows 29.4 -> 26.0 us per call against two waves per row
  // (profiles/r3d/rmsnorm; the forward measured the opposite way, 24.3 vs 25.9 us, and keeps
  // two).  LUMEN_RMS_BWD_WPR=2: two.
  static const int env_bwd_wpr = [] {
    const char* e = getenv("LUMEN_RMS_BWD_WPR");
    return e && atoi(e) == 2 ? 2 : 4;
  }();
  const int wpr = H > 2048 ? env_bwd_wpr : 1;
  dim3 grid((rows + 4 / wpr - 1) / (4 / wpr));
  const int vpl = (H + 512 * wpr - 1) / (512 * wpr);
#define LUMEN_RMS_BWD(V, W)                                                                     \
  hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, V, W>), grid, block, g_rms_lds[1], st, (const T*)dy, \
                     (const T*)s, (const T*)w, rstd, (const T*)ds_res, (T*)dx, dw, rows, H)
  if (wpr == 1) {
    if (vpl <= 1) LUMEN_RMS_BWD(1, 1);
    else if (vpl <= 2) LUMEN_RMS_BWD(2, 1);
    else LUMEN_RMS_BWD(4, 1);
  } else if (wpr == 2) {
    if (vpl <= 4) LUMEN_RMS_BWD(4, 2);
    else if (vpl <= 8) LUMEN_RMS_BWD(8, 2);
    else if (vpl <= 16) LUMEN_RMS_BWD(16, 2);
    else return hipErrorInvalidValue;
  } else {
    if (vpl <= 2) LUMEN_RMS_BWD(2, 4);
    else if (vpl <= 4) LUMEN_RMS_BWD(4, 4);
    else if (vpl <= 8) LUMEN_RMS_BWD(8, 4);
    else return hipErrorInvalidValue;
  }
#undef LUMEN_RMS_BWD
  return hipGetLastError();
}

}  // namespace lumen

// y rows may be strided (ldy >= H): the q|k|v input of a K-extended LoRA GEMM is written straight
// into the first H columns of its [rows, H + 64] operand buffer
extern "C" void lumen_set_rms_lds(int fwd_bytes, int bwd_bytes) {
  lumen::g_rms_lds[0] = fwd_bytes < 0 ? 0 : fwd_bytes;
  lumen::g_rms_lds[1] = bwd_bytes < 0 ? 0 : bwd_bytes;
}

extern "C" hipError_t lumen_rmsnorm_fwd_ld(int dtype, const void* x, const void* residual,
                                           const void* w, void* y, void* s_out, float* rstd,
                                           int rows, int H, float eps, long long ldy,
                                           hipStream_t st) {
  if (H % 8 != 0 || ldy < H || (ldy % 8) != 0) return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::launch_fwd<lumen::bf16>(x, residual, w, y, s_out, rstd, rows, H, eps, ldy, st);
  if (dtype == lumen::kF16)
    return lumen::launch_fwd<lumen::fp16>(x, residual, w, y, s_out, rstd, rows, H, eps, ldy, st);
  if (dtype == lumen::kF32)
    return lumen::launch_fwd<float>(x, residual, w, y, s_out, rstd, rows, H, eps, ldy, st);
  return hipErrorInvalidValue;
}

extern "C" hipError_t lumen_rmsnorm_fwd(int dtype, const void* x, const void* residual,
                                        const void* w, void* y, void* s_out, float* rstd, int rows,
                                        int H, float eps, hipStream_t st) {
  return lumen_rmsnorm_fwd_ld(dtype, x, residual, w, y, s_out, rstd, rows, H, eps, H, st);
}

extern "C" hipError_t lumen_rmsnorm_bwd(int dtype, const void* dy, const void* s, const void* w,
                                        const float* rstd, const void* ds_res, void* dx, float* dw,
                                        int rows, int H, hipStream_t st) {
  if (H % 8 != 0) return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::launch_bwd<lumen::bf16>(dy, s, w, rstd, ds_res, dx, dw, rows, H, st);
  if (dtype == lumen::kF16)
    return lumen::launch_bwd<lumen::fp16>(dy, s, w, rstd, ds_res, dx, dw, rows, H, st);
  if (dtype == lumen::kF32)
    return lumen::launch_bwd<float>(dy, s, w, rstd, ds_res, dx, dw, rows, H, st);
  return hipErrorInvalidValue;
}
