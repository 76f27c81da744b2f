// Optimizer kernels: grad L2-norm / overflow check and fused AdamW.
//
// Reference behaviour: DeepSpeed FusedAdam / torch AdamW with betas (0.9, 0.999), eps 1e-8,
// weight_decay 0 (configs/ds_config_zero1.json:6-14), gradient_clipping 1.0
// (configs/ds_config_zero1.json:44) and fp16 dynamic loss scaling
// (configs/ds_config_zero1.json:25-32) -- i.e. unscale, has_inf_or_nan, global-norm clip and the
// Adam update as separate multi-tensor passes plus a host sync per step.
//
// Here the trainable state lives in ONE flat f32 buffer per rank (the ZeRO partition), so
//  * `grad_norm_sq` is a single grid-stride reduction -> one f32 on device (RCCL all-reduces it
//    across ranks when sharded); a non-finite sum doubles as the overflow flag;
//  * `adamw_step` reads that device scalar and folds unscale (1/loss_scale), clip coefficient
//    min(1, max_norm/||g||) and the skip-on-overflow decision into the update itself, so a bf16
//    step needs no device->host synchronisation at all; optionally it writes a 16-bit copy of the
//    updated parameters in the same pass (the "fp32 master -> bf16 model" copy-out).
#include "common.h"
#include "det.h"

#include <algorithm>

namespace lumen {

// Device-side optimizer schedule (optional).  ``state`` (f32, 8 words):
//   [0] applied updates  [1] skipped steps  [2] loss scale  [3] current hysteresis
//   [4] scaler iteration [5] last overflow iteration
// When present, the Adam bias corrections, the WarmupLR learning rate (DeepSpeed semantics: the
// scheduler advances only on applied steps, warm-up length clamped to >= 2) and the loss-scale
// unscale all come from device memory, and adamw_commit_kernel advances the counters and the
// DynamicLossScaler after the update -- so neither a bf16 nor an fp16 step syncs the host.
struct OptSched {
  float* state;
  float lr_min, lr_max;
  int warm_n, warm_linear;
  float inv_world;
  int dynamic_scale;
  float scale_window;
  int hysteresis;
  float min_scale;
  float decay_total;  // > 0: a decaying schedule over this many steps (kind below)
  int decay_kind;     // 0: HF get_linear_schedule_with_warmup; 1: DeepSpeed WarmupDecayLR;
                      // 2: DeepSpeed WarmupCosineLR (lr_min = warmup_min_ratio * lr_max)
  float cos_min;      // WarmupCosineLR cos_min_ratio
};

__device__ __forceinline__ float sched_lr(const OptSched& s, float it) {
  if (s.decay_total > 0.f && s.decay_kind > 0) {
    // DeepSpeed WarmupDecayLR / WarmupCosineLR: the WarmupLR warm-up (length clamped to >= 2,
    // log or linear from lr_min), then a linear (to lr_min) or cosine (to cos_min * lr_max)
    // decay reaching its floor at decay_total
    const float n = (float)(s.warm_n > 2 ? s.warm_n : 2);
    if (it < n) {
      const float gamma = s.warm_linear ? it / n : logf(it + 1.f) / logf(n);
      return s.lr_min + (s.lr_max - s.lr_min) * gamma;
    }
    if (s.decay_kind == 1)
      return s.lr_min + (s.lr_max - s.lr_min) *
                            fmaxf(0.f, (s.decay_total - it) / fmaxf(1.f, s.decay_total - n));
    const float c = 0.5f * (1.f + cosf(3.14159265358979f * (it - n + 1.f) /
                                       fmaxf(1.f, s.decay_total - n)));
    return s.lr_max * fmaxf(0.f, s.cos_min + (1.f - s.cos_min) * c);
  }
  if (s.decay_total > 0.f) {
    // HF Trainer's default (no DeepSpeed scheduler): linear warm-up from 0, then linear decay
    // to 0 at decay_total (transformers get_linear_schedule_with_warmup)
    const float w = (float)s.warm_n;
    if (it < w) return s.lr_max * it / w;
    return s.lr_max * fmaxf(0.f, (s.decay_total - it) / fmaxf(1.f, s.decay_total - w));
  }
  const float n = (float)(s.warm_n > 2 ? s.warm_n : 2);
  if (it >= n) return s.lr_max;
  const float gamma = s.warm_linear ? it / n : logf(it + 1.f) / logf(n);
  return s.lr_min + (s.lr_max - s.lr_min) * gamma;
}

// deterministic block sum (det.h): one partial per workgroup, the last arriver adds them to *out
// in block order (at most 512 workgroups; one norm_sq launch at a time, as the engine issues it)
constexpr int kNormMaxBlocks = 512;
__device__ float g_norm_slab[kNormMaxBlocks];
__device__ unsigned g_norm_cnt;

template <typename G>
__global__ void __launch_bounds__(256) norm_sq_kernel(const G* __restrict__ g, long long n,
                                                      float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  // whole 8-element chunks, four per trip with every load issued before the first use, from
  // clamped chunk indices (the guarded one-chunk loop waited out each load in turn: 35.6 us for
  // the 16.8 M LoRA gradients of Llama-2-7B); the < 8 tail elements go to block 0
  const long long n8 = n / 8;
  const long long S = static_cast<long long>(gridDim.x) * 256;
  for (long long c0 = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x; c0 < n8;
       c0 += 4 * S) {
    float x[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8(g + min(c0 + u * S, n8 - 1) * 8, x[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[u][j] * x[u][j];
      acc += c0 + u * S < n8 ? s : 0.f;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < n - n8 * 8) {
    const float t = to_f32(g[n8 * 8 + threadIdx.x]);
    acc += t * t;
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) det::st_wt(g_norm_slab + blockIdx.x, acc);
  __shared__ int lastf;
  if (!det::last_arriver(&g_norm_cnt, gridDim.x, &lastf)) return;
  if (threadIdx.x < 64) {
    float v = 0.f;
    for (int b = threadIdx.x; b < static_cast<int>(gridDim.x); b += 64) v += det::ld_wt(g_norm_slab + b);
    v = wave_sum(v);  // fixed butterfly order
    if (threadIdx.x == 0) *out += v;
  }
}

template <typename G, typename O>
__global__ void __launch_bounds__(256) adamw_kernel(
    float* __restrict__ p, const G* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    O* __restrict__ out_copy, long long n, float lr, float beta1, float beta2, float eps, float wd,
    float bc1, float bc2, float inv_scale, const float* __restrict__ norm_sq, float max_norm,
    OptSched sc) {
  if (sc.state) {
    // device-side step counter: t = applied updates so far + 1, so a skipped (non-finite) step
    // never advances the bias correction or the LR schedule (adamw_commit_kernel counts it)
    const float applied = sc.state[0];
    const float t = applied + 1.f;
    bc1 = 1.f - powf(beta1, t);
    bc2 = 1.f - powf(beta2, t);
    lr = sched_lr(sc, applied);
    inv_scale = sc.inv_world / sc.state[2];
  }
  float coef = inv_scale;
  if (norm_sq) {
    const float nsq = *norm_sq;
    if (!isfinite(nsq)) return;  // overflow: skip the step (loss scaler backs off on the host)
    if (max_norm > 0.f) {
      const float gn = sqrtf(nsq) * inv_scale;
      if (gn > max_norm) coef *= max_norm / (gn + 1e-6f);
    }
  }
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const long long stride = static_cast<long long>(gridDim.x) * 256 * 8;
  for (long long i = (static_cast<long long>(blockIdx.x) * 256 + threadIdx.x) * 8; i < n;
       i += stride) {
    if (i + 8 <= n) {
      float pv[8], gv[8], mv[8], vv[8];
      load8(p + i, pv);
      load8(g + i, gv);
      load8(m + i, mv);
      load8(v + i, vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gg = gv[j] * coef;
        mv[j] = beta1 * mv[j] + (1.f - beta1) * gg;
        vv[j] = beta2 * vv[j] + (1.f - beta2) * gg * gg;
        pv[j] -= lr * wd * pv[j];
        const float denom = sqrtf(vv[j]) / bc2_sqrt + eps;
        pv[j] -= step_size * mv[j] / denom;
      }
      store8(p + i, pv);
      store8(m + i, mv);
      store8(v + i, vv);
      if (out_copy) store8(out_copy + i, pv);
    } else {
      for (long long j = i; j < n; ++j) {
        const float gg = to_f32(g[j]) * coef;
        m[j] = beta1 * m[j] + (1.f - beta1) * gg;
        v[j] = beta2 * v[j] + (1.f - beta2) * gg * gg;
        float pp = p[j] - lr * wd * p[j];
        pp -= step_size * m[j] / (sqrtf(v[j]) / bc2_sqrt + eps);
        p[j] = pp;
        if (out_copy) out_copy[j] = from_f32<O>(pp);
      }
    }
  }
}

// after adamw_kernel: count the step as applied (state[0]) or skipped (state[1]) and advance the
// dynamic loss scaler (DeepSpeed DynamicLossScaler, consecutive_hysteresis = false)
__global__ void adamw_commit_kernel(OptSched sc, const float* __restrict__ norm_sq) {
  if (threadIdx.x != 0) return;
  float* st = sc.state;
  const bool overflow = norm_sq != nullptr && !isfinite(*norm_sq);
  st[overflow ? 1 : 0] += 1.f;
  if (!sc.dynamic_scale) return;
  const float it = st[4];
  if (overflow) {
    if (sc.hysteresis == 1 || st[3] <= 1.f) st[2] = fmaxf(st[2] * 0.5f, sc.min_scale);
    else st[3] -= 1.f;
    st[5] = it;
  } else if (fmodf(it - st[5], sc.scale_window) == 0.f) {
    st[2] *= 2.f;
    st[3] = (float)sc.hysteresis;
  }
  st[4] = it + 1.f;
}

static inline unsigned grid_for(long long n) {
  long long blocks = (n + 256 * 8 - 1) / (256 * 8);
  if (blocks > 2048) blocks = 2048;  // grid-stride the rest
  if (blocks < 1) blocks = 1;
  return static_cast<unsigned>(blocks);
}

}  // namespace lumen

// out must be zeroed by the caller (it accumulates, so several buffers can share one scalar).
extern "C" hipError_t lumen_grad_norm_sq(int gdtype, const void* g, long long n, float* out,
                                         hipStream_t st) {
  if (n == 0) return hipSuccess;
  // at most 2 workgroups per CU: every workgroup ends in one f32 atomic on the same scalar, and
  // 2048 of them serialise at the L2 (31.5 us for 16.8 M elements with the adamw grid)
  dim3 grid(std::min(lumen::grid_for(n), 512u)), block(256);
  if (gdtype == lumen::kF32)
    hipLaunchKernelGGL(lumen::norm_sq_kernel<float>, grid, block, 0, st, (const float*)g, n, out);
  else if (gdtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::norm_sq_kernel<lumen::bf16>, grid, block, 0, st,
                       (const lumen::bf16*)g, n, out);
  else if (gdtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::norm_sq_kernel<lumen::fp16>, grid, block, 0, st,
                       (const lumen::fp16*)g, n, out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t lumen_adamw(float* p, int gdtype, const void* g, float* m, float* v,
                                  int out_dtype, void* out_copy, long long n, float lr,
                                  float beta1, float beta2, float eps, float wd, float bc1,
                                  float bc2, float inv_scale, const float* norm_sq, float max_norm,
                                  float* step_state, const double* sched, hipStream_t st) {
  lumen::OptSched sc{};
  sc.state = step_state;
  if (step_state) {
    // sched: lr_min, lr_max, warm_n, warm_linear, inv_world, dynamic, window, hysteresis, min,
    // decay_total, decay_kind, cos_min (the binding pads the list to 12 values)
    sc.lr_min = (float)sched[0];
    sc.lr_max = (float)sched[1];
    sc.warm_n = (int)sched[2];
    sc.warm_linear = (int)sched[3];
    sc.inv_world = (float)sched[4];
    sc.dynamic_scale = (int)sched[5];
    sc.scale_window = (float)sched[6];
    sc.hysteresis = (int)sched[7];
    sc.min_scale = (float)sched[8];
    sc.decay_total = (float)sched[9];
    sc.decay_kind = (int)sched[10];
    sc.cos_min = (float)sched[11];
  }
  if (n == 0) return hipSuccess;
  dim3 grid(lumen::grid_for(n)), block(256);
#define LUMEN_ADAMW(G, O)                                                                    \
  hipLaunchKernelGGL((lumen::adamw_kernel<G, O>), grid, block, 0, st, p, (const G*)g, m, v, \
                     (O*)out_copy, n, lr, beta1, beta2, eps, wd, bc1, bc2, inv_scale, norm_sq,  \
                     max_norm, sc)
  if (gdtype == lumen::kF32) {
    if (out_copy == nullptr || out_dtype == lumen::kF32) LUMEN_ADAMW(float, float);
    else if (out_dtype == lumen::kBF16) LUMEN_ADAMW(float, lumen::bf16);
    else LUMEN_ADAMW(float, lumen::fp16);
  } else if (gdtype == lumen::kBF16) {
    if (out_copy == nullptr || out_dtype == lumen::kF32) LUMEN_ADAMW(lumen::bf16, float);
    else if (out_dtype == lumen::kBF16) LUMEN_ADAMW(lumen::bf16, lumen::bf16);
    else LUMEN_ADAMW(lumen::bf16, lumen::fp16);
  } else if (gdtype == lumen::kF16) {
    if (out_copy == nullptr || out_dtype == lumen::kF32) LUMEN_ADAMW(lumen::fp16, float);
    else if (out_dtype == lumen::kBF16) LUMEN_ADAMW(lumen::fp16, lumen::bf16);
    else LUMEN_ADAMW(lumen::fp16, lumen::fp16);
  } else {
    return hipErrorInvalidValue;
  }
#undef LUMEN_ADAMW
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || step_state == nullptr) return e;
  hipLaunchKernelGGL(lumen::adamw_commit_kernel, dim3(1), dim3(64), 0, st, sc, norm_sq);
  return hipGetLastError();
}
