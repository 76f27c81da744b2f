// Host AdamW for ZeRO-Offload.
//
// Reference behaviour: DeepSpeedCPUAdam (C++ SIMD + OpenMP), selected by
// `"offload_optimizer": {"device": "cpu", "pin_memory": true}` (configs/ds_config_zero3.json:19-22).
// The f32 master/m/v partition lives in pinned host memory; the gradient shard arrives by async
// D2H copy, this kernel updates in place, and the new parameters go back by H2D copy.
//
// AVX-512 path chosen at run time (the GPU box's host CPU is not known at build time); the
// portable path is a plain loop the compiler vectorises for the baseline ISA.  OpenMP splits the
// partition over host threads.
#include <cmath>
#include <cstdint>
#include <immintrin.h>

namespace {

inline void adam_scalar(float* p, const float* g, float* m, float* v, long long i0, long long i1,
                        float lr, float b1, float b2, float eps, float wd, float bc1, float bc2,
                        float gs) {
  const float step = lr / bc1, sb2 = std::sqrt(bc2);
  for (long long i = i0; i < i1; ++i) {
    const float gg = g[i] * gs;
    m[i] = b1 * m[i] + (1.f - b1) * gg;
    v[i] = b2 * v[i] + (1.f - b2) * gg * gg;
    float pp = p[i] - lr * wd * p[i];
    pp -= step * m[i] / (std::sqrt(v[i]) / sb2 + eps);
    p[i] = pp;
  }
}

__attribute__((target("avx512f"))) void adam_avx512(float* p, const float* g, float* m, float* v,
                                                     long long i0, long long i1, float lr, float b1,
                                                     float b2, float eps, float wd, float bc1,
                                                     float bc2, float gs) {
  const __m512 vb1 = _mm512_set1_ps(b1), vb2 = _mm512_set1_ps(b2);
  const __m512 vb1c = _mm512_set1_ps(1.f - b1), vb2c = _mm512_set1_ps(1.f - b2);
  const __m512 vgs = _mm512_set1_ps(gs), veps = _mm512_set1_ps(eps);
  const __m512 vdecay = _mm512_set1_ps(1.f - lr * wd);
  const __m512 vstep = _mm512_set1_ps(lr / bc1), vinv_sb2 = _mm512_set1_ps(1.f / std::sqrt(bc2));
  long long i = i0;
  for (; i + 16 <= i1; i += 16) {
    __m512 gg = _mm512_mul_ps(_mm512_loadu_ps(g + i), vgs);
    __m512 mm = _mm512_fmadd_ps(vb1, _mm512_loadu_ps(m + i), _mm512_mul_ps(vb1c, gg));
    __m512 vv = _mm512_fmadd_ps(vb2, _mm512_loadu_ps(v + i), _mm512_mul_ps(vb2c, _mm512_mul_ps(gg, gg)));
    __m512 pp = _mm512_mul_ps(_mm512_loadu_ps(p + i), vdecay);
    __m512 den = _mm512_add_ps(_mm512_mul_ps(_mm512_sqrt_ps(vv), vinv_sb2), veps);
    pp = _mm512_sub_ps(pp, _mm512_div_ps(_mm512_mul_ps(vstep, mm), den));
    _mm512_storeu_ps(m + i, mm);
    _mm512_storeu_ps(v + i, vv);
    _mm512_storeu_ps(p + i, pp);
  }
  adam_scalar(p, g, m, v, i, i1, lr, b1, b2, eps, wd, bc1, bc2, gs);
}

bool has_avx512() {
#ifdef LUMEN_NO_AVX512  // sanitizer harness: exercise the portable path too
  return false;
#else
  static const int cached = __builtin_cpu_supports("avx512f") ? 1 : 0;
  return cached != 0;
#endif
}

}  // namespace

extern "C" int lumen_cpu_has_avx512() { return has_avx512() ? 1 : 0; }

extern "C" void lumen_cpu_adamw(float* p, const float* g, float* m, float* v, long long n,
                                float lr, float b1, float b2, float eps, float wd, float bc1,
                                float bc2, float grad_scale) {
  const bool avx = has_avx512();
  const long long chunk = 1 << 16;
  const long long nchunks = (n + chunk - 1) / chunk;
#pragma omp parallel for schedule(static)
  for (long long c = 0; c < nchunks; ++c) {
    const long long i0 = c * chunk, i1 = (i0 + chunk < n) ? i0 + chunk : n;
    if (avx) adam_avx512(p, g, m, v, i0, i1, lr, b1, b2, eps, wd, bc1, bc2, grad_scale);
    else adam_scalar(p, g, m, v, i0, i1, lr, b1, b2, eps, wd, bc1, bc2, grad_scale);
  }
}
