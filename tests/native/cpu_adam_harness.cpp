// Host sanitizer harness for lumen/csrc/cpu/cpu_adam.cpp ("host ASan for the C++
// CPU-Adam extension").  Built by tests/test_native_sanitizers.py with
// -fsanitize=address,undefined; every buffer is an exact-size heap allocation, so an
// out-of-bounds vector tail, a chunk-boundary off-by-one or a misaligned access aborts the run.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" void lumen_cpu_adamw(float* p, const float* g, float* m, float* v, long long n,
                                float lr, float b1, float b2, float eps, float wd, float bc1,
                                float bc2, float grad_scale);

int main() {
  const long long sizes[] = {1, 15, 16, 17, 65535, 65536, 65537, 200003};
  int bad = 0;
  for (long long n : sizes) {
    float* p = new float[n];
    float* g = new float[n];
    float* m = new float[n];
    float* v = new float[n];
    std::vector<double> rp(n), rm(n), rv(n);
    for (long long i = 0; i < n; ++i) {
      p[i] = 0.01f * static_cast<float>((i * 37) % 101 - 50);
      g[i] = 0.001f * static_cast<float>((i * 11) % 61 - 30);
      m[i] = 0.f;
      v[i] = 0.f;
      rp[i] = p[i];
      rm[i] = 0.0;
      rv[i] = 0.0;
    }
    const float lr = 1e-3f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.01f, gs = 0.5f;
    for (int t = 1; t <= 3; ++t) {
      const float bc1 = 1.f - std::pow(b1, t), bc2 = 1.f - std::pow(b2, t);
      lumen_cpu_adamw(p, g, m, v, n, lr, b1, b2, eps, wd, bc1, bc2, gs);
      for (long long i = 0; i < n; ++i) {  // double-precision reference of the same update
        const double gg = static_cast<double>(g[i]) * gs;
        rm[i] = b1 * rm[i] + (1.0 - b1) * gg;
        rv[i] = b2 * rv[i] + (1.0 - b2) * gg * gg;
        rp[i] = rp[i] - lr * wd * rp[i];
        rp[i] -= (lr / bc1) * rm[i] / (std::sqrt(rv[i]) / std::sqrt(bc2) + eps);
      }
    }
    double err = 0.0;
    for (long long i = 0; i < n; ++i) err = std::fmax(err, std::fabs(p[i] - rp[i]));
    if (!(err < 1e-5)) {
      std::printf("n=%lld max err %g\n", n, err);
      bad = 1;
    }
    delete[] p;
    delete[] g;
    delete[] m;
    delete[] v;
  }
  std::printf(bad ? "FAIL\n" : "OK\n");
  return bad;
}
