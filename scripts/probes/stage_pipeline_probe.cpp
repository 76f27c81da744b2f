// The decode GEMM's staging pipeline without its math (M = 256 q|k|v: BM 256, BN 128, split-K 2,
// 192 blocks of 8 waves, 3-stage LDS ring of k64 stages = 48 KB each):
//   mode 0: LDS-DMA (global_load_lds_dwordx4), two stages in flight, counted vmcnt + barrier
//           per stage -- the shipped kernels/decode_gemm.hip structure;
//   mode 1: register staging, one stage in flight (loads for t+1 issued before stage t's
//           ds_reads, written to LDS after them), barrier per stage;
//   mode 2: register staging, two register sets (stages t+1 and t+2 in flight);
//   RD = 1: every wave also ds_reads the stage as the MFMA loop would (the LDS read traffic).
// Weights rotate over > 512 MB.  Prints us per launch.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/spp scripts/probes/stage_pipeline_probe.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("hip error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int BM = 256, BN = 128, ROWS = BM + BN, ROWB = 128, STAGE = ROWS * ROWB;
constexpr int NT = 512, NW = 8, PER = ROWS * 8 / NT;  // 6 16-byte chunks per thread per stage

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void dma16(const void* base, unsigned off, const char* lds) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(lds))));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(off), "s"(base), "s"(m0) : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0xF70);
}

__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// source of chunk (row r, chunk c) of stage k0: W rows [0, BN) then x rows [BN, BN + BM)
__device__ __forceinline__ const uint4* src(const uint4* W, const uint4* x, int K, int r, int c,
                                            int k0) {
  const long long kq = K / 8;
  return r < BN ? W + (long long)r * kq + k0 / 8 + c : x + (long long)(r - BN) * kq + k0 / 8 + c;
}

template <int MODE, int RD>
__global__ void __launch_bounds__(NT, 1) pipe_kernel(const uint4* __restrict__ x,
                                                     const uint4* __restrict__ Wall,
                                                     float* __restrict__ out, int K, int S) {
  __shared__ __attribute__((aligned(16))) char lds[3 * STAGE];
  const int tile = blockIdx.x / S, slice = blockIdx.x - tile * S;
  const int nk = K / 64 / S, kb = slice * nk;
  const uint4* W = Wall + (long long)tile * BN * (K / 8);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float acc = 0.f;
  auto rd = [&](const char* img) {  // the MFMA loop's ds_read_b128 pattern (4 x 2 per wave)
    if (!RD) return;
    const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = (i < 4 ? (wid & 1) * 64 + 16 * i : BN + (wid >> 1) * 64 + 16 * (i - 4)) + lr;
        const uint4 v = *reinterpret_cast<const uint4*>(img + r * ROWB + (((4 * s + lg) ^ swz(r)) << 4));
        acc += __uint_as_float(v.x ^ v.w);
      }
  };
  if (MODE == 0) {
    auto stage = [&](char* img, int k0) {
      const int rr = lane >> 3, c = lane & 7;
#pragma unroll
      for (int q = 0; q < ROWS / 8 / NW; ++q) {
        const int p = NW * q + wid, r = 8 * p + rr, ch = c ^ swz(r);
        const long long kq = K / 8;
        if (8 * p < BN)  // piece-uniform (BN % 8 == 0): the base stays in SGPRs
          dma16(W, (unsigned)(((long long)r * kq + k0 / 8 + ch) * 16), img + 8 * p * ROWB);
        else
          dma16(x, (unsigned)(((long long)(r - BN) * kq + k0 / 8 + ch) * 16), img + 8 * p * ROWB);
      }
    };
    stage(lds, kb * 64);
    if (nk > 1) stage(lds + STAGE, (kb + 1) * 64);
    int buf = 0;
    for (int t = 0; t < nk; ++t) {
      if (t + 1 < nk) wait_vm<ROWS / 8 / NW>(); else wait_vm<0>();
      bar();
      if (t + 2 < nk) stage(lds + (buf >= 1 ? buf - 1 : 2) * STAGE, (kb + t + 2) * 64);
      rd(lds + buf * STAGE);
      buf = buf == 2 ? 0 : buf + 1;
    }
  } else {
    uint4 ra[PER], rb[PER];
    auto ld = [&](uint4 (&r)[PER], int k0) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int q = threadIdx.x + i * NT, row = q >> 3, c = q & 7;
        r[i] = *src(W, x, K, row, c, k0);
      }
    };
    auto st = [&](const uint4 (&r)[PER], char* img) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int q = threadIdx.x + i * NT, row = q >> 3, c = q & 7;
        *reinterpret_cast<uint4*>(img + row * ROWB + ((c ^ swz(row)) << 4)) = r[i];
      }
    };
    ld(ra, kb * 64);
    st(ra, lds);
    if (MODE == 2 && nk > 1) ld(rb, (kb + 1) * 64);
    __syncthreads();
    int buf = 0;
    if (MODE == 1) {
      for (int t = 0; t < nk; ++t) {
        const int nb = buf == 2 ? 0 : buf + 1;
        if (t + 1 < nk) ld(ra, (kb + t + 1) * 64);
        rd(lds + buf * STAGE);
        if (t + 1 < nk) st(ra, lds + nb * STAGE);
        __syncthreads();
        buf = nb;
      }
    } else {
      // two register sets, unrolled by two (a register copy of an in-flight load would wait
      // for it): the set stored at step t holds stage t + 1, the other one receives t + 2
      auto step = [&](int t, uint4 (&issue)[PER], const uint4 (&store)[PER]) {
        const int nb = buf == 2 ? 0 : buf + 1;
        if (t + 2 < nk) ld(issue, (kb + t + 2) * 64);
        rd(lds + buf * STAGE);
        if (t + 1 < nk) st(store, lds + nb * STAGE);
        __syncthreads();
        buf = nb;
      };
      for (int t = 0; t < nk; t += 2) {
        step(t, ra, rb);
        if (t + 1 < nk) step(t + 1, rb, ra);
      }
    }
  }
  out[blockIdx.x * NT + threadIdx.x] = acc;
}

template <int MODE, int RD>
int run(const uint4* x, std::vector<uint4*>& Ws, float* out, int N, int K, int S) {
  const int blocks = (N / BN) * S;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 4; ++i)
    hipLaunchKernelGGL((pipe_kernel<MODE, RD>), dim3(blocks), dim3(NT), 0, 0, x, Ws[i % Ws.size()],
                       out, K, S);
  CK(hipDeviceSynchronize());
  const int iters = 30;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((pipe_kernel<MODE, RD>), dim3(blocks), dim3(NT), 0, 0, x, Ws[i % Ws.size()],
                       out, K, S);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("{\"mode\": %d, \"lds_reads\": %d, \"N\": %d, \"K\": %d, \"S\": %d, \"blocks\": %d, "
              "\"us\": %.2f}\n", MODE, RD, N, K, S, blocks, ms * 1e3 / iters);
  std::fflush(stdout);
  return 0;
}

int main() {
  const int K = 4096, N = 12288, S = 2;
  uint4* x;
  float* out;
  CK(hipMalloc(&x, 256LL * K * 2));
  CK(hipMemset(x, 1, 256LL * K * 2));
  CK(hipMalloc(&out, 4096 * 1024 * sizeof(float)));
  std::vector<uint4*> Ws(6);
  for (auto& w : Ws) {
    CK(hipMalloc(&w, (long long)N * K * 2));
    CK(hipMemset(w, 3, (long long)N * K * 2));
  }
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 0>(x, Ws, out, N, K, S);
    run<1, 0>(x, Ws, out, N, K, S);
    run<2, 0>(x, Ws, out, N, K, S);
    run<0, 1>(x, Ws, out, N, K, S);
    run<1, 1>(x, Ws, out, N, K, S);
    run<2, 1>(x, Ws, out, N, K, S);
  }
  return 0;
}
