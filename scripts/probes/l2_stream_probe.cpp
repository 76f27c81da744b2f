// Load-path ceiling of the M = 256 decode projection's access pattern, without LDS or MFMA.
//
// Each block reads x[0:256, krange] (2 MB matrix shared by every block: L2 / Infinity-Cache
// hits) and W[n0:n0+BN, krange] (its private weight rows, streamed from HBM: the weights rotate
// over > 512 MB), exactly the bytes a (BM = 256, BN, split-K S) decode-GEMM block stages, with
// plain global_load_dwordx4 into registers.  U k-steps of loads are issued before any is used
// (XOR-folded so the loads stay live).  Prints us per launch and GB/s per block.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/l2p scripts/probes/l2_stream_probe.cpp && /tmp/l2p
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

template <int NT, int U, bool XONLY, bool WONLY, bool WT = false>
__global__ void __launch_bounds__(NT) stream_kernel(const uint4* __restrict__ x,
                                                    const uint4* __restrict__ W,
                                                    unsigned* __restrict__ out, int K, int BN,
                                                    int S) {
  // rows of a step: 256 x rows then BN W rows; 8 16-byte chunks per row and k-step of 64
  const int tile = blockIdx.x / S, slice = blockIdx.x - tile * S;
  const int ksteps = K / 64 / S;
  const int kc0 = slice * ksteps * 8;      // first 16-byte chunk column of this slice
  const int rows = (XONLY ? 256 : 0) + (WONLY ? BN : 0);
  const int chunks = rows * 8;             // per step
  const int per = (chunks + NT - 1) / NT;  // loads per thread per step
  const long long kq = K / 8;              // 16-byte chunks per row
  const uint4* Wt = W + (long long)tile * BN * kq;
  constexpr int MAXP = (384 * 8 + NT - 1) / NT;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int s = 0; s < ksteps; s += U) {
    uint4 v[U][MAXP];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MAXP; ++i) {
        if (i >= per) break;
        const int c = threadIdx.x + i * NT;
        const int row = min(c >> 3, rows - 1), ch = c & 7;
        const long long col = kc0 + (long long)(s + u) * 8 + ch;
        const uint4* p;
        if (XONLY && row < 256)
          p = x + (long long)row * kq + col;
        else if (WT)  // W pre-tiled [N / BN][K / 64][BN][64]: a step's tile is contiguous
          p = W + (((long long)tile * (K / 64) + slice * ksteps + s + u) * BN +
                   (row - (XONLY ? 256 : 0))) * 8 + ch;
        else
          p = Wt + (long long)(row - (XONLY ? 256 : 0)) * kq + col;
        v[u][i] = *p;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MAXP; ++i) {
        if (i >= per) break;
        acc.x ^= v[u][i].x; acc.y ^= v[u][i].y; acc.z ^= v[u][i].z; acc.w ^= v[u][i].w;
      }
  }
  out[blockIdx.x * NT + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// wave-specialised: threads [0, NT/2) stream x, [NT/2, NT) stream W (separate vmcnt queues,
// so an L2-hit x load never waits behind an HBM W load of the same wave)
template <int NT, int UX, int UW>
__global__ void __launch_bounds__(NT) split_kernel(const uint4* __restrict__ x,
                                                   const uint4* __restrict__ W,
                                                   unsigned* __restrict__ out, int K, int BN,
                                                   int S) {
  const int tile = blockIdx.x / S, slice = blockIdx.x - tile * S;
  const int ksteps = K / 64 / S;
  const int kc0 = slice * ksteps * 8;
  const long long kq = K / 8;
  const bool isx = threadIdx.x < NT / 2;
  const int t = isx ? threadIdx.x : threadIdx.x - NT / 2;
  const int rows = isx ? 256 : BN;
  const int per = (rows * 8 + NT / 2 - 1) / (NT / 2);
  const uint4* base = isx ? x : W + (long long)tile * BN * kq;
  constexpr int MAXP = (256 * 8 + NT / 2 - 1) / (NT / 2);
  uint4 acc = make_uint4(0, 0, 0, 0);
  const int U = isx ? UX : UW;
  for (int s = 0; s < ksteps; s += U) {
    uint4 v[UX > UW ? UX : UW][MAXP];
#pragma unroll
    for (int u = 0; u < (UX > UW ? UX : UW); ++u) {
      if (u >= U) break;
#pragma unroll
      for (int i = 0; i < MAXP; ++i) {
        if (i >= per) break;
        const int c = t + i * (NT / 2);
        const int row = min(c >> 3, rows - 1), ch = c & 7;
        v[u][i] = base[(long long)row * kq + kc0 + (long long)(s + u) * 8 + ch];
      }
    }
#pragma unroll
    for (int u = 0; u < (UX > UW ? UX : UW); ++u) {
      if (u >= U) break;
#pragma unroll
      for (int i = 0; i < MAXP; ++i) {
        if (i >= per) break;
        acc.x ^= v[u][i].x; acc.y ^= v[u][i].y; acc.z ^= v[u][i].z; acc.w ^= v[u][i].w;
      }
    }
  }
  out[blockIdx.x * NT + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int NT, int UX, int UW>
int run_split(const uint4* x, std::vector<uint4*>& Ws, unsigned* out, int N, int K, int BN, int S) {
  const int blocks = (N / BN) * S;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 4; ++i)
    hipLaunchKernelGGL((split_kernel<NT, UX, UW>), dim3(blocks), dim3(NT), 0, 0, x,
                       Ws[i % Ws.size()], out, K, BN, S);
  CK(hipDeviceSynchronize());
  const int iters = 30;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((split_kernel<NT, UX, UW>), dim3(blocks), dim3(NT), 0, 0, x,
                       Ws[i % Ws.size()], out, K, BN, S);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / iters;
  const double per_block = (256.0 + BN) * (K / S) * 2.0;
  std::printf("{\"pattern\": \"x | W split waves\", \"N\": %d, \"K\": %d, \"BN\": %d, "
              "\"S\": %d, \"NT\": %d, \"UX\": %d, \"UW\": %d, \"blocks\": %d, \"us\": %.2f, "
              "\"GBps_per_block\": %.1f, \"TBps_total\": %.2f}\n",
              N, K, BN, S, NT, UX, UW, blocks, us, per_block / us / 1e3,
              per_block * blocks / us / 1e6);
  std::fflush(stdout);
  return 0;
}

template <int NT, int U, bool XO, bool WO, bool WT = false>
int run(const char* name, const uint4* x, std::vector<uint4*>& Ws, unsigned* out, int N, int K,
        int BN, int S) {
  const int blocks = (N / BN) * S;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 4; ++i)
    hipLaunchKernelGGL((stream_kernel<NT, U, XO, WO, WT>), dim3(blocks), dim3(NT), 0, 0, x,
                       Ws[i % Ws.size()], out, K, BN, S);
  CK(hipDeviceSynchronize());
  const int iters = 30;
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((stream_kernel<NT, U, XO, WO, WT>), dim3(blocks), dim3(NT), 0, 0, x,
                       Ws[i % Ws.size()], out, K, BN, S);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / iters;
  const double per_block = ((XO ? 256.0 : 0.0) + (WO ? BN : 0)) * (K / S) * 2.0;
  std::printf("{\"pattern\": \"%s\", \"N\": %d, \"K\": %d, \"BN\": %d, \"S\": %d, \"NT\": %d, "
              "\"U\": %d, \"blocks\": %d, \"us\": %.2f, \"GBps_per_block\": %.1f, "
              "\"TBps_total\": %.2f}\n",
              name, N, K, BN, S, NT, U, blocks, us, per_block / us / 1e3,
              per_block * blocks / us / 1e6);
  std::fflush(stdout);
  return 0;
}

int main() {
  const int K = 4096, N = 12288;
  uint4* x;
  unsigned* out;
  CK(hipMalloc(&x, 256LL * K * 2));
  CK(hipMemset(x, 1, 256LL * K * 2));
  CK(hipMalloc(&out, 4096 * 1024 * sizeof(unsigned)));
  std::vector<uint4*> Ws(6);
  for (auto& w : Ws) {
    CK(hipMalloc(&w, (long long)N * K * 2));
    CK(hipMemset(w, 3, (long long)N * K * 2));
  }
  // the shipped plan's shapes (qkv: BN 64 S 1; BN 128 S 2) and a square-ish split
  for (int cfg = 0; cfg < 4; ++cfg) {
    const int BN = cfg == 0 ? 64 : cfg == 1 ? 128 : cfg == 2 ? 128 : 48;
    const int S = cfg == 1 ? 2 : 1;
    run_split<512, 1, 2>(x, Ws, out, N, K, BN, S);
    run_split<512, 1, 4>(x, Ws, out, N, K, BN, S);
    run_split<1024, 1, 2>(x, Ws, out, N, K, BN, S);
    run_split<1024, 1, 4>(x, Ws, out, N, K, BN, S);
    run_split<1024, 2, 8>(x, Ws, out, N, K, BN, S);
  }
  for (int pat = 4; pat < 5; ++pat) {
    const char* nm = pat == 0 ? "x+W" : pat == 1 ? "x only" : pat == 2 ? "W only"
                   : pat == 3 ? "W tiled only" : "x+W tiled";
    for (int cfg = 0; cfg < 3; ++cfg) {
      const int BN = cfg == 0 ? 64 : 128, S = cfg == 0 ? 1 : cfg == 1 ? 2 : 1;
      if (pat == 0) {
        run<512, 1, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<512, 2, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<256, 2, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<1024, 1, true, true>(nm, x, Ws, out, N, K, BN, S);
      } else if (pat == 1) {
        run<512, 1, true, false>(nm, x, Ws, out, N, K, BN, S);
        run<512, 2, true, false>(nm, x, Ws, out, N, K, BN, S);
      } else if (pat == 2) {
        run<512, 1, false, true>(nm, x, Ws, out, N, K, BN, S);
        run<512, 2, false, true>(nm, x, Ws, out, N, K, BN, S);
      } else if (pat == 3) {
        run<512, 1, false, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<512, 2, false, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<512, 4, false, true, true>(nm, x, Ws, out, N, K, BN, S);
      } else {
        run<512, 1, true, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<512, 2, true, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<1024, 1, true, true, true>(nm, x, Ws, out, N, K, BN, S);
        run<1024, 2, true, true, true>(nm, x, Ws, out, N, K, BN, S);
      }
    }
  }
  return 0;
}
