// RETIRED (round 4, measured slower than hipBLASLt and than decode_gemm.hip's split-K kernel at
// every serving shape: profiles/r4_dgemm/README.md).  Kept for the record; not built.  It lived in
// namespace lumen::dg of lumen/csrc/kernels/decode_gemm.hip and used that file's helpers (BK, swz,
// Mfma, f32x4, pk2).

// ---------------------------------------------------------------------------------------------
// Weight-streaming variant (wsg): W goes global -> registers (each W element is read by exactly
// one wave, so it never needs LDS), x is staged once per block per k64 stage in a swizzled LDS
// image that all 4 waves read.  Every wave owns 32 output columns (NI = 2 MFMA row tiles of W)
// for ALL BM = 16 MJ decode rows, so the block's x traffic per W byte is BM / 128 and the LDS
// carries only x.  W for the next two stages is in flight in two register sets while a stage is
// multiplied; x for the next stage is loaded into registers and written to the other LDS buffer
// after the stage's MFMAs (one barrier per stage).  All loads are compiler-visible (no LDS-DMA),
// so the compiler's counted waits keep the W stream overlapped.  Split-K as dgemm_kernel.
// ---------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void wsg_wload(uint4 (&wr)[2][2], const T* w0, const T* w1,
                                          long long k0) {
  wr[0][0] = *reinterpret_cast<const uint4*>(w0 + k0);
  wr[0][1] = *reinterpret_cast<const uint4*>(w0 + k0 + 32);
  wr[1][0] = *reinterpret_cast<const uint4*>(w1 + k0);
  wr[1][1] = *reinterpret_cast<const uint4*>(w1 + k0 + 32);
}

// x chunk q of this thread: row (threadIdx.x >> 3) + 32 q, 16-byte chunk threadIdx.x & 7
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T, int XQ>
__device__ __forceinline__ void wsg_xload(u32x4 (&xr)[XQ], const T* xbase, long long ldx, int M,
                                          long long k0) {
  const int row0 = threadIdx.x >> 3;
#pragma unroll
  for (int q = 0; q < XQ; ++q) {
    // rows past M re-read row M - 1 (finite; those outputs are never stored)
    const long long off = (long long)(min(row0 + 32 * q, M - 1) - min(row0, M - 1)) * ldx;
    xr[q] = *reinterpret_cast<const u32x4*>(xbase + off + k0);
  }
}

template <int XQ>
__device__ __forceinline__ void wsg_xstore(const u32x4 (&xr)[XQ], uint4* img) {
  const int row0 = threadIdx.x >> 3, ch = threadIdx.x & 7;
#pragma unroll
  for (int q = 0; q < XQ; ++q) {
    const int row = row0 + 32 * q;
    *reinterpret_cast<u32x4*>(img + row * 8 + (ch ^ swz(row))) = xr[q];
  }
}

template <typename T, int MJ>
__device__ __forceinline__ void wsg_compute(f32x4 (&acc)[2][MJ], const uint4 (&wr)[2][2],
                                            const uint4* img, int lr, int lg) {
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int r = 16 * j + lr;
      const uint4 b = img[r * 8 + ((4 * s2 + lg) ^ swz(r))];
      acc[0][j] = Mfma<T>::run(wr[0][s2], b, acc[0][j]);
      acc[1][j] = Mfma<T>::run(wr[1][s2], b, acc[1][j]);
    }
}

template <typename T, int MJ>
__global__ void __launch_bounds__(256, MJ >= 16 ? 1 : 2)
wsg_kernel(const T* __restrict__ x, const T* __restrict__ W, T* __restrict__ y,
           float* __restrict__ ws, int* __restrict__ cnt, int M, int N, int K, long long ldx,
           long long ldy, int tiles_n, int S, int kt_total) {
  constexpr int NI = 2, BN = 128, BM = 16 * MJ, NT = 256;
  constexpr int XQ = BM * 8 / NT;            // x uint4 chunks per thread per stage
  static_assert(XQ >= 1 && BM * 8 % NT == 0, "BM must be a multiple of 32");
  __shared__ __attribute__((aligned(16))) uint4 xs[2][BM * 8];
  __shared__ int flag;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int nb = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = v / S, slice = v - tile * S;
  const int n0 = (tile % tiles_n) * BN;
  const int per = kt_total / S, extra = kt_total - per * S;
  const int kb = slice * per + min(slice, extra);
  const int nk = per + (slice < extra ? 1 : 0);

  // this lane's W rows (clamped: rows past N re-read row N-1, never stored)
  const T* wrow0 = W + (long long)min(n0 + wid * 32 + lr, N - 1) * K + 8 * lg;
  const T* wrow1 = W + (long long)min(n0 + wid * 32 + 16 + lr, N - 1) * K + 8 * lg;
  const T* xbase = x + (long long)min((int)(threadIdx.x >> 3), M - 1) * ldx + 8 * (threadIdx.x & 7);
  f32x4 acc[NI][MJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // W ring: four register sets, stage t + 4 is requested as soon as stage t's set is consumed
  uint4 w0[2][2], w1[2][2], w2[2][2], w3[2][2];
  u32x4 xr[XQ];
  const long long kbase = (long long)kb * BK;
  if (nk > 0) wsg_wload<T>(w0, wrow0, wrow1, kbase);
  if (nk > 1) wsg_wload<T>(w1, wrow0, wrow1, kbase + BK);
  if (nk > 2) wsg_wload<T>(w2, wrow0, wrow1, kbase + 2 * BK);
  if (nk > 3) wsg_wload<T>(w3, wrow0, wrow1, kbase + 3 * BK);
  if (nk > 0) {
    wsg_xload<T, XQ>(xr, xbase, ldx, M, kbase);
    wsg_xstore<XQ>(xr, xs[0]);
  }
  __syncthreads();
#define LUMEN_WSG_STAGE(WR, U)                                                                 \
  {                                                                                            \
    const int tt = t + (U);                                                                    \
    if (tt >= nk) break;                                                                       \
    const long long k0 = kbase + (long long)tt * BK;                                           \
    if (tt + 1 < nk) wsg_xload<T, XQ>(xr, xbase, ldx, M, k0 + BK);                             \
    wsg_compute<T, MJ>(acc, WR, xs[(U) & 1], lr, lg);                                          \
    if (tt + 4 < nk) wsg_wload<T>(WR, wrow0, wrow1, k0 + 4 * BK);                              \
    if (tt + 1 < nk) wsg_xstore<XQ>(xr, xs[((U) + 1) & 1]);                                    \
    __syncthreads();                                                                           \
  }
  for (int t = 0; t < nk; t += 4) {
    LUMEN_WSG_STAGE(w0, 0)
    LUMEN_WSG_STAGE(w1, 1)
    LUMEN_WSG_STAGE(w2, 2)
    LUMEN_WSG_STAGE(w3, 3)
  }
#undef LUMEN_WSG_STAGE

  if (S > 1) {
    float* slab = ws + ((long long)tile * S + slice) * (NT * NI * MJ * 4);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        *reinterpret_cast<f32x4*>(slab + ((i * MJ + j) * NT + threadIdx.x) * 4) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = last;
    }
    __syncthreads();
    if (!flag) return;
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int o = 0; o < S; ++o) {
      if (o == slice) continue;
      const float* os = ws + ((long long)tile * S + o) * (NT * NI * MJ * 4);
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(os + ((i * MJ + j) * NT + threadIdx.x) * 4);
    }
  }
  // lane holds y^T[n = n0 + 32 wid + 16 i + 4 lg + 0..3][m = 16 j + lr]
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int m = 16 * j + lr;
    if (m >= M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int n = n0 + wid * 32 + 16 * i + 4 * lg;
      if (n >= N) continue;
      const uint2 val = make_uint2(pk2<T>(acc[i][j][0], acc[i][j][1]),
                                   pk2<T>(acc[i][j][2], acc[i][j][3]));
      *reinterpret_cast<uint2*>(y + (long long)m * ldy + n) = val;
    }
  }
}

template <typename T>
hipError_t launch_wsg(const void* x, const void* W, void* y, float* ws, int* cnt, int M, int N,
                      int K, long long ldx, long long ldy, int mj, int S, hipStream_t st) {
  const int tiles_n = (N + 127) / 128;
  dim3 grid(tiles_n * S), block(256);
  const int kt = K / BK;
#define LUMEN_WSG_CASE(MJV)                                                                    \
  if (mj == MJV) {                                                                             \
    hipLaunchKernelGGL((wsg_kernel<T, MJV>), grid, block, 0, st, (const T*)x, (const T*)W,    \
                       (T*)y, ws, cnt, M, N, K, ldx, ldy, tiles_n, S, kt);                     \
    return hipGetLastError();                                                                  \
  }
  LUMEN_WSG_CASE(4) LUMEN_WSG_CASE(8) LUMEN_WSG_CASE(12) LUMEN_WSG_CASE(16)
#undef LUMEN_WSG_CASE
  return hipErrorInvalidValue;
}


// weight-streaming variant: y[M, N] = x[M, K] @ W[N, K]^T, M <= 16 * mj (mj in 4, 8, 12, 16),
// 128-column tiles, split-K S (ws: ceil(N / 128) * S * 16 mj * 128 floats; cnt: ceil(N / 128)
// zeroed ints).  N % 4 == 0, K % 64 == 0, 16-byte aligned bases and row strides % 8.
extern "C" hipError_t lumen_wsgemm(int dtype, const void* x, const void* W, void* y, float* ws,
                                   int* cnt, int M, int N, int K, long long ldx, long long ldy,
                                   int mj, int S, hipStream_t st) {
  if (M < 1 || M > 16 * mj || N < 4 || N % 4 != 0 || K < 64 || K % 64 != 0 || ldx % 8 != 0 ||
      ldy % 4 != 0 || ldx < K || ldy < N || S < 1 || S > K / 64 ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W) |
        reinterpret_cast<uintptr_t>(y)) & 15) != 0)
    return hipErrorInvalidValue;
  if (S > 1 && (ws == nullptr || cnt == nullptr)) return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::dg::launch_wsg<lumen::bf16>(x, W, y, ws, cnt, M, N, K, ldx, ldy, mj, S, st);
  if (dtype == lumen::kF16)
    return lumen::dg::launch_wsg<lumen::fp16>(x, W, y, ws, cnt, M, N, K, ldx, ldy, mj, S, st);
  return hipErrorInvalidValue;
}
