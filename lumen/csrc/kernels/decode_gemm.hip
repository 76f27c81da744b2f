// Decode-batch projection GEMM on the matrix cores: y[M, N] = x[M, K] @ W[N, K]^T, 5 <= M <= 256.
//
// Reference behaviour: vLLM's decode projections (the serving stack the reference declares,
// SURVEY D11 / CS6) run these as library GEMMs.  At 128-256 running sequences hipBLASLt (tuned
// table) streams Llama-2-7B's projection weights at only ~2.4 TB/s (5.6 ms of an 18.7 ms decode
// step, profiles/r3_serve): its macro tiles leave most of the 256 CUs idle at these M.
//
// Why the previous hand-written attempt lost (scripts/probes/batch_gemm.hip): one workgroup per
// ~48 output columns and ALL of K, so every workgroup pulled all of x (M x K, 2 MB at M = 256)
// through its CU's L2->L1 path -- the per-CU load path, not HBM, was the bound.  Here the
// per-CU traffic is balanced instead:
//
//  * block tile = BM rows (the padded decode batch) x BN output columns x a K range (split-K S):
//    per CU (BM + BN) * Kc * 2 bytes in, 2 * BM * BN * Kc MFMA FLOPs; (BN, S) are chosen per
//    shape so the grid is ~one block per CU and the tile stays near the link / MFMA balance;
//  * BOTH operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, lane-linear 1-KiB
//    pieces = 8 image rows of 128 bytes, the 16-byte chunks XOR-swizzled through the per-lane
//    SOURCE address) into a 3-stage ring: two k64 stages in flight while one is multiplied, one
//    counted vmcnt wait + one barrier per stage;
//  * the product is formed transposed, y^T = W x^T (v_mfma_f32_16x16x32_{bf16,f16}: W rows are
//    the A operand, x rows the B operand), so a lane's four accumulators are four consecutive
//    output columns of one row: 8-byte stores;
//  * split-K (S > 1) is reduced IN the launch: every slice writes its f32 slab, takes a ticket
//    on the tile's counter (agent-scope release), and the last arriver (agent-scope acquire) sums
//    the other slabs into its registers and stores the tile.  Slices of a tile are mapped to
//    neighbouring virtual block ids under the XCD-aware remap, so they share an XCD.
#include "common.h"

namespace lumen {
namespace dg {

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

constexpr int BK = 64;      // k elements per stage = one 128-byte image row per matrix row
constexpr int ROWB = 128;
constexpr int NSTAGE = 3;

// 16-byte chunk c of image row r lives at chunk c ^ swz(r): a ds_read_b128 fragment read (16
// rows at one chunk, lane groups of 16) then touches 16 distinct 16-byte bank slots (rows of
// either parity share the 256-byte bank row's halves; the XOR spreads the 8 row pairs)
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0xF70);
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Opaque LDS-DMA, 16 bytes per lane (saddr form: wave-uniform 64-bit base + 32-bit lane offset).
// As inline asm the compiler's wait insertion does not see it (with the builtin it puts
// s_waitcnt vmcnt(0) before the next stage's ds_reads and serialises the ring); completion is
// ordered by the kernel's own counted vmcnt waits.  M0 = LDS address of lane 0's 16 bytes.
__device__ __forceinline__ void dma16(const void* base, unsigned off, const char* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(lds_wave_base))));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(off), "s"(base), "s"(m0) : "memory", "m0");
}

// One stage: image rows [0, BN) = W rows n0 .. n0+BN-1, rows [BN, BN+BM) = x rows 0 .. BM-1, k
// range [k0, k0 + 64).  Piece p (8 rows) is issued by wave p % NW; rows past N / M re-read the
// last valid row (finite data; those outputs are never stored).
template <typename T, int BM, int BN, int NW, bool XT = false>
__device__ __forceinline__ void stage(char* img, const T* Wt, int K, int nvalid, const T* x,
                                      long long ldx, int M, int k0, int wid, int lane) {
  constexpr int PIECES = (BN + BM) / 8;
  static_assert(PIECES % NW == 0, "(BN + BM) / 8 must be a multiple of the wave count");
  const int rr = lane >> 3;           // row within the piece
  const int c = lane & 7;             // LDS chunk (lane-linear)
#pragma unroll
  for (int q = 0; q < PIECES / NW; ++q) {
    const int p = NW * q + wid;
    const int r = 8 * p + rr;         // image row
    const int ch = c ^ swz(r);        // source chunk that belongs at LDS chunk c
    if (8 * p < BN) {                 // piece-uniform: BN % 8 == 0
      const int n = min(r, nvalid - 1);
      const unsigned off = (unsigned)(((long long)n * K + k0 + 8 * ch) * (long long)sizeof(T));
      dma16(Wt, off, img + 8 * p * ROWB);
    } else if constexpr (XT) {
      // k-tiled x ([K / 64][BM][64]): the stage's x rows are one contiguous BM x 128-byte run
      const int m = r - BN;
      const unsigned off = (unsigned)(((long long)(k0 >> 6) * BM * 64 + m * 64 + 8 * ch) *
                                      (long long)sizeof(T));
      dma16(x, off, img + 8 * p * ROWB);
    } else {
      const int m = min(r - BN, M - 1);
      const unsigned off = (unsigned)(((long long)m * ldx + k0 + 8 * ch) * (long long)sizeof(T));
      dma16(x, off, img + 8 * p * ROWB);
    }
  }
}

template <typename T, int NI, int MJ>
__device__ __forceinline__ void compute(const char* img, int nrow0, int mrow0,
                                        f32x4 (&acc)[NI][MJ], int lane) {
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 a[NI], b[MJ];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = nrow0 + 16 * i + lr;
      a[i] = *reinterpret_cast<const uint4*>(img + r * ROWB + (((4 * s + lg) ^ swz(r)) << 4));
    }
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int r = mrow0 + 16 * j + lr;
      b[j] = *reinterpret_cast<const uint4*>(img + r * ROWB + (((4 * s + lg) ^ swz(r)) << 4));
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j) acc[i][j] = Mfma<T>::run(a[i], b[j], acc[i][j]);
  }
}

// WM x WN waves (4 or 8); each wave: BN / WN output columns (NI blocks of 16) x BM / WM rows
// (MJ blocks).  8 waves: half the accumulators per wave, two waves per SIMD to hide the LDS /
// DMA latency.
// ROT (runtime, rot != 0): each block starts its k loop at a different stage (tile-dependent
// rotation), so the blocks running at once read different x / W k-ranges instead of all
// sweeping the same x lines together; XT: x in the k-tiled layout (see stage)
template <typename T, int BM, int BN, int WM, int WN, bool XT = false>
__global__ void __launch_bounds__(64 * WM * WN, 1)
dgemm_kernel(const T* __restrict__ x, const T* __restrict__ W, T* __restrict__ y,
             float* __restrict__ ws, int* __restrict__ cnt, int M, int N, int K, long long ldx,
             long long ldy, int tiles_n, int S, int kt_total, int rot, int skip) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int NI = BN / WN / 16, MJ = BM / WM / 16;
  static_assert(NI * WN * 16 == BN && MJ * WM * 16 == BM, "wave tiling");
  constexpr int STAGE_B = (BN + BM) * ROWB;
  constexpr int G = (BN + BM) / (8 * NW);  // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * STAGE_B + 16];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware bijective remap (blocks round-robin over 8 XCDs): consecutive virtual ids -- the
  // S slices of one tile, then the next tile -- land on one XCD
  const int nb = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile = v / S, slice = v - tile * S;
  const int tn = tile % tiles_n;
  const int n0 = tn * BN;
  const int nvalid = min(BN, N - n0);
  // k64 tiles of this slice: an even share, the first (kt_total % S) slices one more
  const int per = kt_total / S, extra = kt_total - per * S;
  const int kb = slice * per + min(slice, extra);
  const int nk = per + (slice < extra ? 1 : 0);
  const T* Wt = W + (long long)n0 * K;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int nrow0 = wn * (BN / WN), mrow0 = BN + wm * (BM / WM);

  f32x4 acc[NI][MJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r0 = rot ? (tile * rot) % nk : 0;
  const auto kat = [&](int t) {  // k offset of loop step t
    const int u = t + r0;
    return (kb + (u >= nk ? u - nk : u)) * BK;
  };
  stage<T, BM, BN, NW, XT>(lds, Wt, K, nvalid, x, ldx, M, kat(0), wid, lane);
  if (nk > 1)
    stage<T, BM, BN, NW, XT>(lds + STAGE_B, Wt, K, nvalid, x, ldx, M, kat(1), wid, lane);
  int buf = 0;
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) wait_vm<G>(); else wait_vm<0>();
    lds_barrier();  // stage t landed for every wave; every wave is done with stage t - 1
    if (t + 2 < nk) {
      const int nbuf = buf >= 1 ? buf - 1 : 2;  // (t + 2) % 3 == (t - 1) % 3
      stage<T, BM, BN, NW, XT>(lds + nbuf * STAGE_B, Wt, K, nvalid, x, ldx, M, kat(t + 2), wid,
                               lane);
    }
    if (!skip) compute<T, NI, MJ>(lds + buf * STAGE_B, nrow0, mrow0, acc, lane);
    buf = buf == 2 ? 0 : buf + 1;
  }

  if (S > 1) {
    // slab of this slice: register-major, one 1-KiB wave-instruction per accumulator tile
    float* slab = ws + ((long long)tile * S + slice) * (NT * NI * MJ * 4);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        *reinterpret_cast<f32x4*>(slab + ((i * MJ + j) * NT + threadIdx.x) * 4) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds + NSTAGE * STAGE_B);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
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

  // lane holds y^T[n = n0 + nrow0 + 16 i + 4 (lane >> 4) + 0..3][m = mrow0 - BN + 16 j + (lane & 15)]
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int m = mrow0 - BN + 16 * j + lr;
    if (m >= M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int n = nrow0 + 16 * i + 4 * lg;
      if (n >= nvalid) continue;
      const uint2 val = make_uint2(pk2<T>(acc[i][j][0], acc[i][j][1]),
                                   pk2<T>(acc[i][j][2], acc[i][j][3]));
      *reinterpret_cast<uint2*>(y + (long long)m * ldy + n0 + n) = val;
    }
  }
}

// compiled (BM, BN, waves) variants.  4 waves, WM x WN: BM 256 -> 4 x 1, 128 -> 2 x 2,
// 64 -> 1 x 4; 8 waves: BM 256 -> 4 x 2, 128 -> 2 x 4
#define LUMEN_DG_VARIANTS(X)                                                                   \
  X(256, 64, 4, 1) X(256, 96, 4, 1) X(256, 128, 4, 1) X(256, 160, 4, 1)                         \
  X(192, 64, 4, 1) X(192, 96, 4, 1) X(192, 128, 4, 1)                                           \
  X(128, 64, 2, 2) X(128, 96, 2, 2) X(128, 128, 2, 2) X(128, 192, 2, 2) X(128, 256, 2, 2)       \
  X(64, 64, 1, 4) X(64, 128, 1, 4) X(64, 192, 1, 4) X(64, 256, 1, 4)                            \
  X(256, 64, 4, 2) X(256, 128, 4, 2) X(128, 128, 2, 4) X(128, 256, 2, 4)

// k-tiled x variants (flags bit 1): the BM = 256 tiles
#define LUMEN_DG_XT_VARIANTS(X) X(256, 64, 4, 1) X(256, 128, 4, 1) X(256, 64, 4, 2) X(256, 128, 4, 2)

template <typename T>
hipError_t launch(const void* x, const void* W, void* y, float* ws, int* cnt, int M, int N, int K,
                  long long ldx, long long ldy, int BM, int BN, int NW, int S, int flags,
                  hipStream_t st) {
  const int tiles_n = (N + BN - 1) / BN;
  const int kt = K / BK;
  const int rot = (flags & 1) ? 1 : 0;
  const int skip = (flags >> 2) & 1;  // cost probe: the k loop without its MFMA work
  dim3 grid(tiles_n * S), block(64 * NW);
#define LUMEN_DG_CASE(bm, bn, wm, wn)                                                          \
  if (BM == bm && BN == bn && NW == wm * wn && !(flags & 2)) {                                 \
    hipLaunchKernelGGL((dgemm_kernel<T, bm, bn, wm, wn>), grid, block, 0, st, (const T*)x,     \
                       (const T*)W, (T*)y, ws, cnt, M, N, K, ldx, ldy, tiles_n, S, kt, rot, skip);  \
    return hipGetLastError();                                                                  \
  }
  LUMEN_DG_VARIANTS(LUMEN_DG_CASE)
#undef LUMEN_DG_CASE
#define LUMEN_DG_XT_CASE(bm, bn, wm, wn)                                                       \
  if (BM == bm && BN == bn && NW == wm * wn && (flags & 2)) {                                  \
    hipLaunchKernelGGL((dgemm_kernel<T, bm, bn, wm, wn, true>), grid, block, 0, st,            \
                       (const T*)x, (const T*)W, (T*)y, ws, cnt, M, N, K, ldx, ldy, tiles_n, S, \
                       kt, rot, skip);                                                         \
    return hipGetLastError();                                                                  \
  }
  LUMEN_DG_XT_VARIANTS(LUMEN_DG_XT_CASE)
#undef LUMEN_DG_XT_CASE
  return hipErrorInvalidValue;
}

}  // namespace dg
}  // namespace lumen

// y[M, N] = x[M, K] @ W[N, K]^T.  M <= BM; K % 64 == 0; N % 4 == 0; W contiguous [N, K]; x rows
// at stride ldx (% 8), y rows at stride ldy (% 4), 16-byte aligned bases.  S > 1: ``ws`` holds
// ceil(N / BN) * S * 256 * (BM * BN / 256) floats and ``cnt`` ceil(N / BN) zeroed ints (the last
// slice of each tile re-zeroes its counter, so they stay zero between launches).
// flags: bit 0 = per-tile k rotation; bit 1 = x in the k-tiled layout [K / 64][BM][64]
// (ldx ignored; BM = 256 variants only); bit 2 = cost probe, the k loop without its ds_reads and
// MFMAs (the output is garbage)
extern "C" hipError_t lumen_decode_gemm(int dtype, const void* x, const void* W, void* y,
                                        float* ws, int* cnt, int M, int N, int K, long long ldx,
                                        long long ldy, int BM, int BN, int NW, int S, int flags,
                                        hipStream_t st) {
  if (M < 1 || M > BM || N < 4 || N % 4 != 0 || K < 64 || K % 64 != 0 || ldx % 8 != 0 ||
      ldy % 4 != 0 || ldx < K || ldy < N || S < 1 || S > K / 64 ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W) |
        reinterpret_cast<uintptr_t>(y)) & 15) != 0)
    return hipErrorInvalidValue;
  if (S > 1 && (ws == nullptr || cnt == nullptr)) return hipErrorInvalidValue;
  // every 32-bit lane offset of the DMAs stays below 2^32 bytes
  if ((long long)BN * K * 2 >= (1LL << 32) || (long long)BM * ldx * 2 >= (1LL << 32))
    return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::dg::launch<lumen::bf16>(x, W, y, ws, cnt, M, N, K, ldx, ldy, BM, BN, NW, S,
                                          flags, st);
  if (dtype == lumen::kF16)
    return lumen::dg::launch<lumen::fp16>(x, W, y, ws, cnt, M, N, K, ldx, ldy, BM, BN, NW, S,
                                          flags, st);
  return hipErrorInvalidValue;
}
