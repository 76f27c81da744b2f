// PROBE, NOT BUILT (moved out of lumen/csrc/kernels after measuring it against hipBLASLt):
// 3.7-4.7 TB/s at M <= 64 (hipBLASLt with the tuned table ties or wins), 1.5 TB/s at M = 256 where
// every workgroup re-reads all of x from L2 (q|k|v 68 vs 38 us); serving 6.6k vs 7.6k tok/s
// with it (profiles/r3_serve/batch_gemm_sweep.jsonl).  Kept for the record of what was tried.
// Decode-batch GEMM on the matrix cores: y[M, N] = x[M, K] @ W[N, K]^T for 5 <= M <= 256.
//
// Reference behaviour: vLLM's decode projections (the serving stack the reference declares,
// SURVEY D11 / CS6) run these as library GEMMs.  At 128-256 running sequences hipBLASLt (tuned
// table) runs Llama-2-7B's projections at 2.4-4 TB/s of weight traffic and 0.5-0.7 PF/s:
// q|k|v 42 us, o 23 us, gate|up 61 us, down 49 us at M = 224 (configs/tunableop), ~5.6 ms of
// an 18.7 ms decode step (profiles/r3_serve).  Its macro tiles leave most CUs idle at these M
// (256 x 64 tiles: 192 workgroups for q|k|v).
//
// Design (gfx950, wave64, v_mfma_f32_16x16x32_{bf16,f16}):
//  * one workgroup = 4 waves = ALL M rows (64 * MB, MB = ceil(M / 64)) x 16 * NB output columns,
//    NB picked so the grid is ~one workgroup per CU (q|k|v: 48 columns, 256 workgroups; gate|up
//    96, 230; lm_head 128, 250; o / down 16, 256): every weight byte is read from HBM once, by
//    one CU, and the whole chip streams;
//  * the product is formed transposed, y^T = W x^T: W is the MFMA A operand, so a lane's four
//    accumulators are four consecutive n of one row m -- 8-byte stores;
//  * W streams in 128-column (k) chunks through two separately declared LDS images (256-byte
//    rows, XOR-swizzled 16-byte chunks, the flash-attention image format) filled by LDS-DMA
//    (global_load_lds from a wave-uniform base + 32-bit lane offsets: no VGPRs); all 4 waves read
//    every W fragment from LDS;
//  * x (L2-resident: <= 256 x K) goes straight to registers in the MFMA B layout, each wave its
//    own 16 * MB rows, one chunk ahead of the MFMAs;
//  * the DMA / x loads of chunk c + 1 are in flight while chunk c is multiplied (one counted
//    vmcnt wait + a barrier per chunk; the loop is unrolled by two so every LDS access names its
//    image statically and the compiler adds no vmcnt(0) of its own).
#include "common.h"

namespace lumen {
namespace bg {

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

constexpr int BK = 128;  // k elements per chunk (one 256-byte image row per weight row)

// image row r, 16-byte chunk c -> byte offset (chunks XOR-swizzled per row: the 16 rows of one
// wave's 16-byte fragment read spread over the banks)
__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * 256 + ((chunk ^ swz(row)) << 4);
}

// s_waitcnt vmcnt(N) as the builtin (the compiler's wait insertion understands it): gfx9 simm16
// keeps vmcnt bits [3:0] and [15:14], expcnt [6:4] and lgkmcnt [11:8] at "don't care"
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

// Opaque LDS-DMA of 16 bytes per lane: global_load_lds_dwordx4 in its saddr form (wave-uniform
// 64-bit base in SGPRs + a 32-bit lane offset).  As inline asm the compiler's wait insertion does
// not see it: with the builtin it could not tell the DMA into one image from the ds_reads of the
// other and put s_waitcnt vmcnt(0) in front of every chunk's first LDS read (serialising the
// prefetch).  Completion is ordered by the kernel's own counted vmcnt waits; operations the
// compiler cannot see only make its own counted waits stricter (the counter retires in order).
// M0 = LDS destination of lane 0 (lane-linear, +16 bytes per lane).
__device__ __forceinline__ void dma16(const void* base, unsigned off, const char* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(lds_wave_base))));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(off), "s"(base), "s"(m0) : "memory", "m0");
}

// DMA rows [0, 16 NB) x k [0, 128) of the weight tile at `wt` (row stride ld elements) into img:
// wave w issues rows 16 j + 4 w + 0..3 (one KiB per instruction, lane-linear in LDS; the swizzle
// moves to the per-lane SOURCE chunk).  Rows >= nvalid re-read the last valid row (finite data,
// their outputs are never stored).
template <typename T, int NB>
__device__ __forceinline__ void stage_w(char* img, const T* wt, int ld, int nvalid, int wid,
                                        int lane) {
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int r = 16 * j + 4 * wid + (lane >> 4);
    const int rs = r < nvalid ? r : nvalid - 1;
    const int ch = (lane & 15) ^ swz(r);
    const unsigned off = (unsigned)(rs * ld + ch * 8) * (unsigned)sizeof(T);
    dma16(wt, off, img + (16 * j + 4 * wid) * 256);
  }
}

// this wave's x fragments for one chunk: block i = rows mbase + 16 i + (lane & 15), k32 step s =
// k0 + 32 s + 8 (lane >> 4) .. + 7 (the MFMA B layout).  Rows >= M re-read row M - 1: output
// column m of y^T depends on x row m only, and those columns are never stored -- so every lane
// issues every load (no exec-masked branches: the counted vmcnt waits stay exact).
template <typename T, int MB>
__device__ __forceinline__ void load_x(uint4 (&xf)[MB][4], const T* x, long long ldx, int M,
                                       int mbase, int k0, int lane) {
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int m = min(mbase + 16 * i + (lane & 15), M - 1);
    const T* p = x + (long long)m * ldx + k0 + 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) xf[i][s] = *reinterpret_cast<const uint4*>(p + 32 * s);
  }
}

template <typename T, int MB, int NB>
__device__ __forceinline__ void mma_chunk(const char* img, const uint4 (&xf)[MB][4],
                                          f32x4 (&acc)[MB][NB], int lane) {
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint4 wf[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
      wf[j] = *reinterpret_cast<const uint4*>(img + img_off(16 * j + lr, 4 * s + lg));
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = Mfma<T>::run(wf[j], xf[i][s], acc[i][j]);
  }
}

template <typename T, int MB, int NB>
__global__ void __launch_bounds__(256, 1) bgemm_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ W,
                                                       T* __restrict__ y, int M, int N, int K,
                                                       long long ldx, long long ldy) {
  __shared__ __attribute__((aligned(16))) char bufA[16 * NB * 256];
  __shared__ __attribute__((aligned(16))) char bufB[16 * NB * 256];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * 16 * NB;
  const int nvalid = min(16 * NB, N - n0);
  const int mbase = 16 * MB * wid;
  const T* wt = W + (long long)n0 * K;
  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 xa[MB][4], xb[MB][4];
  const int nc = K / BK;
  constexpr int INFL = NB + 4 * MB;  // vm operations one chunk issues per wave
  // K % 256 == 0: an even chunk count, so the steady-state loop body is straight-line (no
  // conditional prefetch -- branches there made the compiler shuttle the accumulators between
  // AGPRs and VGPRs every iteration and wait vmcnt(0) before the MFMAs)
  stage_w<T, NB>(bufA, wt, K, nvalid, wid, lane);
  load_x<T, MB>(xa, x, ldx, M, mbase, 0, lane);
  for (int c = 0; c < nc - 2; c += 2) {
    stage_w<T, NB>(bufB, wt + (c + 1) * BK, K, nvalid, wid, lane);
    load_x<T, MB>(xb, x, ldx, M, mbase, (c + 1) * BK, lane);
    wait_vm<INFL>();
    lds_barrier();  // every wave's share of chunk c has landed
    mma_chunk<T, MB, NB>(bufA, xa, acc, lane);
    lds_barrier();  // every wave is done with bufA before it is refilled
    stage_w<T, NB>(bufA, wt + (c + 2) * BK, K, nvalid, wid, lane);
    load_x<T, MB>(xa, x, ldx, M, mbase, (c + 2) * BK, lane);
    wait_vm<INFL>();
    lds_barrier();
    mma_chunk<T, MB, NB>(bufB, xb, acc, lane);
    lds_barrier();
  }
  stage_w<T, NB>(bufB, wt + (nc - 1) * BK, K, nvalid, wid, lane);
  load_x<T, MB>(xb, x, ldx, M, mbase, (nc - 1) * BK, lane);
  wait_vm<INFL>();
  lds_barrier();
  mma_chunk<T, MB, NB>(bufA, xa, acc, lane);
  wait_vm<0>();
  lds_barrier();
  mma_chunk<T, MB, NB>(bufB, xb, acc, lane);
  // lane holds y^T[n = 16 j + 4 (lane >> 4) + 0..3][m = mbase + 16 i + (lane & 15)]
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int m = mbase + 16 * i + lr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = 16 * j + 4 * lg;
      if (n >= nvalid) continue;
      const uint2 v = make_uint2(pk2<T>(acc[i][j][0], acc[i][j][1]),
                                 pk2<T>(acc[i][j][2], acc[i][j][3]));
      *reinterpret_cast<uint2*>(y + (long long)m * ldy + n0 + n) = v;
    }
  }
}

template <typename T, int MB>
hipError_t launch_mb(int nb, dim3 grid, const void* x, const void* W, void* y, int M, int N,
                     int K, long long ldx, long long ldy, hipStream_t st) {
  dim3 block(256);
#define LUMEN_BG(NBV)                                                                          \
  hipLaunchKernelGGL((bgemm_kernel<T, MB, NBV>), grid, block, 0, st, (const T*)x, (const T*)W, \
                     (T*)y, M, N, K, ldx, ldy)
  switch (nb) {
    case 1: LUMEN_BG(1); break;
    case 2: LUMEN_BG(2); break;
    case 3: LUMEN_BG(3); break;
    case 4: LUMEN_BG(4); break;
    case 6: LUMEN_BG(6); break;
    case 8: LUMEN_BG(8); break;
    default: return hipErrorInvalidValue;
  }
#undef LUMEN_BG
  return hipGetLastError();
}

template <typename T>
hipError_t launch(const void* x, const void* W, void* y, int M, int N, int K, long long ldx,
                  long long ldy, int cus, hipStream_t st) {
  // output-column blocks per workgroup: the smallest NB whose grid fits one wave on the chip
  const int blocks = N / 16;
  static const int kNB[] = {1, 2, 3, 4, 6, 8};
  int nb = 8;
  for (int v : kNB)
    if ((blocks + v - 1) / v <= cus) { nb = v; break; }
  dim3 grid((blocks + nb - 1) / nb);
  const int mb = (M + 63) / 64;
  switch (mb) {
    case 1: return launch_mb<T, 1>(nb, grid, x, W, y, M, N, K, ldx, ldy, st);
    case 2: return launch_mb<T, 2>(nb, grid, x, W, y, M, N, K, ldx, ldy, st);
    case 3: return launch_mb<T, 3>(nb, grid, x, W, y, M, N, K, ldx, ldy, st);
    case 4: return launch_mb<T, 4>(nb, grid, x, W, y, M, N, K, ldx, ldy, st);
    default: return hipErrorInvalidValue;
  }
}

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace bg
}  // namespace lumen

// y[M, N] = x[M, K] @ W[N, K]^T: 1 <= M <= 256, N % 16 == 0, K % 256 == 0, W contiguous
// [N, K]; x rows at stride ldx (% 8), y rows at stride ldy (% 4); 16-byte aligned bases.
extern "C" hipError_t lumen_batch_gemm(int dtype, const void* x, const void* W, void* y, int M,
                                       int N, int K, long long ldx, long long ldy,
                                       hipStream_t st) {
  if (M < 1 || M > 256 || N < 16 || N % 16 != 0 || K < 256 || K % 256 != 0 || ldx % 8 != 0 ||
      ldy % 4 != 0 || ldx < K || ldy < N ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W) |
        reinterpret_cast<uintptr_t>(y)) & 15) != 0)
    return hipErrorInvalidValue;
  // every 32-bit lane offset of the weight DMA stays below 2^32 bytes
  if ((long long)128 * K * 2 >= (1LL << 32)) return hipErrorInvalidValue;
  const int cus = lumen::bg::cu_count();
  if (dtype == lumen::kBF16)
    return lumen::bg::launch<lumen::bf16>(x, W, y, M, N, K, ldx, ldy, cus, st);
  if (dtype == lumen::kF16)
    return lumen::bg::launch<lumen::fp16>(x, W, y, M, N, K, ldx, ldy, cus, st);
  return hipErrorInvalidValue;
}
