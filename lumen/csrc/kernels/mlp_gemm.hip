// Training-shape MLP GEMMs on the matrix cores with the SwiGLU fused into the epilogue
// (VERDICT r5 "Next" #1).
//
// Reference behaviour: the reference's MLP is transformers' LlamaMLP inside the model loaded at
// training/train_baseline.py:122-126 -- `down(act(gate(x)) * up(x))`: library GEMMs with the
// activation as separate elementwise passes.  Here:
//
//  * forward (EPI 1): gu = y @ [Wg | Wu]^T and act = silu(g) * u in ONE launch.  Each 256 x 256
//    block tile holds 128 activation columns: its W image interleaves 32 gate rows and the 32 up
//    rows of the same activation columns per wave, so a lane's accumulators for gate column c and
//    up column c are the same (row, column) positions of two fragments and the SwiGLU is formed
//    in registers.  gu (the backward needs g and u) and act leave the block; the separate
//    SwiGLU pass (a read of the whole [T, 2F] gu) is gone.
//  * backward (EPI 2): dact = dout @ Wd (against the cached Wd^T, both operands K-contiguous)
//    with the SwiGLU backward in the epilogue: it reads g / u at the tile's positions and writes
//    dg | du, so dact never goes to HBM.
//  * EPI 0 is the plain C = x @ W^T store (standalone A/B against hipBLASLt).
//
// Kernel: 256 x 256 x 64 block tile, 8 waves (2 along M x 4 along N; 128 x 64 outputs per wave,
// v_mfma_f32_16x16x32_bf16), both operands global -> LDS by LDS-DMA (global_load_lds_dwordx4,
// 1-KiB lane-linear pieces of 8 rows x 128 bytes, 16-byte chunks XOR-swizzled through the
// per-lane SOURCE address: conflict-free ds_read_b128 fragment reads), two 64-KiB stages: stage
// k + 1 streams in while stage k is multiplied, one counted wait + one barrier per k-step.  The
// product is formed transposed (W rows are the MFMA A operand), so a lane's four accumulators
// are four consecutive output columns of one row: 8-byte stores.  Block ids are remapped
// XCD-aware (the blocks of one XCD get consecutive tiles) and tiles are visited in groups of
// GROUP_M row tiles, so the blocks that run together on an XCD share x and W panels in its L2.
#include "common.h"

namespace lumen {
namespace mg {

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

constexpr int BM = 256, BN = 256, BK = 64, ROWB = 128;
constexpr int NW = 8, NT = 64 * NW, WM = 2, WN = 4;
constexpr int NI = BN / WN / 16;  // n fragments per wave (4)
constexpr int MJ = BM / WM / 16;  // m fragments per wave (8)
constexpr int IMG = 256 * ROWB;   // one operand image per stage: 32 KiB
constexpr int STAGE_B = 2 * IMG;  // [W image | x image]
constexpr int NSTAGE = 2;

enum Epi : int { kStore = 0, kSwiGLU = 1, kSwiGLUBwd = 2 };

struct Args {
  const void* x;   // [M, K] rows at ldx
  const void* w;   // [Nw, K] rows at ldw (EPI 1: [2F, K] = gate rows then up rows)
  void* c;         // EPI 0: C [M, N]; EPI 1: gu [M, 2F]; EPI 2: dgu [M, 2F]  (rows at ldc)
  void* act;       // EPI 1: act [M, F] (rows at ldact)
  const void* gu;  // EPI 2: saved gu [M, 2F] (rows at ldgu)
  long long ldx, ldw, ldc, ldact, ldgu;
  int M, N, K, F;  // N: GEMM output columns (EPI 1: 2F)
  int tiles_m, tiles_n, group_m;
};

// 16-byte chunk c of image row r lives at chunk c ^ swz(r) (see decode_gemm.hip: a ds_read_b128
// fragment read -- 16 rows at one chunk -- touches 16 distinct bank slots)
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

// LDS-DMA of 16 bytes per lane from a wave-uniform base + 32-bit lane offset into the wave's
// lane-linear 1-KiB LDS piece (M0 = its LDS address).  Inline asm: hipcc's own wait insertion
// does not see it, so the kernel's counted vmcnt waits order it.
__device__ __forceinline__ void dma16(const void* base, unsigned off, const char* lds_piece) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(lds_piece))));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(off), "s"(base), "s"(m0) : "memory", "m0");
}

// One k-step's images: pieces 0..31 = W image rows 0..255, pieces 32..63 = x image rows 0..255;
// wave wid issues pieces wid, wid + 8, ..., so q < 4 is the W image for every wave (uniform).
template <typename T, int EPI>
__device__ __forceinline__ void stage(char* img, const Args& a, const T* xb, int mvalid, int tn,
                                      int k0, int wid, int lane) {
  const int rr = lane >> 3, c = lane & 7;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = wid + 8 * q;
    if (q < 4) {
      const int r = 8 * p + rr;
      const int ch = c ^ swz(r);
      int wrow;
      if constexpr (EPI == kSwiGLU) {
        // wave slot wn = r / 64: rows 0..31 gate, 32..63 up, of activation columns
        // 128 tn + 32 wn + (r % 32)
        const int w = r & 63;
        wrow = (w < 32 ? 0 : a.F) + tn * 128 + (r >> 6) * 32 + (w & 31);
      } else {
        wrow = tn * BN + r;
      }
      const unsigned off =
          (unsigned)(((long long)wrow * a.ldw + k0 + 8 * ch) * (long long)sizeof(T));
      dma16(a.w, off, img + p * 8 * ROWB);
    } else {
      const int r = 8 * (p - 32) + rr;
      const int ch = c ^ swz(r);
      const int m = min(r, mvalid - 1);  // rows past M re-read the last row (never stored)
      const unsigned off = (unsigned)(((long long)m * a.ldx + k0 + 8 * ch) * (long long)sizeof(T));
      dma16(xb, off, img + p * 8 * ROWB);
    }
  }
}

template <typename T>
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
      b[j] = *reinterpret_cast<const uint4*>(img + IMG + r * ROWB +
                                              (((4 * s + lg) ^ swz(r)) << 4));
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j) acc[i][j] = Mfma<T>::run(a[i], b[j], acc[i][j]);
  }
}

__device__ __forceinline__ float bf_round(float v, bf16*) { return __bfloat162float(__float2bfloat16(v)); }
__device__ __forceinline__ float bf_round(float v, fp16*) { return __half2float(__float2half(v)); }

template <typename T>
__device__ __forceinline__ void unpack4(uint2 v, float (&o)[4]) {
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = to_f32(e[k]);
}

// Fragments of one k-step (both 32-deep halves) for one wave: W rows nrow0 + [0, 64), x rows
// mrow0 + [0, 128)
template <typename T>
__device__ __forceinline__ void read_frags(const char* img, int nrow0, int mrow0, uint4 (&fa)[2][NI],
                                           uint4 (&fb)[2][MJ], int lane) {
  const int lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = nrow0 + 16 * i + lr;
      fa[s][i] = *reinterpret_cast<const uint4*>(img + r * ROWB + (((4 * s + lg) ^ swz(r)) << 4));
    }
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int r = mrow0 + 16 * j + lr;
      fb[s][j] = *reinterpret_cast<const uint4*>(img + IMG + r * ROWB +
                                                 (((4 * s + lg) ^ swz(r)) << 4));
    }
  }
}

template <typename T>
__device__ __forceinline__ void mfma_step(const uint4 (&fa)[2][NI], const uint4 (&fb)[2][MJ],
                                          f32x4 (&acc)[NI][MJ]) {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j) acc[i][j] = Mfma<T>::run(fa[s][i], fb[s][j], acc[i][j]);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void wait_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <typename T, int EPI, bool PP>
__global__ void __launch_bounds__(NT, 1) mlp_gemm_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * STAGE_B];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware bijective remap: blocks are dealt round-robin over the 8 XCDs, so XCD x gets the
  // consecutive virtual ids [x * nb / 8, (x + 1) * nb / 8)
  const int nb = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // grouped order: GROUP_M row tiles x every column tile, row tile fastest
  const int gsz = a.group_m * a.tiles_n;
  const int g = v / gsz, first_m = g * a.group_m;
  const int gm = min(a.tiles_m - first_m, a.group_m);
  const int tm = first_m + (v - g * gsz) % gm, tn = (v - g * gsz) / gm;
  const int m0 = tm * BM, mvalid = min(BM, a.M - m0);
  const T* xb = reinterpret_cast<const T*>(a.x) + (long long)m0 * a.ldx;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int nrow0 = wn * (BN / WN), mrow0 = wm * (BM / WM);

  f32x4 acc[NI][MJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
  if constexpr (!PP) {
    stage<T, EPI>(lds, a, xb, mvalid, tn, 0, wid, lane);
    for (int kt = 0; kt < nk; ++kt) {
      wait_vm<0>();   // this wave's pieces of stage kt have landed
      lds_barrier();  // ... every wave's; and every wave is done reading stage kt - 1's buffer
      if (kt + 1 < nk)
        stage<T, EPI>(lds + ((kt + 1) & 1) * STAGE_B, a, xb, mvalid, tn, (kt + 1) * BK, wid, lane);
      compute<T>(lds + (kt & 1) * STAGE_B, nrow0, mrow0, acc, lane);
    }
  } else {
    // Ping-pong: wave group 0 (waves 0-3, output rows 0-127) and group 1 (waves 4-7, rows
    // 128-255) alternate between a LOAD interval (this k-step's fragments LDS -> registers, plus
    // its share of a later stage's LDS-DMA) and a COMPUTE interval (64 MFMAs on the fragments in
    // registers), one barrier between intervals, group 1 one interval behind group 0: on every
    // SIMD (one wave of each group) one wave's MFMAs cover the other's LDS reads and DMA issue.
    // Stage k (buffer k & 1) is read in intervals 2k (group 0) and 2k + 1 (group 1).  Its buffer
    // is refilled with stage k + 2 by group 1 at the end of interval 2k + 1 (after its own reads
    // completed) and by group 0 at the start of 2k + 2; both halves are waited for (counted
    // vmcnt) before the barrier that ends interval 2k + 3.
    uint4 fa[2][NI], fb[2][MJ];
    const bool g1 = wid >= 4;
    stage<T, EPI>(lds, a, xb, mvalid, tn, 0, wid, lane);
    if (g1) {
      if (nk > 1) {
        stage<T, EPI>(lds + STAGE_B, a, xb, mvalid, tn, BK, wid, lane);
        wait_vm<8>();
      } else {
        wait_vm<0>();
      }
    } else {
      wait_vm<0>();
    }
    bar();
    if (!g1) {
      for (int k = 0; k < nk; ++k) {
        // interval 2k: load step k, issue this group's half of stage k + 1
        read_frags<T>(lds + (k & 1) * STAGE_B, nrow0, mrow0, fa, fb, lane);
        if (k + 1 < nk)
          stage<T, EPI>(lds + ((k + 1) & 1) * STAGE_B, a, xb, mvalid, tn, (k + 1) * BK, wid, lane);
        wait_lds();
        bar();
        // interval 2k + 1: compute step k; stage k + 1 (this group's half) must have landed
        mfma_step<T>(fa, fb, acc);
        if (k + 1 < nk) wait_vm<0>();
        bar();
      }
    } else {
      for (int k = 0; k < nk; ++k) {
        // interval 2k: compute step k - 1
        if (k > 0) mfma_step<T>(fa, fb, acc);
        bar();
        // interval 2k + 1: load step k; refill its buffer with stage k + 2; stage k + 1 landed
        read_frags<T>(lds + (k & 1) * STAGE_B, nrow0, mrow0, fa, fb, lane);
        wait_lds();
        if (k + 2 < nk) {
          stage<T, EPI>(lds + (k & 1) * STAGE_B, a, xb, mvalid, tn, (k + 2) * BK, wid, lane);
          wait_vm<8>();
        } else {
          wait_vm<0>();
        }
        bar();
      }
      mfma_step<T>(fa, fb, acc);  // interval 2 nk: the last step
    }
  }

  // lane holds C[m = mrow0 + 16 j + (lane & 15)][n = nrow0 + 16 i + 4 (lane >> 4) + 0..3]
  const int lr = lane & 15, lg = lane >> 4;
  T* c = reinterpret_cast<T*>(a.c);
  if constexpr (EPI == kStore) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = mrow0 + 16 * j + lr;
      if (m >= mvalid) continue;
      T* row = c + (long long)(m0 + m) * a.ldc + tn * BN + nrow0 + 4 * lg;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        *reinterpret_cast<uint2*>(row + 16 * i) =
            make_uint2(pk2<T>(acc[i][j][0], acc[i][j][1]), pk2<T>(acc[i][j][2], acc[i][j][3]));
    }
  } else if constexpr (EPI == kSwiGLU) {
    // fragments 0, 1: gate of activation columns 128 tn + 32 wn + 16 i + 4 lg + e; 2, 3: up
    T* act = reinterpret_cast<T*>(a.act);
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = mrow0 + 16 * j + lr;
      if (m >= mvalid) continue;
      const long long row = m0 + m;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int na = tn * 128 + wn * 32 + 16 * i + 4 * lg;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // the activation of the ROUNDED g / u: the values the backward reads back
          const float gg = bf_round(acc[i][j][e], (T*)nullptr);
          const float uu = bf_round(acc[i + 2][j][e], (T*)nullptr);
          o[e] = silu(gg) * uu;
        }
        *reinterpret_cast<uint2*>(c + row * a.ldc + na) =
            make_uint2(pk2<T>(acc[i][j][0], acc[i][j][1]), pk2<T>(acc[i][j][2], acc[i][j][3]));
        *reinterpret_cast<uint2*>(c + row * a.ldc + a.F + na) = make_uint2(
            pk2<T>(acc[i + 2][j][0], acc[i + 2][j][1]), pk2<T>(acc[i + 2][j][2], acc[i + 2][j][3]));
        *reinterpret_cast<uint2*>(act + row * a.ldact + na) =
            make_uint2(pk2<T>(o[0], o[1]), pk2<T>(o[2], o[3]));
      }
    }
  } else {
    // dact = acc (f32, never rounded); g / u from the saved gu; writes dg | du
    const T* gu = reinterpret_cast<const T*>(a.gu);
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = mrow0 + 16 * j + lr;
      const long long row = m0 + min(m, mvalid - 1);  // clamped: loads stay unconditional
      uint2 gv[NI], uv[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int n = tn * BN + nrow0 + 16 * i + 4 * lg;
        gv[i] = *reinterpret_cast<const uint2*>(gu + row * a.ldgu + n);
        uv[i] = *reinterpret_cast<const uint2*>(gu + row * a.ldgu + a.F + n);
      }
      if (m >= mvalid) continue;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int n = tn * BN + nrow0 + 16 * i + 4 * lg;
        float g[4], u[4], dg[4], du[4];
        unpack4<T>(gv[i], g);
        unpack4<T>(uv[i], u);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[i][j][e];
          const float sg = 1.f / (1.f + __expf(-g[e]));
          du[e] = d * g[e] * sg;
          dg[e] = d * u[e] * sg * (1.f + g[e] * (1.f - sg));
        }
        *reinterpret_cast<uint2*>(c + row * a.ldc + n) =
            make_uint2(pk2<T>(dg[0], dg[1]), pk2<T>(dg[2], dg[3]));
        *reinterpret_cast<uint2*>(c + row * a.ldc + a.F + n) =
            make_uint2(pk2<T>(du[0], du[1]), pk2<T>(du[2], du[3]));
      }
    }
  }
}

template <typename T, bool PP>
hipError_t launch(int epi, const Args& a, hipStream_t st) {
  dim3 grid(a.tiles_m * a.tiles_n), block(NT);
  if (epi == kStore)
    hipLaunchKernelGGL((mlp_gemm_kernel<T, kStore, PP>), grid, block, 0, st, a);
  else if (epi == kSwiGLU)
    hipLaunchKernelGGL((mlp_gemm_kernel<T, kSwiGLU, PP>), grid, block, 0, st, a);
  else if (epi == kSwiGLUBwd)
    hipLaunchKernelGGL((mlp_gemm_kernel<T, kSwiGLUBwd, PP>), grid, block, 0, st, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace mg
}  // namespace lumen

// epi 0: c[M, N] = x[M, K] @ w[N, K]^T                     (N % 256 == 0)
// epi 1: c = gu[M, 2F] = x @ w[2F, K]^T, act[M, F] = silu(g) * u   (N == 2F, F % 128 == 0)
// epi 2: dact = x @ w[F, K]^T (x = dout, w = Wd^T); c = dgu[M, 2F] from dact and gu[M, 2F]
//        (N == F, F % 256 == 0)
// K % 64 == 0; row strides in elements: ldx, ldw % 8 == 0, ldc / ldact / ldgu % 4 == 0; every
// base 16-byte aligned; group_m: row tiles per tile group (L2 reuse order), >= 1.
extern "C" hipError_t lumen_mlp_gemm(int dtype, int epi, const void* x, long long ldx,
                                     const void* w, long long ldw, void* c, long long ldc,
                                     void* act, long long ldact, const void* gu, long long ldgu,
                                     int M, int N, int K, int F, int group_m, hipStream_t st) {
  using namespace lumen::mg;
  const bool pp = (epi & 16) == 0;  // bit 4: the plain two-stage loop (A/B probe)
  epi &= 15;
  if (M < 1 || K < BK || K % BK || group_m < 1 || ldx < K || ldw < K || ldx % 8 || ldw % 8 ||
      ldc % 4 || x == nullptr || w == nullptr || c == nullptr)
    return hipErrorInvalidValue;
  long long wrows = N;
  if (epi == kStore) {
    if (N % BN || ldc < N) return hipErrorInvalidValue;
  } else if (epi == kSwiGLU) {
    if (N != 2 * F || F % 128 || ldc < 2LL * F || act == nullptr || ldact < F || ldact % 4)
      return hipErrorInvalidValue;
  } else if (epi == kSwiGLUBwd) {
    if (N != F || F % BN || ldc < 2LL * F || gu == nullptr || ldgu < 2LL * F || ldgu % 4)
      return hipErrorInvalidValue;
  } else {
    return hipErrorInvalidValue;
  }
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) |
        reinterpret_cast<uintptr_t>(c) | reinterpret_cast<uintptr_t>(act) |
        reinterpret_cast<uintptr_t>(gu)) & 15) != 0)
    return hipErrorInvalidValue;
  // every 32-bit lane offset of the DMAs stays below 2^32 bytes
  if (wrows * ldw * 2 >= (1LL << 32) || (long long)BM * ldx * 2 >= (1LL << 32))
    return hipErrorInvalidValue;
  Args a{x, w, c, act, gu, ldx, ldw, ldc, ldact, ldgu, M, N, K, F, (M + BM - 1) / BM,
         epi == kSwiGLU ? F / 128 : N / BN, group_m};
  if (dtype == lumen::kBF16)
    return pp ? launch<lumen::bf16, true>(epi, a, st) : launch<lumen::bf16, false>(epi, a, st);
  if (dtype == lumen::kF16)
    return pp ? launch<lumen::fp16, true>(epi, a, st) : launch<lumen::fp16, false>(epi, a, st);
  return hipErrorInvalidValue;
}
