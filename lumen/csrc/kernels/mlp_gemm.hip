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
  // last-wave split: tiles [full, full + split) run as two k halves each (blocks full + 2u,
  // full + 2u + 1), f32 partial slabs in ws, the last-arriving half (ticket in cnt[u]) sums
  // both and runs the epilogue
  int full, split;
  float* ws;
  int* cnt;
};

// W image row r -> output column within its 32-row group: image row 16 i' + 4 g + e (fragment
// i' of a pair, lane group g, accumulator e) holds column 8 g + 4 i' + e, so a lane's
// accumulators of the two fragments of a pair are 8 CONSECUTIVE columns: 16-byte stores
__device__ __forceinline__ int colperm(int r) {
  return (r & ~31) | (((r >> 2) & 3) << 3) | (((r >> 4) & 1) << 2) | (r & 3);
}

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
        wrow = (w < 32 ? 0 : a.F) + tn * 128 + (r >> 6) * 32 + colperm(w & 31);
      } else {
        wrow = tn * BN + colperm(r);
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

// The W image rows of wave slot wn (rows 64 wn .. 64 wn + 63 = pieces 8 wn .. 8 wn + 7), issued by
// one wave (ping-pong loop)
template <typename T, int EPI>
__device__ __forceinline__ void stage_w(char* img, const Args& a, int tn, int k0, int wn,
                                        int lane) {
  const int rr = lane >> 3, c = lane & 7;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = 8 * wn + q;
    const int r = 8 * p + rr;
    const int ch = c ^ swz(r);
    int wrow;
    if constexpr (EPI == kSwiGLU) {
      const int w = r & 63;
      wrow = (w < 32 ? 0 : a.F) + tn * 128 + (r >> 6) * 32 + colperm(w & 31);
    } else {
      wrow = tn * BN + colperm(r);
    }
    const unsigned off = (unsigned)(((long long)wrow * a.ldw + k0 + 8 * ch) * (long long)sizeof(T));
    dma16(a.w, off, img + p * 8 * ROWB);
  }
}

// The whole x image (32 pieces), issued by the 4 waves of one group: wave wl issues wl + 4q
template <typename T>
__device__ __forceinline__ void stage_x(char* img, const Args& a, const T* xb, int mvalid, int k0,
                                        int wl, int lane) {
  const int rr = lane >> 3, c = lane & 7;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = wl + 4 * q;
    const int r = 8 * p + rr;
    const int ch = c ^ swz(r);
    const int m = min(r, mvalid - 1);
    const unsigned off = (unsigned)(((long long)m * a.ldx + k0 + 8 * ch) * (long long)sizeof(T));
    dma16(xb, off, img + IMG + p * 8 * ROWB);
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

// keeps fragment registers alive in a probe build without MFMAs (no DCE of the reads)
__device__ __forceinline__ void keep_live(uint4 (&fa)[2][NI], uint4 (&fb)[2][MJ]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      asm volatile("" : "+v"(fa[s][i].x), "+v"(fa[s][i].y), "+v"(fa[s][i].z), "+v"(fa[s][i].w));
#pragma unroll
    for (int j = 0; j < MJ; ++j)
      asm volatile("" : "+v"(fb[s][j].x), "+v"(fb[s][j].y), "+v"(fb[s][j].z), "+v"(fb[s][j].w));
  }
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void wait_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// PROBE (cost split, plain store only; the output is garbage): bit 0 = no LDS-DMA after the
// prologue, bit 1 = no fragment reads, bit 2 = no MFMAs.  LOOP: 0 plain two-stage loop, 1
// ping-pong over two 64-deep stages.  (Two LDS rings -- 5 half-step slots of 64-byte rows, and 10
// quarter slots -- were measured 1.22-1.25x the library and removed: profiles/r6_mlp_gemm.)
template <typename T, int EPI, int LOOP, int PROBE = 0>
__global__ void __launch_bounds__(NT, 1) mlp_gemm_kernel(Args a) {
  constexpr bool PP = LOOP == 1;
  __shared__ __attribute__((aligned(16))) char lds[NSTAGE * STAGE_B];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware bijective remap: blocks are dealt round-robin over the 8 XCDs, so XCD x gets the
  // consecutive virtual ids [x * nb / 8, (x + 1) * nb / 8)
  const int bid = blockIdx.x;
  int v, slice = -1;
  if (bid < a.full) {
    const int nb = a.full;
    const int xcd = bid & 7, q8 = nb >> 3, r8 = nb & 7;
    v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  } else {  // the split last wave: dispatched last, dealt over every XCD in block order
    const int u = bid - a.full;
    v = a.full + (u >> 1);
    slice = u & 1;
  }
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

  // k-steps of this block: all of K, or one half of it for a split tile
  const int nk_all = a.K / BK;
  const int kb = slice == 1 ? nk_all / 2 : 0;
  const int nk = slice < 0 ? nk_all : slice == 0 ? nk_all / 2 : nk_all - nk_all / 2;
  const int kofs = kb * BK;
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
    // LDS-DMA of a later stage) and a COMPUTE interval (64 MFMAs on the fragments in registers),
    // one barrier between intervals, group 1 one interval behind group 0: on every SIMD (one
    // wave of each group) one wave's MFMAs cover the other's LDS reads and DMA issue.  DMA is
    // issued only in load intervals (issued before its MFMAs it delays the MFMA cluster: measured
    // 1.22x slower).
    // Stage k (buffer k & 1) is read in intervals 2k (group 0) and 2k + 1 (group 1).  Refills,
    // race-free by construction:
    //  * W image of stage k + 2: group 1 wave wn, right after its own reads of stage k complete,
    //    writes exactly the 64 W rows only it (and group 0's wave wn, one interval earlier) reads;
    //  * x image of stage k + 1: group 0 at the start of interval 2k, after the barrier that
    //    follows group 1's last reads of that buffer (interval 2k - 1).
    // Each group retires its pieces (counted vmcnt) before the barrier ahead of their first
    // reader: ~2 intervals of load latency covered.
    uint4 fa[2][NI], fb[2][MJ];
    const bool g1 = wid >= 4;
    const int wl = wid & 3;
    if (!g1) {
      stage_x<T>(lds, a, xb, mvalid, kofs, wl, lane);
      wait_vm<0>();
    } else {
      stage_w<T, EPI>(lds, a, tn, kofs, wn, lane);
      if (nk > 1) {
        stage_w<T, EPI>(lds + STAGE_B, a, tn, kofs + BK, wn, lane);
        wait_vm<8>();
      } else {
        wait_vm<0>();
      }
    }
    bar();
    if (!g1) {
      for (int k = 0; k < nk; ++k) {
        // interval 2k: x image of stage k + 1; load step k
        if (k + 1 < nk && !(PROBE & 1))
          stage_x<T>(lds + ((k + 1) & 1) * STAGE_B, a, xb, mvalid, kofs + (k + 1) * BK, wl, lane);
        if (!(PROBE & 2)) read_frags<T>(lds + (k & 1) * STAGE_B, nrow0, mrow0, fa, fb, lane);
        wait_lds();
        bar();
        // interval 2k + 1: compute step k; the x image of stage k + 1 must have landed
        if (!(PROBE & 4)) mfma_step<T>(fa, fb, acc); else keep_live(fa, fb);
        if (k + 1 < nk) wait_vm<0>();
        bar();
      }
    } else {
      for (int k = 0; k < nk; ++k) {
        // interval 2k: compute step k - 1
        if (k > 0) {
          if (!(PROBE & 4)) mfma_step<T>(fa, fb, acc); else keep_live(fa, fb);
        }
        bar();
        // interval 2k + 1: load step k; then this wave's W rows of stage k + 2; W of stage
        // k + 1 landed
        if (!(PROBE & 2)) read_frags<T>(lds + (k & 1) * STAGE_B, nrow0, mrow0, fa, fb, lane);
        wait_lds();
        if (k + 2 < nk && !(PROBE & 1)) {
          stage_w<T, EPI>(lds + (k & 1) * STAGE_B, a, tn, kofs + (k + 2) * BK, wn, lane);
          wait_vm<8>();
        } else {
          wait_vm<0>();
        }
        bar();
      }
      if (!(PROBE & 4)) mfma_step<T>(fa, fb, acc); else keep_live(fa, fb);  // the last step
    }
  }

  if (slice >= 0) {
    // split tile: publish this half's partial sums, take a ticket; the second half to arrive
    // adds the other's slab and runs the epilogue (decode_gemm.hip's protocol: plain slab
    // stores, agent-scope release before the ticket, acquire by the last arriver)
    const int u = v - a.full;
    float* mine = a.ws + ((long long)u * 2 + slice) * (NT * NI * MJ * 4);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        *reinterpret_cast<f32x4*>(mine + ((i * MJ + j) * NT + threadIdx.x) * 4) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(a.cnt + u, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == 1;
      if (last) {
        __hip_atomic_store(a.cnt + u, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    const float* other = a.ws + ((long long)u * 2 + (slice ^ 1)) * (NT * NI * MJ * 4);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        acc[i][j] += *reinterpret_cast<const f32x4*>(other + ((i * MJ + j) * NT + threadIdx.x) * 4);
  }

  // lane (lr, lg) holds, for the fragment pair h (fragments 2h, 2h + 1), row
  // m = mrow0 + 16 j + lr and the 8 consecutive columns nrow0 + 32 h + 8 lg + [0, 8) (colperm):
  // v[0..3] = acc[2h][j][0..3], v[4..7] = acc[2h + 1][j][0..3]
  const int lr = lane & 15, lg = lane >> 4;
  T* c = reinterpret_cast<T*>(a.c);
  const auto pack8 = [&](const f32x4& x, const f32x4& y) {
    return make_uint4(pk2<T>(x[0], x[1]), pk2<T>(x[2], x[3]), pk2<T>(y[0], y[1]),
                      pk2<T>(y[2], y[3]));
  };
  if constexpr (EPI == kStore) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = mrow0 + 16 * j + lr;
      if (m >= mvalid) continue;
      T* row = c + (long long)(m0 + m) * a.ldc + tn * BN + nrow0 + 8 * lg;
#pragma unroll
      for (int h = 0; h < NI / 2; ++h)
        *reinterpret_cast<uint4*>(row + 32 * h) = pack8(acc[2 * h][j], acc[2 * h + 1][j]);
    }
  } else if constexpr (EPI == kSwiGLU) {
    // pair 0 (fragments 0, 1): gate of activation columns 128 tn + 32 wn + 8 lg + [0, 8);
    // pair 1 (fragments 2, 3): up of the same columns
    T* act = reinterpret_cast<T*>(a.act);
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = mrow0 + 16 * j + lr;
      if (m >= mvalid) continue;
      const long long row = m0 + m;
      const int na = tn * 128 + wn * 32 + 8 * lg;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // the activation of the ROUNDED g / u: the values the backward reads back
        const float gg = bf_round(acc[e >> 2][j][e & 3], (T*)nullptr);
        const float uu = bf_round(acc[2 + (e >> 2)][j][e & 3], (T*)nullptr);
        o[e] = silu(gg) * uu;
      }
      *reinterpret_cast<uint4*>(c + row * a.ldc + na) = pack8(acc[0][j], acc[1][j]);
      *reinterpret_cast<uint4*>(c + row * a.ldc + a.F + na) = pack8(acc[2][j], acc[3][j]);
      *reinterpret_cast<uint4*>(act + row * a.ldact + na) =
          make_uint4(pk2<T>(o[0], o[1]), pk2<T>(o[2], o[3]), pk2<T>(o[4], o[5]),
                     pk2<T>(o[6], o[7]));
    }
  } else {
    // dact = acc (f32, never rounded); g / u from the saved gu; writes dg | du
    const T* gu = reinterpret_cast<const T*>(a.gu);
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = mrow0 + 16 * j + lr;
      const long long row = m0 + min(m, mvalid - 1);  // clamped: loads stay unconditional
      uint4 gv[NI / 2], uv[NI / 2];
#pragma unroll
      for (int h = 0; h < NI / 2; ++h) {
        const int n = tn * BN + nrow0 + 32 * h + 8 * lg;
        gv[h] = *reinterpret_cast<const uint4*>(gu + row * a.ldgu + n);
        uv[h] = *reinterpret_cast<const uint4*>(gu + row * a.ldgu + a.F + n);
      }
      if (m >= mvalid) continue;
#pragma unroll
      for (int h = 0; h < NI / 2; ++h) {
        const int n = tn * BN + nrow0 + 32 * h + 8 * lg;
        float g[8], u[8], dg[8], du[8];
        const T* ge = reinterpret_cast<const T*>(&gv[h]);
        const T* ue = reinterpret_cast<const T*>(&uv[h]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          g[e] = to_f32(ge[e]);
          u[e] = to_f32(ue[e]);
          const float d = acc[2 * h + (e >> 2)][j][e & 3];
          const float sg = 1.f / (1.f + __expf(-g[e]));
          du[e] = d * g[e] * sg;
          dg[e] = d * u[e] * sg * (1.f + g[e] * (1.f - sg));
        }
        store8(c + row * a.ldc + n, dg);
        store8(c + row * a.ldc + a.F + n, du);
      }
    }
  }
}

template <typename T, int LOOP>
hipError_t launch(int epi, const Args& a, hipStream_t st) {
  dim3 grid(a.full + 2 * a.split), block(NT);
  const int probe = (epi >> 5) & 7;
  epi &= 15;
  if (probe && LOOP && epi == kStore) {
#define LUMEN_MG_PROBE(P) \
    if (probe == P) hipLaunchKernelGGL((mlp_gemm_kernel<T, kStore, LOOP, P>), grid, block, 0, st, a);
    LUMEN_MG_PROBE(1) LUMEN_MG_PROBE(2) LUMEN_MG_PROBE(3) LUMEN_MG_PROBE(4) LUMEN_MG_PROBE(5)
    LUMEN_MG_PROBE(6)
#undef LUMEN_MG_PROBE
    return hipGetLastError();
  }
  if (epi == kStore)
    hipLaunchKernelGGL((mlp_gemm_kernel<T, kStore, LOOP>), grid, block, 0, st, a);
  else if (epi == kSwiGLU)
    hipLaunchKernelGGL((mlp_gemm_kernel<T, kSwiGLU, LOOP>), grid, block, 0, st, a);
  else if (epi == kSwiGLUBwd)
    hipLaunchKernelGGL((mlp_gemm_kernel<T, kSwiGLUBwd, LOOP>), grid, block, 0, st, a);
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
// ws / cnt (optional, both or neither): when the last wave of tiles fills at most half the CUs
// it runs split in two k halves (ws: split * 2 * 65536 floats, cnt: split zeroed ints, which
// the launch leaves zeroed); lumen_mlp_gemm_split() says how many tiles that is
extern "C" int lumen_mlp_gemm_split(int M, int N, int K, int epi, int cus) {
  const int tm = (M + lumen::mg::BM - 1) / lumen::mg::BM;
  const int tn = (epi & 15) == lumen::mg::kSwiGLU ? N / 256 : N / lumen::mg::BN;
  const int total = tm * tn, rem = cus > 0 ? total % cus : 0;
  if ((epi & 16) || total < cus || rem == 0 || 2 * rem > cus || K / lumen::mg::BK < 4) return 0;
  return rem;
}

extern "C" hipError_t lumen_mlp_gemm(int dtype, int epi, const void* x, long long ldx,
                                     const void* w, long long ldw, void* c, long long ldc,
                                     void* act, long long ldact, const void* gu, long long ldgu,
                                     int M, int N, int K, int F, int group_m, float* ws, int* cnt,
                                     int split, hipStream_t st) {
  using namespace lumen::mg;
  // bit 4: the plain two-stage loop (A/B probe); default: ping-pong over two stages
  if (epi & ~(15 | 16 | (7 << 5))) return hipErrorInvalidValue;
  const int loop = (epi & 16) ? 0 : 1;
  const int probe_bits = epi & (7 << 5);  // bits 5-7: cost-split probe builds (plain store)
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
  const int tiles_m = (M + BM - 1) / BM, tiles_n = epi == kSwiGLU ? F / 128 : N / BN;
  if (split < 0 || split > tiles_m * tiles_n || (split > 0 && (ws == nullptr || cnt == nullptr)) ||
      (split > 0 && loop != 1))
    return hipErrorInvalidValue;
  Args a{x, w, c, act, gu, ldx, ldw, ldc, ldact, ldgu, M, N, K, F, tiles_m, tiles_n, group_m,
         tiles_m * tiles_n - split, split, ws, cnt};
  if (dtype == lumen::kBF16)
    return loop == 1 ? launch<lumen::bf16, 1>(epi | probe_bits, a, st)
                       : launch<lumen::bf16, 0>(epi, a, st);
  if (dtype == lumen::kF16)
    return loop == 1 ? launch<lumen::fp16, 1>(epi, a, st) : launch<lumen::fp16, 0>(epi, a, st);
  return hipErrorInvalidValue;
}
