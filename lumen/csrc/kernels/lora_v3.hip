// LoRA adapter passes, third generation (gfx950, v_mfma_f32_16x16x32 on bf16/fp16).
//
// Reference behaviour: PEFT LoraLayer under fp16 autocast (training/train_baseline.py:131-141,
// r=16, alpha=32, dropout 0.05 on q/k/v/o).  The adapter products are memory-bound streams over
// the [T, K] activation and the [T, N] output / output-gradient; lora_v2.hip ran them at ~50% of
// HBM speed (profiles/r03_lora).  This file restructures them around bytes in flight and the
// number of passes instead of around LDS images:
//
//   down3  Z  = drop(x) A^T           one shot per wave: 64 rows x 128 k loaded straight into the
//                                     MFMA A-operand registers (no LDS image), the 8 waves of a
//                                     block cover 1024 k and meet in an LDS tile (ds_add_f32);
//                                     one global f32 atomic per (row, j) per 1024 k.
//   up3    y  += s Z B^T  (+RoPE)     swapped-operand MFMA whose row map puts 32 consecutive output
//          dx += drop(dZ A)           columns of one row in each lane: the read-modify-write of the
//                                     output is lane-local 16-byte vectors (no f32 LDS scratch) and
//                                     the rotate_half partner (column ^ 64) is in the same lane.
//   dy3    dZ = s dY B,  dB = s dY^T Z   ONE pass over dY for both backward products (v2 read dY
//                                     twice): the staged [64 x 128] dY tile feeds the dZ MFMAs with
//                                     row reads and the dB MFMAs with ds_read_b64_tr_b16 reads.
//
// Dropout is the same counter hash as lora_v2 (common.h dropout_keep8), so masks regenerate
// bit-identically across kernels and against lumen.ops.lora.dropout_mask_ref.
#include "tile128.h"
#include "det.h"

namespace lumen {
namespace lv3 {

using namespace tile;

struct Drop {
  unsigned int seed, thresh;
  float scale;      // 1 / (1 - p)
  long long ld;     // logical row length of the dropout index (t * ld + col0 + col)
  long long col0;
};

__device__ __forceinline__ uint4 mask8(uint4 u, uint32_t keep) {
  const auto wm = [keep](int w) {
    return ((keep >> (2 * w)) & 1u ? 0x0000FFFFu : 0u) | ((keep >> (2 * w + 1)) & 1u ? 0xFFFF0000u : 0u);
  };
  return make_uint4(u.x & wm(0), u.y & wm(1), u.z & wm(2), u.w & wm(3));
}

// 8 consecutive f32 -> packed 16-bit MFMA operand (zeros when !ok)
template <typename T>
__device__ __forceinline__ uint4 ld_f32x8(const float* p, bool ok) {
  if (!ok) return make_uint4(0, 0, 0, 0);
  const float4 u = *reinterpret_cast<const float4*>(p);
  const float4 v = *reinterpret_cast<const float4*>(p + 4);
  return make_uint4(pk2<T>(u.x, u.y), pk2<T>(u.z, u.w), pk2<T>(v.x, v.y), pk2<T>(v.z, v.w));
}

// ------------------------------------------------------------------------------------------
// down3:  Z[t, j] += alpha * sum_k drop(x)[t, k] * A[j, k]      j < R = 16 * NJ
// grid (ceil(T / 64), ceil(K / 1024)), block 512 (8 waves x 128 k)
// ------------------------------------------------------------------------------------------
struct DownArgs {
  const void* x; long long ldx;
  const float* A; long long lda;
  float* Z; long long ldz;
  int T, K;
  float alpha;
  Drop drop;
  int probe;   // cost probes (0 in production): 1 no dropout hash, 2 no A loads, 4 no reduction,
               // 8 no global atomics
  // fused fold tail (xe != nullptr): the last of the gridDim.y K-blocks of a 64-row tile to
  // arrive writes xe[t, xk + c] = c < J ? Z[t, c] : 0 for c < KP (16-bit), so no separate
  // z_tail launch.  cnt[blockIdx.x] arrival counters: zero on entry, left at zero.
  void* xe; long long ldxe; int xk, KP;
  unsigned* cnt;
  // deterministic sum (slab != nullptr, cnt required): each K-block's [64 x J] partial goes to
  // slab[(blockIdx.x * gridDim.y + blockIdx.y) * 64 * J] (write-through), the last K-block of the
  // row tile sums them in K order and writes Z (det.h) -- no f32 atomics
  float* slab;
};

template <typename T, bool DROP, int NJ>
__global__ void __launch_bounds__(512) down3_kernel(DownArgs a) {
  constexpr int J = NJ * 16, JP = J + 4;   // padded LDS row: the 4 g-rows of a store hit
  __shared__ float red[4][64 * JP];        // distinct bank groups
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, L = lane & 15, g = lane >> 4;
  const int t0 = blockIdx.x * 64;
  const int k0 = (blockIdx.y * 8 + wid) * 128;
  f32x4 acc[4][NJ];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int jt = 0; jt < NJ; ++jt) acc[rt][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (k0 < a.K) {
    const T* x = reinterpret_cast<const T*>(a.x);
    uint4 xv[4][4];
    // every load of the wave's 64 x 128 tile is in flight before the first MFMA
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = t0 + rt * 16 + L, c = k0 + 32 * i + 8 * g;
        xv[rt][i] = (t < a.T && c < a.K)
                        ? *reinterpret_cast<const uint4*>(x + (long long)t * a.ldx + c)
                        : make_uint4(0, 0, 0, 0);
      }
    // the A operand (f32 rows, L2-resident) is loaded right behind the x tile and
    // unconditionally (clamped addresses, out-of-range columns zeroed by a select after the
    // load): guarded loads made hipcc wait for every pair of them in turn -- 12 dependent L2
    // round trips after the x tile had landed -- instead of one wait for both
    float4 af[4][NJ][2];
    if (!(a.probe & 2)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = min(k0 + 32 * i + 8 * g, a.K - 8);
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt) {
          const float* ap = a.A + (long long)(jt * 16 + L) * a.lda + c;
          af[i][jt][0] = *reinterpret_cast<const float4*>(ap);
          af[i][jt][1] = *reinterpret_cast<const float4*>(ap + 4);
        }
      }
    }
    if (DROP && !(a.probe & 1)) {
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long long t = t0 + rt * 16 + L;
          const int c = k0 + 32 * i + 8 * g;
          xv[rt][i] = mask8(xv[rt][i], dropout_keep8(a.drop.seed,
                                                     (unsigned long long)(t * a.drop.ld + a.drop.col0 + c),
                                                     a.drop.thresh));
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool cok = k0 + 32 * i + 8 * g < a.K;
      uint4 bop[NJ];
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) {
        const float4 u = af[i][jt][0], v = af[i][jt][1];
        const uint4 w = make_uint4(pk2<T>(u.x, u.y), pk2<T>(u.z, u.w), pk2<T>(v.x, v.y),
                                   pk2<T>(v.z, v.w));
        bop[jt] = (a.probe & 2) ? xv[jt & 3][i] : (cok ? w : make_uint4(0, 0, 0, 0));
      }
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt) acc[rt][jt] = Mfma<T>::run(xv[rt][i], bop[jt], acc[rt][jt]);
    }
  }
  if (a.probe & 4) {
    float sacc = 0.f;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) sacc += acc[rt][jt][0] + acc[rt][jt][3];
    if (sacc == 1234.5f) a.Z[threadIdx.x] = sacc;
    return;
  }
  // two-phase LDS reduction of the 8 waves' [64 x J] partials with plain stores / loads:
  // waves 4..7 park theirs in slots 0..3, waves 0..3 add their own in place, then every thread
  // sums the 4 slots of its output elements.  Accumulator lane (L, g), element r = row
  // 16 rt + 4 g + r, column 16 jt + L.
  float* slot = red[wid & 3];
  if (wid >= 4) {
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) slot[(rt * 16 + g * 4 + r) * JP + jt * 16 + L] = acc[rt][jt][r];
  }
  __syncthreads();
  if (wid < 4) {
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) slot[(rt * 16 + g * 4 + r) * JP + jt * 16 + L] += acc[rt][jt][r];
  }
  __syncthreads();
  const float alpha = DROP ? a.alpha * a.drop.scale : a.alpha;
  if (a.slab != nullptr) {
    float* mine = a.slab + ((long long)blockIdx.x * gridDim.y + blockIdx.y) * (64 * J);
    for (int i = threadIdx.x; i < 64 * J; i += 512) {
      const int o = (i / J) * JP + i % J;
      det::st_wt(mine + i, alpha * (red[0][o] + red[1][o] + red[2][o] + red[3][o]));
    }
    if (a.cnt == nullptr) return;  // split form: down3_reduce_kernel sums the slabs
    __shared__ int lastf;
    if (!det::last_arriver(a.cnt + blockIdx.x, gridDim.y, &lastf)) return;
    // the row tile's sum in K-block order; Z written once, the fold tail straight from it
    const float* base = a.slab + (long long)blockIdx.x * gridDim.y * (64 * J);
    T* xe = reinterpret_cast<T*>(a.xe);
    for (int i = threadIdx.x; i < 32 * J; i += 512) {  // pairs of columns
      const int row = (2 * i) / J, j = (2 * i) % J, t = t0 + row;
      const float2 v = det::sum_pairs(base + 2 * i, 64LL * J, gridDim.y);
      if (t < a.T) {
        *reinterpret_cast<float2*>(a.Z + (long long)t * a.ldz + j) = v;
        if (xe != nullptr) {
          xe[(long long)t * a.ldxe + a.xk + j] = from_f32<T>(v.x);
          xe[(long long)t * a.ldxe + a.xk + j + 1] = from_f32<T>(v.y);
        }
      }
    }
    if (xe != nullptr) {  // zero tail columns J .. KP
      for (int i = threadIdx.x; i < 64 * (a.KP - J); i += 512) {
        const int row = i / (a.KP - J), c = J + i % (a.KP - J), t = t0 + row;
        if (t < a.T) xe[(long long)t * a.ldxe + a.xk + c] = from_f32<T>(0.f);
      }
    }
    return;
  }
  for (int i = threadIdx.x; i < 64 * J; i += 512) {
    const int row = i / J, j = i % J, t = t0 + row;
    const int o = row * JP + j;
    const float v = alpha * (red[0][o] + red[1][o] + red[2][o] + red[3][o]);
    if (t < a.T) {
      if (a.probe & 8) { if (v == 1234.5f) a.Z[i] = v; }
      else atomicAdd(a.Z + (long long)t * a.ldz + j, v);
    }
  }
  if (a.xe == nullptr) return;
  // last-arriver tail.  No RELEASE fence: an agent-scope release writes back the whole L2
  // (measured +36 us per call), and the Z atomics execute at the memory side already, so each
  // wave's drained vector memory counter orders them before the block counts in.  The last
  // arriver takes an agent-scope ACQUIRE (invalidate only) before it reads the sums.
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0), expcnt / lgkmcnt untouched (gfx9 encoding)
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    unsigned* cp = a.cnt + blockIdx.x;
    const unsigned prev = __hip_atomic_fetch_add(cp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int l = prev == gridDim.y - 1;
    if (l) {
      __hip_atomic_store(cp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // agent-scope ACQUIRE (invalidate only, no L2 writeback): the other blocks' Z adds
      // landed at the memory side, and nothing this CU cached before them may serve the
      // reads below (MI355X_MICROARCH.md, inter-workgroup visibility); the wait holds the
      // barrier until the invalidate has completed
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last = l;
  }
  __syncthreads();
  if (!last) return;
  T* xe = reinterpret_cast<T*>(a.xe);
  const int nch = a.KP / 8;
  for (int i = threadIdx.x; i < 64 * nch; i += 512) {
    const int row = i / nch, c = (i % nch) * 8, t = t0 + row;
    if (t >= a.T) continue;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = c + e < J ? __hip_atomic_load(a.Z + (long long)t * a.ldz + c + e, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                       : 0.f;
    store8(xe + (long long)t * a.ldxe + a.xk + c, v);
  }
}

// ------------------------------------------------------------------------------------------
// up3:  out[t, c] += alpha * sum_j S1[t, j] * S2(c, j)   (16-bit read-modify-write)
//   FWD (mode 6):  y  += s Z_seg B_seg^T   S2(c, j) = B[c][j];   optional RoPE on the result
//   !FWD (mode 5): dx += drop'(dZ A)       S2(c, j) = A[j][c];   dropout mask on the delta
// Block: 128 output columns of one segment x 4 waves x RT row tiles of 16.
// Swapped MFMA: A-operand = S2 rows (output columns via cmap), B-operand = S1^T (k = j), so the
// accumulator of n-tile n holds out^T[m = 4g + r][t = L] and column cmap(n, 4g + r) =
// 32 (n >> 1) + 8 g + 4 (n & 1) + r: lane (L, g) owns columns 32 i + 8 g + [0, 8) of row t0 + L
// for i = 0..3 -- four 16-byte vectors, each wave instruction covering 64 contiguous bytes of 16
// rows; RoPE's rotate_half partner (column ^ 64) is i ^ 2 in the same lane.
// ------------------------------------------------------------------------------------------
struct UpSeg {
  long long out_off[4];  // first output column of the segment
  long long s1_off[4];   // first S1 column
  long long s2_off[4];   // FWD: first B row; !FWD: first A column
  int ncols[4];
  int nseg;
};

struct UpArgs {
  void* out; long long ldo;
  const float* s1; long long ld1;
  const float* s2; long long ld2;
  int T, J;
  float alpha;
  Drop drop;
  UpSeg seg;
  const float* rope_cos; const float* rope_sin; const int* rope_pos;
  int rope_mask;
};

constexpr int kUpRT = 4;

__device__ __forceinline__ int up_cmap(int n, int L) {
  return 32 * (n >> 1) + 8 * (L >> 2) + 4 * (n & 1) + (L & 3);
}

template <typename T, bool FWD, bool DROP, int KJ>
__global__ void __launch_bounds__(256) up3_kernel(UpArgs a) {
  constexpr int NKS = KJ / 32, SP = KJ + 8;   // k-steps; LDS row stride (16-bit elements)
  __shared__ __attribute__((aligned(16))) T s2[128 * SP];
  const int seg = blockIdx.z;
  const int NC = a.seg.ncols[seg];
  const int c0 = blockIdx.x * 128;
  if (c0 >= NC) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, L = lane & 15, g = lane >> 4;
  const int J = a.J;
  // stage S2(c, j) for c in [c0, c0 + 128), j < KJ as 16-bit [c][j] (zeros beyond J / NC)
  if (FWD) {
    const float* B = a.s2 + a.seg.s2_off[seg] * a.ld2;
    for (int idx = threadIdx.x; idx < 128 * (KJ / 4); idx += 256) {
      const int c = idx / (KJ / 4), j = (idx % (KJ / 4)) * 4;
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c0 + c < NC && j < J) f = *reinterpret_cast<const float4*>(B + (long long)(c0 + c) * a.ld2 + j);
      *reinterpret_cast<uint2*>(s2 + c * SP + j) = pack4<T>(f.x, f.y, f.z, f.w);
    }
  } else {
    const float* A = a.s2 + a.seg.s2_off[seg];
    for (int idx = threadIdx.x; idx < 32 * KJ; idx += 256) {
      const int j = idx / 32, c = (idx % 32) * 4;
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
      if (j < J && c0 + c < NC) f = *reinterpret_cast<const float4*>(A + (long long)j * a.ld2 + c0 + c);
      s2[(c + 0) * SP + j] = from_f32<T>(f.x);
      s2[(c + 1) * SP + j] = from_f32<T>(f.y);
      s2[(c + 2) * SP + j] = from_f32<T>(f.z);
      s2[(c + 3) * SP + j] = from_f32<T>(f.w);
    }
  }
  __syncthreads();
  uint4 aop[8][NKS];
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      aop[n][ks] = *reinterpret_cast<const uint4*>(s2 + up_cmap(n, L) * SP + ks * 32 + g * 8);

  T* out = reinterpret_cast<T*>(a.out) + a.seg.out_off[seg];
  const float* s1 = a.s1 + a.seg.s1_off[seg];
  const bool rope = FWD && ((a.rope_mask >> seg) & 1);
  const int tw0 = (blockIdx.y * 4 + wid) * kUpRT * 16;

  // double-buffered per-row-tile operands: S1 row (B-operand), 4 output vectors
  uint4 bcur[NKS], bnxt[NKS], ycur[4], ynxt[4];
  const auto load_tile = [&](int t0, uint4 (&bop)[NKS], uint4 (&yv)[4]) {
    const int t = t0 + L;
    const bool tok = t < a.T;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int j = ks * 32 + g * 8;
      bop[ks] = ld_f32x8<T>(s1 + (long long)t * a.ld1 + j, tok && j < J);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + 32 * i + 8 * g;
      yv[i] = (tok && c < NC) ? *reinterpret_cast<const uint4*>(out + (long long)t * a.ldo + c)
                              : make_uint4(0, 0, 0, 0);
    }
  };
  if (tw0 >= a.T) return;
  load_tile(tw0, bcur, ycur);
#pragma unroll
  for (int rt = 0; rt < kUpRT; ++rt) {
    const int t0 = tw0 + rt * 16;
    if (t0 >= a.T) break;
    if (rt + 1 < kUpRT && t0 + 16 < a.T) load_tile(t0 + 16, bnxt, ynxt);
    f32x4 acc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[n] = Mfma<T>::run(aop[n][ks], bcur[ks], acc[n]);
    const int t = t0 + L;
    float y[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unpack8<T>(ycur[i], y[i]);
      const int c = c0 + 32 * i + 8 * g;
      const uint32_t keep = DROP ? dropout_keep8(a.drop.seed,
                                                 (unsigned long long)((long long)t * a.drop.ld + a.drop.col0 + a.seg.out_off[seg] + c),
                                                 a.drop.thresh)
                                 : 0xFFu;
      const float sc = DROP ? a.alpha * a.drop.scale : a.alpha;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = acc[2 * i + (e >> 2)][e & 3];
        y[i][e] += ((keep >> e) & 1u) ? sc * d : 0.f;
      }
    }
    if (rope && t < a.T) {
      // block-uniform: c0 is a head boundary, the block's 128 columns are one head
      const long long p = (long long)a.rope_pos[t] * 64;
      float cs[2][8], sn[2][8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float* cp = a.rope_cos + p + 32 * h + 8 * g;
        const float* sp = a.rope_sin + p + 32 * h + 8 * g;
        const float4 c_lo = *reinterpret_cast<const float4*>(cp), c_hi = *reinterpret_cast<const float4*>(cp + 4);
        const float4 s_lo = *reinterpret_cast<const float4*>(sp), s_hi = *reinterpret_cast<const float4*>(sp + 4);
        cs[h][0] = c_lo.x; cs[h][1] = c_lo.y; cs[h][2] = c_lo.z; cs[h][3] = c_lo.w;
        cs[h][4] = c_hi.x; cs[h][5] = c_hi.y; cs[h][6] = c_hi.z; cs[h][7] = c_hi.w;
        sn[h][0] = s_lo.x; sn[h][1] = s_lo.y; sn[h][2] = s_lo.z; sn[h][3] = s_lo.w;
        sn[h][4] = s_hi.x; sn[h][5] = s_hi.y; sn[h][6] = s_hi.z; sn[h][7] = s_hi.w;
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float lo = y[i][e], hi = y[i + 2][e];   // columns h and h + 64 of the head
          y[i][e] = lo * cs[i][e] - hi * sn[i][e];
          y[i + 2][e] = hi * cs[i][e] + lo * sn[i][e];
        }
    }
    if (t < a.T) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + 32 * i + 8 * g;
        if (c < NC) store8(out + (long long)t * a.ldo + c, y[i]);
      }
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bcur[ks] = bnxt[ks];
#pragma unroll
    for (int i = 0; i < 4; ++i) ycur[i] = ynxt[i];
  }
}

// ------------------------------------------------------------------------------------------
// dy3: per segment (dY columns [n_off, n_off + n_len), adapter columns [r_off, r_off + r)):
//   dZ[t, r_off + j] += alpha * sum_c dY[t, n_off + c] * B[b_off + c, j]
//   dB[b_off + c, j] += alpha * sum_t dY[t, n_off + c] * Z[t, r_off + j]
// Block (4 waves) = 256 columns (2 chunks of 128) x TW rows (64-row sub-tiles); the staged dY
// sub-tile [64][128] is read row-wise for dZ (wave w: rows 16w..16w+15) and transposed for dB
// (wave w: columns 32w..32w+31 of the chunk).  dZ partials are flushed per sub-tile, dB partials
// stay in registers for the whole row range and are flushed once.
// grid (ceil(maxlen / 256), ceil(T / TW), nseg)
// ------------------------------------------------------------------------------------------
struct DySeg {
  long long n_off[4], r_off[4], b_off[4];
  int n_len[4];
  int nseg;
};

struct DyArgs {
  const void* dy; long long ldy;
  const float* B; int r;        // B [*, r]
  const float* Z; long long ldz;
  float* dZ; long long lddz;
  float* dB;                    // [*, r]
  int T, TW;
  float alpha;
  DySeg seg;
  int probe;  // cost probes (0 in production): 16 dZ atomics, 32 dB atomics only when v == 1234.5
  // deterministic sums (slab_z != nullptr; det.h): dZ partials per (segment, row block, column
  // block) [TW][r], dB partials per (segment, column block, row block) [256][r]; the last
  // column block of a row block sums dZ, the last row block of a column block sums dB
  float* slab_z; float* slab_b;
  unsigned* cnt_z; unsigned* cnt_b;
};

constexpr int kDyCC = 2;

template <typename T>
__device__ __forceinline__ void dy_load(uint4 (&v)[4], const T* base, long long ld, int r0, int rmax,
                                        int c0, int cmax) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // unconditional from a clamped address, zeroed by a select: a guarded load here made hipcc
    // drain every load in flight at the branch join (rmax > r0, cmax >= 8)
    const int idx = threadIdx.x + i * 256;
    const int r = r0 + (idx >> 4), c = c0 + (idx & 15) * 8;
    const uint4 u = *reinterpret_cast<const uint4*>(base + (long long)min(r, rmax - 1) * ld +
                                                     min(c, cmax - 8));
    v[i] = (r < rmax && c < cmax) ? u : make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void dy_store(char* img, const uint4 (&v)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + i * 256;
    *reinterpret_cast<uint4*>(img + img_off_b(idx >> 4, idx & 15)) = v[i];
  }
}

template <typename T, int NJ>
__global__ void __launch_bounds__(256) dy3_kernel(DyArgs a) {
  __shared__ __attribute__((aligned(16))) char img[2][64 * 256];
  const int seg = blockIdx.z;
  const int NL = a.seg.n_len[seg];
  const int cb = blockIdx.x * 128 * kDyCC;
  const int tb = blockIdx.y * a.TW, te = min(a.T, tb + a.TW);
  if (cb >= NL || tb >= a.T) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, L = lane & 15, g = lane >> 4;
  const T* dy = reinterpret_cast<const T*>(a.dy) + a.seg.n_off[seg];
  const float* B = a.B + a.seg.b_off[seg] * a.r;
  const float* Z = a.Z + a.seg.r_off[seg];
  float* dZ = a.dZ + a.seg.r_off[seg];
  float* dB = a.dB + a.seg.b_off[seg] * a.r;
  const int nch = min(kDyCC, (NL - cb + 127) / 128);

  // dZ B-operand for every chunk: lane (L, g) <- B[cb + 128 cc + 32 i + 8 g + e][16 jt + L]
  uint4 bop[kDyCC][4][NJ];
#pragma unroll
  for (int cc = 0; cc < kDyCC; ++cc)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) {
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // unconditional (clamped column), zeroed after
          const int c = cb + cc * 128 + 32 * i + 8 * g + e;
          const float u = B[(long long)min(c, NL - 1) * a.r + jt * 16 + L];
          f[e] = c < NL ? u : 0.f;
        }
        bop[cc][i][jt] = pack8<T>(f);
      }
  f32x4 dbacc[kDyCC][2][NJ];
#pragma unroll
  for (int cc = 0; cc < kDyCC; ++cc)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) dbacc[cc][m][jt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsub = (te - tb + 63) / 64;
  const int nstage = nsub * nch;
  uint4 v[4];
  dy_load<T>(v, dy, a.ldy, tb, te, cb, NL);
  int buf = 0;
  f32x4 dzacc[NJ];
  uint4 zop[2][NJ];
  for (int s = 0; s < nstage; ++s, buf ^= 1) {
    const int ts = s / nch, cc = s % nch;
    const int t0 = tb + ts * 64, cbase = cb + cc * 128;
    dy_store(img[buf], v);
    __syncthreads();
    // dB B-operand: lane (L, g) <- Z[t0 + 32 ks + 8 g + e][16 jt + L], loaded every stage (the
    // chunks of a sub-tile reload the same L2-resident rows) and BEFORE the next stage's dY
    // prefetch, all unconditional from clamped rows: the wait for them is then a counted
    // vmcnt that leaves the prefetch in flight.  (Loaded after it behind `if (cc == 0)`, with
    // guarded loads, hipcc drained the prefetch with vmcnt(0) before the dB products.)
    float zf[2][NJ][8];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int t = t0 + 32 * ks + 8 * g + e;
          zf[ks][jt][e] = Z[(long long)min(t, te - 1) * a.ldz + jt * 16 + L];
        }
    {  // the last stage reloads itself (results unused): no branch around the prefetch
      const int s1 = min(s + 1, nstage - 1);
      const int ts1 = s1 / nch, cc1 = s1 % nch;
      dy_load<T>(v, dy, a.ldy, tb + ts1 * 64, te, cb + cc1 * 128, NL);
    }
    if (cc == 0) {
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) dzacc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const char* im = img[buf];
    // dZ: rows 16 wid + L, k = chunk columns
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 av = row_read_b(im, wid * 16 + L, i * 4 + g);
#pragma unroll
      for (int c2 = 0; c2 < kDyCC; ++c2)
        if (c2 == cc) {
#pragma unroll
          for (int jt = 0; jt < NJ; ++jt) dzacc[jt] = Mfma<T>::run(av, bop[c2][i][jt], dzacc[jt]);
        }
    }
    // dB: columns 32 wid + 16 m + (4 g + r), k = sub-tile rows
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) {
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = t0 + 32 * ks + 8 * g + e < te ? zf[ks][jt][e] : 0.f;
        zop[ks][jt] = pack8<T>(f);
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const uint4 tv = tr_read_img_b(im, ks * 32, wid * 32 + m * 16, lane);
#pragma unroll
        for (int c2 = 0; c2 < kDyCC; ++c2)
          if (c2 == cc) {
#pragma unroll
            for (int jt = 0; jt < NJ; ++jt) dbacc[c2][m][jt] = Mfma<T>::run(tv, zop[ks][jt], dbacc[c2][m][jt]);
          }
      }
    if (cc == nch - 1) {
      // flush this sub-tile's dZ rows: accumulator row 4 g + r, column 16 jt + L
      if (a.slab_z != nullptr) {
        float* sz = a.slab_z + (((long long)seg * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) *
                                   ((long long)a.TW * a.r);
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = t0 + wid * 16 + g * 4 + r;
            if (t < te) det::st_wt(sz + (long long)(t - tb) * a.r + jt * 16 + L, dzacc[jt][r]);
          }
      } else {
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = t0 + wid * 16 + g * 4 + r;
            if (t < te && (!(a.probe & 16) || dzacc[jt][r] == 1234.5f))
              atomicAdd(dZ + (long long)t * a.lddz + jt * 16 + L, a.alpha * dzacc[jt][r]);
          }
      }
    }
  }
  if (a.slab_z != nullptr) {
    // dB partials of this (segment, column block, row block), then the two last-arriver sums
    float* sb = a.slab_b + (((long long)seg * gridDim.x + blockIdx.x) * gridDim.y + blockIdx.y) *
                               (256LL * a.r);
#pragma unroll
    for (int cc = 0; cc < kDyCC; ++cc) {
      if (cc >= nch) break;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cl = cc * 128 + wid * 32 + m * 16 + g * 4 + r;
            if (cb + cl < NL) det::st_wt(sb + (long long)cl * a.r + jt * 16 + L, dbacc[cc][m][jt][r]);
          }
    }
    // split form (no counters): dy3_reduce_kernel sums the slabs in a second launch
    if (a.cnt_z == nullptr) return;
    __shared__ int lastf;
    const int ncb = (NL + 128 * kDyCC - 1) / (128 * kDyCC);  // column blocks of this segment
    const int J = NJ * 16;
    if (det::last_arriver(a.cnt_z + (long long)seg * gridDim.y + blockIdx.y, ncb, &lastf)) {
      // dZ rows [tb, te) of this segment: column blocks summed in order
      const float* base = a.slab_z + ((long long)seg * gridDim.y + blockIdx.y) * gridDim.x *
                                         ((long long)a.TW * a.r);
      for (int i = threadIdx.x; i < (te - tb) * (J / 2); i += 256) {
        const int tl = i / (J / 2), j = (i % (J / 2)) * 2;
        const float2 v = det::sum_pairs(base + (long long)tl * a.r + j, (long long)a.TW * a.r, ncb);
        float* o = dZ + (long long)(tb + tl) * a.lddz + j;
        o[0] = a.alpha * v.x;
        o[1] = a.alpha * v.y;
      }
    }
    if (det::last_arriver(a.cnt_b + (long long)seg * gridDim.x + blockIdx.x, gridDim.y, &lastf)) {
      // dB rows [cb, cb + 256) of this segment: row blocks summed in order, added to dB
      const float* base = a.slab_b + ((long long)seg * gridDim.x + blockIdx.x) * gridDim.y *
                                         (256LL * a.r);
      const int nc = min(256, NL - cb);
      for (int i = threadIdx.x; i < nc * (J / 2); i += 256) {
        const int cl = i / (J / 2), j = (i % (J / 2)) * 2;
        const float2 v = det::sum_pairs(base + (long long)cl * a.r + j, 256LL * a.r, gridDim.y);
        float* o = dB + (long long)(cb + cl) * a.r + j;
        o[0] += a.alpha * v.x;
        o[1] += a.alpha * v.y;
      }
    }
    return;
  }
#pragma unroll
  for (int cc = 0; cc < kDyCC; ++cc) {
    if (cc >= nch) break;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb + cc * 128 + wid * 32 + m * 16 + g * 4 + r;
          if (c < NL && (!(a.probe & 32) || dbacc[cc][m][jt][r] == 1234.5f))
            atomicAdd(dB + (long long)c * a.r + jt * 16 + L, a.alpha * dbacc[cc][m][jt][r]);
        }
      }
  }
}

// The deterministic dZ / dB sums of dy3 as their own whole-chip launch (split form): one thread
// per output pair, the partials of the column blocks (dZ) / row blocks (dB) added in block order
// with 16 loads in flight.  In the in-kernel form one last-arriving workgroup pulled each 128-400
// KB reduction through a single CU (latency-bound, profiles/r6_det).
// grid (ceil(max(T, max n_len) * r / 2 / 256), nseg, 2): z = 0 dZ, z = 1 dB
__device__ __forceinline__ float2 sum_pairs_plain(const float* base, long long stride, int n) {
  float2 v = make_float2(0.f, 0.f);
  for (int q0 = 0; q0 < n; q0 += 16) {
    float2 u[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = q0 + k < n ? q0 + k : n - 1;
      u[k] = *reinterpret_cast<const float2*>(base + q * stride);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (q0 + k < n) {
        v.x += u[k].x;
        v.y += u[k].y;
      }
  }
  return v;
}

__global__ void __launch_bounds__(256) dy3_reduce_kernel(DyArgs a, int gx_n, int gy_n) {
  const int seg = blockIdx.y;
  const int NL = a.seg.n_len[seg];
  const int hr = a.r / 2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int j = (int)(i % hr) * 2;
  if (blockIdx.z == 0) {
    const long long t = i / hr;
    if (t >= a.T) return;
    const int gy = (int)(t / a.TW), tl = (int)(t % a.TW);
    const int ncb = (NL + 128 * kDyCC - 1) / (128 * kDyCC);
    const float* base = a.slab_z + (((long long)seg * gy_n + gy) * gx_n) * ((long long)a.TW * a.r) +
                        (long long)tl * a.r + j;
    const float2 v = sum_pairs_plain(base, (long long)a.TW * a.r, ncb);
    float* o = a.dZ + a.seg.r_off[seg] + t * a.lddz + j;
    o[0] = a.alpha * v.x;
    o[1] = a.alpha * v.y;
  } else {
    const long long c = i / hr;
    if (c >= NL) return;
    const int gx = (int)(c / (128 * kDyCC)), cl = (int)(c % (128 * kDyCC));
    const float* base = a.slab_b + (((long long)seg * gx_n + gx) * gy_n) * (256LL * a.r) +
                        (long long)cl * a.r + j;
    const float2 v = sum_pairs_plain(base, 256LL * a.r, gy_n);
    float* o = a.dB + (a.seg.b_off[seg] + c) * a.r + j;
    o[0] += a.alpha * v.x;
    o[1] += a.alpha * v.y;
  }
}

// dxa3's deterministic dA sums as their own launch (split form, as dy3_reduce_kernel): one
// thread per (row j, column pair), the row blocks' partials [gx][gy][R][128] added in order.
// grid (ceil(R * K / 2 / 256))
__global__ void __launch_bounds__(256) dxa3_reduce_kernel(const float* __restrict__ slab,
                                                          float* __restrict__ dA, long long ldda,
                                                          int R, int K, int gy_n, float scale) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int hk = K / 2;
  if (i >= (long long)R * hk) return;
  const int j = (int)(i / hk), k = (int)(i % hk) * 2;
  const int gx = k / 128, kl = k % 128;
  const float2 v = sum_pairs_plain(slab + ((long long)gx * gy_n) * (128LL * R) +
                                       (long long)j * 128 + kl,
                                   128LL * R, gy_n);
  float* o = dA + (long long)j * ldda + k;
  o[0] += scale * v.x;
  o[1] += scale * v.y;
}

// down3's deterministic Z sums as their own launch (split form): one thread per (row, column
// pair), the K blocks' partials [tile][gy][64][J] added in order.  grid (ceil(T * J / 2 / 256))
__global__ void __launch_bounds__(256) down3_reduce_kernel(const float* __restrict__ slab,
                                                           float* __restrict__ Z, long long ldz,
                                                           int T, int J, int gy_n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int hj = J / 2;
  if (i >= (long long)T * hj) return;
  const int t = (int)(i / hj), j = (int)(i % hj) * 2;
  const int tile = t / 64, row = t % 64;
  const float2 v = sum_pairs_plain(slab + ((long long)tile * gy_n) * (64LL * J) +
                                       (long long)row * J + j,
                                   64LL * J, gy_n);
  *reinterpret_cast<float2*>(Z + (long long)t * ldz + j) = v;
}

// ------------------------------------------------------------------------------------------
// dxa3: ONE pass over the [T, K] activation rows for both x-side backward products
//   dA[j, k] += scale * sum_t dZ[t, j] * drop(x)[t, k]          (keep-scale folded into scale)
//   dx[t, k] += drop'(sum_j dZ[t, j] * A[j, k])                 (16-bit read-modify-write)
// Block (4 waves) = 128 columns of K x TW rows (64-row sub-tiles).  Per sub-tile the x tile is
// staged (dropout-masked) as a swizzled LDS image and dZ^T as a 16-bit LDS tile: dA MFMAs read
// x^T with ds_read_b64_tr_b16 (wave w: columns 32w..32w+31, accumulators live across the row
// range and land with one f32 atomic each at the end); wave w also updates the dx rows
// 16w..16w+15 of the sub-tile lane-locally (the up3 column map: 4 x 16-byte vectors per lane),
// its dx / dZ loads issued before the dA products so they land under them.
// grid (ceil(K / 128), ceil(T / TW)), block 256.
// ------------------------------------------------------------------------------------------
struct DxaArgs {
  const void* x; long long ldx;
  void* dx; long long lddx;
  const float* dZ;            // [T][R]
  const float* A;             // [R][lda]
  long long lda;
  float* dA;                  // [R][ldda]
  long long ldda;
  int T, K, R, TW;
  float da_scale, dx_scale;   // dA: keep-scale; dx: keep-scale (dZ already carries s)
  Drop drop;
  int probe;  // cost probe (0 in production): 64 dA atomics only when v == 1234.5
  // deterministic dA sum (slab != nullptr; det.h): partials per (column block, row block)
  // [R][128], the last row block of a column block adds their in-order sum into dA
  float* slab; unsigned* cnt;
  // flash-attention delta hand-off (DELTA instantiation; x = the attention output O, dx = dO
  // once updated, 128-column blocks = heads): delta[c0 / 128][t] = sum_c dO[t][c] O[t][c] over
  // the block, written here so the attention backward skips its delta pass.
  float* delta;
};

constexpr int kDxST = 72;     // dZ^T LDS row stride (16-bit): 144 B

template <typename T, bool DROP, int NJ, bool DELTA = false>
__global__ void __launch_bounds__(256) dxa3_kernel(DxaArgs a) {
  constexpr int J = NJ * 16, KJ = J > 32 ? 64 : 32, NKS = KJ / 32, SP = KJ + 8;
  __shared__ __attribute__((aligned(16))) char img[2][64 * 256];
  __shared__ __attribute__((aligned(16))) T st[2][J * kDxST];
  __shared__ __attribute__((aligned(16))) T s2[128 * SP];
  // the sub-tile's dropout keep-masks (one byte per 8 elements, [row][chunk]), hashed once in
  // store_stage for the dA image and re-read by the dx update of the same elements (it hashed
  // them a second time: the dropout hash, four 32-bit multiplies per element pair, was the
  // kernel's largest VALU cost)
  __shared__ uint8_t mk[DROP ? 2 : 1][DROP ? 64 * 16 : 1];
  const int c0 = blockIdx.x * 128;
  const int tb = blockIdx.y * a.TW, te = min(a.T, tb + a.TW);
  if (c0 >= a.K || tb >= a.T) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, L = lane & 15, g = lane >> 4;
  const T* x = reinterpret_cast<const T*>(a.x);
  T* dx = reinterpret_cast<T*>(a.dx);
  // A^T slice for the dx products: s2[c][j] = A[j][c0 + c] (zero beyond R / K).  Every load is
  // issued before the first LDS store (clamped addresses, zeroed by a select): a guarded load
  // per loop trip made hipcc wait for each in turn, KJ / 8 serial L2 round trips per block
  constexpr int NS2 = 32 * KJ / 256;
  float4 f2[NS2];
#pragma unroll
  for (int q = 0; q < NS2; ++q) {
    const int idx = threadIdx.x + q * 256, j = idx / 32, c = (idx % 32) * 4;
    const int jj = min(j, a.R - 1), cc = min(c0 + c, a.K - 4);
    f2[q] = *reinterpret_cast<const float4*>(a.A + (long long)jj * a.lda + cc);
  }
#pragma unroll
  for (int q = 0; q < NS2; ++q) {
    const int idx = threadIdx.x + q * 256, j = idx / 32, c = (idx % 32) * 4;
    const bool ok = j < a.R && c0 + c < a.K;
    const float4 f = ok ? f2[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    s2[(c + 0) * SP + j] = from_f32<T>(f.x);
    s2[(c + 1) * SP + j] = from_f32<T>(f.y);
    s2[(c + 2) * SP + j] = from_f32<T>(f.z);
    s2[(c + 3) * SP + j] = from_f32<T>(f.w);
  }
  f32x4 da[2][NJ];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int jt = 0; jt < NJ; ++jt) da[m][jt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging registers: x tile (4 x 16 B per thread) and dZ tile (J / 4 float4 per row)
  uint4 xv[4];
  float4 zv[(64 * J / 4 + 255) / 256];
  // every staging / row load is unconditional (clamped address) and out-of-range values are
  // zeroed by a select afterwards: with per-lane guarded loads hipcc could not count the loads
  // in flight across the branches and drained the whole prefetch with vmcnt(0)
  const auto load_stage = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + i * 256;
      const int r = t0 + (idx >> 4), c = c0 + (idx & 15) * 8;
      const uint4 u = *reinterpret_cast<const uint4*>(x + (long long)min(r, te - 1) * a.ldx +
                                                       min(c, a.K - 8));
      xv[i] = (r < te && c < a.K) ? u : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < (64 * J / 4 + 255) / 256; ++i) {
      const int idx = threadIdx.x + i * 256;
      const int r = idx / (J / 4), j = (idx % (J / 4)) * 4;
      const float4 u = *reinterpret_cast<const float4*>(a.dZ + (long long)min(t0 + r, te - 1) * a.R + j);
      zv[i] = (r < 64 && t0 + r < te) ? u : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const auto store_stage = [&](int t0, int b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + i * 256;
      const int row = idx >> 4, ch = idx & 15;
      uint4 u = xv[i];
      if (DROP) {
        const uint32_t keep = dropout_keep8(
            a.drop.seed,
            (unsigned long long)((long long)(t0 + row) * a.drop.ld + a.drop.col0 + c0 + ch * 8),
            a.drop.thresh);
        u = mask8(u, keep);
        mk[b][row * 16 + ch] = static_cast<uint8_t>(keep);
      }
      *reinterpret_cast<uint4*>(img[b] + img_off(row, ch)) = u;
    }
#pragma unroll
    for (int i = 0; i < (64 * J / 4 + 255) / 256; ++i) {
      const int idx = threadIdx.x + i * 256;
      const int r = idx / (J / 4), j = (idx % (J / 4)) * 4;
      if (r < 64) {
        st[b][(j + 0) * kDxST + r] = from_f32<T>(zv[i].x);
        st[b][(j + 1) * kDxST + r] = from_f32<T>(zv[i].y);
        st[b][(j + 2) * kDxST + r] = from_f32<T>(zv[i].z);
        st[b][(j + 3) * kDxST + r] = from_f32<T>(zv[i].w);
      }
    }
  };
  // dx operands of a wave's 16 rows (dZ row, the dx row, O for the delta dot), loaded one
  // sub-tile ahead: loaded right before use they left one HBM round trip exposed per 64 rows
  // (dZ rows as f32 pairs, loaded unconditionally from clamped addresses and zeroed / packed
  // at use: the guarded form made hipcc wait for each pair right after issuing it)
  float4 nbf[NKS][2];
  uint4 ndv[4];
  uint4 nov[DELTA ? 4 : 1];  // O (un-dropped x) in the dx lane layout, for the delta dot
  const auto load_rows = [&](int t0) {
    const int t = t0 + wid * 16 + L;
    const bool tok = t < te;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int j = min(ks * 32 + g * 8, a.R - 8);
      const float* zp = a.dZ + (long long)min(t, te - 1) * a.R + j;
      nbf[ks][0] = *reinterpret_cast<const float4*>(zp);
      nbf[ks][1] = *reinterpret_cast<const float4*>(zp + 4);
    }
    const long long tc = min(t, te - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + 32 * i + 8 * g;
      const uint4 u = *reinterpret_cast<const uint4*>(dx + tc * a.lddx + min(c, a.K - 8));
      ndv[i] = (tok && c < a.K) ? u : make_uint4(0, 0, 0, 0);
    }
    if constexpr (DELTA) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + 32 * i + 8 * g;
        const uint4 u = *reinterpret_cast<const uint4*>(x + tc * a.ldx + min(c, a.K - 8));
        nov[i] = (tok && c < a.K) ? u : make_uint4(0, 0, 0, 0);
      }
    }
  };
  load_stage(tb);
  load_rows(tb);
  int buf = 0;
  for (int t0 = tb; t0 < te; t0 += 64, buf ^= 1) {
    store_stage(t0, buf);
    __syncthreads();
    // unconditional (the last trip re-reads clamped rows it never stores): a branch around
    // the loads made hipcc drain the prefetch with vmcnt(0) at the join
    load_stage(t0 + 64);
    const int t = t0 + wid * 16 + L;
    const bool tok = t < te;
    uint4 bop[NKS], dv[4], ov[DELTA ? 4 : 1];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const float4 u = nbf[ks][0], v = nbf[ks][1];
      bop[ks] = (tok && ks * 32 + g * 8 < a.R)
                    ? make_uint4(pk2<T>(u.x, u.y), pk2<T>(u.z, u.w), pk2<T>(v.x, v.y), pk2<T>(v.z, v.w))
                    : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) dv[i] = ndv[i];
    if constexpr (DELTA) {
#pragma unroll
      for (int i = 0; i < 4; ++i) ov[i] = nov[i];
    }
    load_rows(t0 + 64);
    // dA: D[j][k] += dZ^T[j][t] x[t][k] over the sub-tile's 64 rows
    const char* im = img[buf];
    const T* sz = st[buf];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 xt[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) xt[m] = tr_read_img(im, ks * 32, wid * 32 + m * 16, lane);
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt) {
        const uint4 zt = *reinterpret_cast<const uint4*>(sz + (jt * 16 + L) * kDxST + ks * 32 + g * 8);
#pragma unroll
        for (int m = 0; m < 2; ++m) da[m][jt] = Mfma<T>::run(zt, xt[m], da[m][jt]);
      }
    }
    // dx += drop'(dZ A) for rows t (lane-local, column map as in up3)
    f32x4 acc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int n = 0; n < 8; ++n)  // A^T operand re-read from LDS (keeps 2 waves per SIMD)
        acc[n] = Mfma<T>::run(*reinterpret_cast<const uint4*>(s2 + up_cmap(n, L) * SP + ks * 32 + g * 8),
                              bop[ks], acc[n]);
    float dot = 0.f;
    if (tok) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + 32 * i + 8 * g;
        if (c >= a.K) continue;
        float y[8];
        unpack8<T>(dv[i], y);
        // row t = t0 + 16 wid + L, chunk (c - c0) / 8 = 4 i + g: the mask store_stage hashed
        // (hashing these masks a second time here measured 35.9 / 32.5 against 34.9 / 31.4 us
        // per q|k|v / o call, gpurun r5_49)
        const uint32_t keep = DROP ? static_cast<uint32_t>(mk[buf][(wid * 16 + L) * 16 + 4 * i + g])
                                   : 0xFFu;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = acc[2 * i + (e >> 2)][e & 3];
          y[e] += ((keep >> e) & 1u) ? a.dx_scale * d : 0.f;
        }
        if constexpr (DELTA) {  // the dot of the 16-bit values the attention backward reads
          float o[8];
          unpack8<T>(ov[i], o);
#pragma unroll
          for (int e = 0; e < 8; ++e) dot = fmaf(to_f32(from_f32<T>(y[e])), o[e], dot);
        }
        store8(dx + (long long)t * a.lddx + c, y);
      }
    }
    if constexpr (DELTA) {
      // lanes L, L + 16, L + 32, L + 48 hold the four 32-column quarters of row t's head
      dot += __shfl_xor(dot, 16);
      dot += __shfl_xor(dot, 32);
      if (tok && g == 0) a.delta[(long long)(c0 >> 7) * a.T + t] = dot;
    }
  }
  // dA flush: accumulator (row j = 16 jt + 4 g + r, column k = c0 + 32 wid + 16 m + L)
  if (a.slab != nullptr) {
    float* sp = a.slab + ((long long)blockIdx.x * gridDim.y + blockIdx.y) * (128LL * a.R);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kl = wid * 32 + m * 16 + L, j = jt * 16 + g * 4 + r;
          if (c0 + kl < a.K && j < a.R) det::st_wt(sp + (long long)j * 128 + kl, da[m][jt][r]);
        }
    if (a.cnt == nullptr) return;  // split form: dxa3_reduce_kernel sums the slabs
    __shared__ int lastf;
    if (!det::last_arriver(a.cnt + blockIdx.x, gridDim.y, &lastf)) return;
    const float* base = a.slab + (long long)blockIdx.x * gridDim.y * (128LL * a.R);
    for (int i = threadIdx.x; i < a.R * 64; i += 256) {  // pairs of columns
      const int j = i / 64, kl = (i % 64) * 2;
      if (c0 + kl >= a.K) continue;
      const float2 v = det::sum_pairs(base + (long long)j * 128 + kl, 128LL * a.R, gridDim.y);
      float* o = a.dA + (long long)j * a.ldda + c0 + kl;
      o[0] += a.da_scale * v.x;
      if (c0 + kl + 1 < a.K) o[1] += a.da_scale * v.y;
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = c0 + wid * 32 + m * 16 + L, j = jt * 16 + g * 4 + r;
        if (k < a.K && j < a.R && (!(a.probe & 64) || da[m][jt][r] == 1234.5f))
          atomicAdd(a.dA + (long long)j * a.ldda + k, a.da_scale * da[m][jt][r]);
      }
}

// ------------------------------------------------------------------------------------------
// K-extension ("fold") of the forward UP into the frozen-weight GEMM:
//   y = [x | Z | 0] [W | s B_bd | 0]^T   with the adapter tail of 64 extra K columns.
// z_tail writes the (16-bit) Z tail of the activation operand next to x (which its producer --
// RMSNorm / flash attention -- already wrote into the first K columns); w_tail refreshes the
// weight tail s * B of every segment after an optimizer step (block-diagonal over segments:
// rows of segment i use tail columns r_off_i .. r_off_i + r).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) z_tail_kernel(const float* __restrict__ Z, int R,
                                                     T* __restrict__ xe, long long ldx, int K,
                                                     int KP, int T_) {
  const int nch = KP / 8;
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= static_cast<long long>(T_) * nch) return;
  const int t = static_cast<int>(i / nch), c = static_cast<int>(i % nch) * 8;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = c + e < R ? Z[static_cast<long long>(t) * R + c + e] : 0.f;
  store8(xe + static_cast<long long>(t) * ldx + K + c, v);
}

struct TailSeg {
  long long n_off[4], b_off[4];
  int n_len[4], r_off[4];
  int nseg;
};

template <typename T>
__global__ void __launch_bounds__(256) w_tail_kernel(T* __restrict__ w, long long ldw, int K,
                                                     const float* __restrict__ B, int r,
                                                     TailSeg sg, float scale) {
  const int seg = blockIdx.y;
  const int nch = r / 8;
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= static_cast<long long>(sg.n_len[seg]) * nch) return;
  const int n = static_cast<int>(i / nch), c = static_cast<int>(i % nch) * 8;
  float v[8];
  load8(B + (sg.b_off[seg] + n) * r + c, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= scale;
  store8(w + (sg.n_off[seg] + n) * ldw + K + sg.r_off[seg] + c, v);
}

// All folded linears of a model in ONE launch after an optimizer publish (64 single-linear
// launches of w_tail_kernel cost ~0.3 ms per Llama-2-7B step, almost all launch overhead: a
// linear's tail is only N x 16 16-bit values per segment).  desc: per linear 24 int64 =
// {w, ldw, B, K, r, nseg, float bits of scale, dtype, n_off[4], n_len[4], r_off[4], b_off[4]};
// blockIdx.y = linear * 4 + segment.
template <typename T>
__global__ void __launch_bounds__(256) w_tail_batch_kernel(const long long* __restrict__ desc) {
  const long long* d = desc + (blockIdx.y >> 2) * 24;
  const int seg = blockIdx.y & 3;
  if (seg >= static_cast<int>(d[5])) return;
  const int r = static_cast<int>(d[4]), K = static_cast<int>(d[3]);
  const int nch = r / 8;
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const long long n_len = d[12 + seg];
  if (i >= n_len * nch) return;
  const long long n = i / nch;
  const int c = static_cast<int>(i % nch) * 8;
  const float scale = __builtin_bit_cast(float, static_cast<unsigned>(d[6]));
  const float* B = reinterpret_cast<const float*>(d[2]);
  T* w = reinterpret_cast<T*>(d[0]);
  float v[8];
  load8(B + (d[20 + seg] + n) * r + c, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= scale;
  store8(w + (d[8 + seg] + n) * d[1] + K + d[16 + seg] + c, v);
}

}  // namespace lv3
}  // namespace lumen

using namespace lumen;

// desc: n linears x 24 int64 on the device (see w_tail_batch_kernel), all of one 16-bit dtype;
// max_chunks = the largest n_len * r / 8 over all segments
extern "C" hipError_t lumen_lora3_w_tail_batch(int dtype, const long long* desc, int n,
                                               long long max_chunks, hipStream_t st) {
  if (n <= 0 || max_chunks <= 0) return hipSuccess;
  if (n > 16383) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>((max_chunks + 255) / 256), 4 * n), block(256);
  if (dtype == kBF16) hipLaunchKernelGGL(lv3::w_tail_batch_kernel<bf16>, grid, block, 0, st, desc);
  else if (dtype == kF16) hipLaunchKernelGGL(lv3::w_tail_batch_kernel<fp16>, grid, block, 0, st, desc);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

#include <cstdlib>
static int lv3_probe() {
  static int v = [] { const char* e = std::getenv("LUMEN_LV3_PROBE"); return e ? std::atoi(e) : 0; }();
  return v;
}

// Z[t, j] += alpha * sum_k drop(x)[t, k] A[j, k]; R = 16 * nj (nj 1..4); K, ldx multiples of 8
extern "C" hipError_t lumen_lora3_down(int dtype, const void* x, long long ldx, const float* A,
                                       long long lda, float* Z, long long ldz, int T, int K, int R,
                                       float alpha, unsigned long long seed, unsigned int thresh,
                                       float drop_scale, long long drop_ld, long long drop_col0,
                                       void* xe, long long ldxe, int xk, int KP, unsigned* cnt,
                                       float* slab, hipStream_t st) {
  if (T <= 0 || K <= 0 || R < 16 || R > 64 || (R & 15) || (K & 7) || (ldx & 7) || (lda & 3))
    return hipErrorInvalidValue;
  if (xe != nullptr && (cnt == nullptr || (KP & 7) || KP < R || (ldxe & 7) || (xk & 7)))
    return hipErrorInvalidValue;
  // slab with cnt: in-kernel last-arriver sums; slab without cnt (and no fold tail): the split
  // form, down3_reduce_kernel after
  if (slab != nullptr && ((ldz & 1) || (cnt == nullptr && xe != nullptr)))
    return hipErrorInvalidValue;
  lv3::DownArgs a{x, ldx, A, lda, Z, ldz, T, K, alpha,
                  {static_cast<unsigned>(seed) ^ static_cast<unsigned>(seed >> 32), thresh, drop_scale,
                   drop_ld, drop_col0}, lv3_probe(), xe, ldxe, xk, KP, cnt, slab};
  const dim3 grid((T + 63) / 64, (K + 1023) / 1024), block(512);
  const bool drop = thresh != 0;
#define LV3_DOWN(TT, NJ)                                                                           \
  do {                                                                                           \
    if (drop) hipLaunchKernelGGL((lv3::down3_kernel<TT, true, NJ>), grid, block, 0, st, a);     \
    else hipLaunchKernelGGL((lv3::down3_kernel<TT, false, NJ>), grid, block, 0, st, a);         \
  } while (0)
#define LV3_DOWN_NJ(TT)                                                                            \
  switch (R / 16) {                                                                              \
    case 1: LV3_DOWN(TT, 1); break;                                                              \
    case 2: LV3_DOWN(TT, 2); break;                                                              \
    case 3: LV3_DOWN(TT, 3); break;                                                              \
    default: LV3_DOWN(TT, 4); break;                                                             \
  }
  if (dtype == kBF16) { LV3_DOWN_NJ(bf16) }
  else if (dtype == kF16) { LV3_DOWN_NJ(fp16) }
  else return hipErrorInvalidValue;
#undef LV3_DOWN_NJ
#undef LV3_DOWN
  if (slab != nullptr && cnt == nullptr) {
    const long long n = (long long)T * (R / 2);
    hipLaunchKernelGGL(lv3::down3_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       st, (const float*)slab, Z, ldz, T, R, (int)grid.y);
  }
  return hipGetLastError();
}

// fwd != 0: out[t, out_off + c] += alpha * sum_j s1[t, s1_off + j] * s2[s2_off + c][j]  (+RoPE)
// fwd == 0: out[t, out_off + c] += drop(alpha * sum_j s1[t, s1_off + j] * s2[j][s2_off + c])
// J <= 64; segment widths, out_off, ldo multiples of 8; RoPE segments start on 128-col heads
extern "C" hipError_t lumen_lora3_up(int dtype, int fwd, void* out, long long ldo, const float* s1,
                                     long long ld1, const float* s2, long long ld2, int T, int J,
                                     float alpha, unsigned long long seed, unsigned int thresh,
                                     float drop_scale, long long drop_ld, long long drop_col0,
                                     int nseg, const long long* out_off, const long long* s1_off,
                                     const long long* s2_off, const int* ncols,
                                     const float* rope_cos, const float* rope_sin,
                                     const int* rope_pos, int rope_mask, hipStream_t st) {
  if (T <= 0 || J < 1 || J > 64 || nseg < 1 || nseg > 4 || (ldo & 7) || (ld1 & 3) || (ld2 & 3))
    return hipErrorInvalidValue;
  lv3::UpArgs a;
  a.out = out; a.ldo = ldo; a.s1 = s1; a.ld1 = ld1; a.s2 = s2; a.ld2 = ld2; a.T = T; a.J = J;
  a.alpha = alpha;
  a.drop = {static_cast<unsigned>(seed) ^ static_cast<unsigned>(seed >> 32), thresh, drop_scale,
            drop_ld, drop_col0};
  a.seg.nseg = nseg;
  int maxc = 0;
  for (int i = 0; i < 4; ++i) {
    const bool v = i < nseg;
    a.seg.out_off[i] = v ? out_off[i] : 0; a.seg.s1_off[i] = v ? s1_off[i] : 0;
    a.seg.s2_off[i] = v ? s2_off[i] : 0; a.seg.ncols[i] = v ? ncols[i] : 0;
    if (v && ((ncols[i] & 7) || (out_off[i] & 7) || (s1_off[i] & 3))) return hipErrorInvalidValue;
    if (v && ncols[i] > maxc) maxc = ncols[i];
  }
  a.rope_cos = rope_cos; a.rope_sin = rope_sin; a.rope_pos = rope_pos;
  a.rope_mask = (fwd && rope_cos && rope_sin && rope_pos) ? rope_mask : 0;
  for (int i = 0; i < nseg; ++i)
    if (((a.rope_mask >> i) & 1) && ((out_off[i] & 127) || (ncols[i] & 127))) return hipErrorInvalidValue;
  if (maxc == 0) return hipSuccess;
  const dim3 grid((maxc + 127) / 128, (T + 64 * lv3::kUpRT - 1) / (64 * lv3::kUpRT), nseg), block(256);
  const bool drop = !fwd && thresh != 0;
#define LV3_UP(TT, KJ)                                                                             \
  do {                                                                                           \
    if (fwd) hipLaunchKernelGGL((lv3::up3_kernel<TT, true, false, KJ>), grid, block, 0, st, a);   \
    else if (drop) hipLaunchKernelGGL((lv3::up3_kernel<TT, false, true, KJ>), grid, block, 0, st, a); \
    else hipLaunchKernelGGL((lv3::up3_kernel<TT, false, false, KJ>), grid, block, 0, st, a);     \
  } while (0)
  if (dtype == kBF16) { if (J <= 32) LV3_UP(bf16, 32); else LV3_UP(bf16, 64); }
  else if (dtype == kF16) { if (J <= 32) LV3_UP(fp16, 32); else LV3_UP(fp16, 64); }
  else return hipErrorInvalidValue;
#undef LV3_UP
  return hipGetLastError();
}

// fused dZ / dB over one pass of dY (see dy3_kernel); r in {16, 32, 64}; tw multiple of 64
extern "C" hipError_t lumen_lora3_dy(int dtype, const void* dy, long long ldy, const float* B, int r,
                                     const float* Z, long long ldz, float* dZ, long long lddz,
                                     float* dB, int T, int tw, float alpha, int nseg,
                                     const long long* n_off, const long long* r_off,
                                     const long long* b_off, const int* n_len, float* slab_z,
                                     float* slab_b, unsigned* cnt_z, unsigned* cnt_b,
                                     hipStream_t st) {
  if (T <= 0 || nseg < 1 || nseg > 4 || (r != 16 && r != 32 && r != 64) || tw < 64 || (tw & 63) ||
      (ldy & 7))
    return hipErrorInvalidValue;
  lv3::DyArgs a;
  a.probe = lv3_probe();
  a.dy = dy; a.ldy = ldy; a.B = B; a.r = r; a.Z = Z; a.ldz = ldz; a.dZ = dZ; a.lddz = lddz;
  a.dB = dB; a.T = T; a.TW = tw; a.alpha = alpha;
  a.slab_z = slab_z; a.slab_b = slab_b; a.cnt_z = cnt_z; a.cnt_b = cnt_b;
  // deterministic sums: slabs with counters = in-kernel last-arriver sums; slabs without
  // counters = the split form (dy3_reduce_kernel launched after dy3)
  if (slab_z != nullptr && (slab_b == nullptr || (cnt_z == nullptr) != (cnt_b == nullptr) ||
                            (lddz & 1)))
    return hipErrorInvalidValue;
  a.seg.nseg = nseg;
  int maxl = 0;
  for (int i = 0; i < 4; ++i) {
    const bool v = i < nseg;
    a.seg.n_off[i] = v ? n_off[i] : 0; a.seg.r_off[i] = v ? r_off[i] : 0;
    a.seg.b_off[i] = v ? b_off[i] : 0; a.seg.n_len[i] = v ? n_len[i] : 0;
    if (v && ((n_len[i] & 7) || (n_off[i] & 7))) return hipErrorInvalidValue;
    if (v && n_len[i] > maxl) maxl = n_len[i];
  }
  if (maxl == 0) return hipSuccess;
  const dim3 grid((maxl + 128 * lv3::kDyCC - 1) / (128 * lv3::kDyCC), (T + tw - 1) / tw, nseg), block(256);
#define LV3_DY(TT)                                                                                 \
  switch (r) {                                                                                   \
    case 16: hipLaunchKernelGGL((lv3::dy3_kernel<TT, 1>), grid, block, 0, st, a); break;          \
    case 32: hipLaunchKernelGGL((lv3::dy3_kernel<TT, 2>), grid, block, 0, st, a); break;          \
    default: hipLaunchKernelGGL((lv3::dy3_kernel<TT, 4>), grid, block, 0, st, a); break;          \
  }
  if (dtype == kBF16) { LV3_DY(bf16) }
  else if (dtype == kF16) { LV3_DY(fp16) }
  else return hipErrorInvalidValue;
#undef LV3_DY
  if (slab_z != nullptr && cnt_z == nullptr) {
    const long long n = (long long)(T > maxl ? T : maxl) * (r / 2);
    const dim3 rgrid((unsigned)((n + 255) / 256), nseg, 2);
    hipLaunchKernelGGL(lv3::dy3_reduce_kernel, rgrid, dim3(256), 0, st, a, (int)grid.x,
                       (int)grid.y);
  }
  return hipGetLastError();
}

// xe[t, K + c] = c < R ? Z[t, c] : 0 for c < KP (16-bit xe, row stride ldx)
extern "C" hipError_t lumen_lora3_z_tail(int dtype, const float* Z, int R, void* xe, long long ldx,
                                         int K, int KP, int T, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  if ((KP & 7) || R > KP || (ldx & 7) || (K & 7)) return hipErrorInvalidValue;
  const long long n = static_cast<long long>(T) * (KP / 8);
  const dim3 grid(static_cast<unsigned>((n + 255) / 256)), block(256);
  if (dtype == kBF16) hipLaunchKernelGGL(lv3::z_tail_kernel<bf16>, grid, block, 0, st, Z, R, (bf16*)xe, ldx, K, KP, T);
  else if (dtype == kF16) hipLaunchKernelGGL(lv3::z_tail_kernel<fp16>, grid, block, 0, st, Z, R, (fp16*)xe, ldx, K, KP, T);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// w[n_off + n, K + r_off + j] = scale * B[(b_off + n) * r + j] per segment (n < n_len, j < r)
extern "C" hipError_t lumen_lora3_w_tail(int dtype, void* w, long long ldw, int K, const float* B,
                                         int r, int nseg, const long long* n_off,
                                         const long long* b_off, const int* n_len,
                                         const int* r_off, float scale, hipStream_t st) {
  if (nseg < 1 || nseg > 4 || (r & 7) || (ldw & 7) || (K & 7)) return hipErrorInvalidValue;
  lv3::TailSeg sg;
  sg.nseg = nseg;
  int maxn = 0;
  for (int i = 0; i < 4; ++i) {
    const bool v = i < nseg;
    sg.n_off[i] = v ? n_off[i] : 0; sg.b_off[i] = v ? b_off[i] : 0;
    sg.n_len[i] = v ? n_len[i] : 0; sg.r_off[i] = v ? r_off[i] : 0;
    if (v && (r_off[i] & 7)) return hipErrorInvalidValue;
    if (v && n_len[i] > maxn) maxn = n_len[i];
  }
  if (maxn == 0) return hipSuccess;
  const long long n = static_cast<long long>(maxn) * (r / 8);
  const dim3 grid(static_cast<unsigned>((n + 255) / 256), nseg), block(256);
  if (dtype == kBF16) hipLaunchKernelGGL(lv3::w_tail_kernel<bf16>, grid, block, 0, st, (bf16*)w, ldw, K, B, r, sg, scale);
  else if (dtype == kF16) hipLaunchKernelGGL(lv3::w_tail_kernel<fp16>, grid, block, 0, st, (fp16*)w, ldw, K, B, r, sg, scale);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// fused x-side backward: dA += scale * dZ^T drop(x) and dx += drop'(dZ A) in one pass over the
// [T, K] rows (see dxa3_kernel); R = 16 * nj (nj 1..4), K, ldx, lddx multiples of 8
extern "C" hipError_t lumen_lora3_dxa(int dtype, const void* x, long long ldx, void* dx,
                                      long long lddx, const float* dZ, const float* A,
                                      long long lda, float* dA, long long ldda, int T, int K,
                                      int R, int tw, unsigned long long seed, unsigned int thresh,
                                      float drop_scale, long long drop_ld, long long drop_col0,
                                      float* delta, float* slab, unsigned* cnt, hipStream_t st) {
  if (T <= 0 || K <= 0 || R < 16 || R > 64 || (R & 15) || (K & 7) || (ldx & 7) || (lddx & 7) ||
      (lda & 3) || tw < 64 || (tw & 63))
    return hipErrorInvalidValue;
  if (delta != nullptr && ((K & 127) || R != 16)) return hipErrorInvalidValue;
  lv3::DxaArgs a;
  a.probe = lv3_probe();
  a.x = x; a.ldx = ldx; a.dx = dx; a.lddx = lddx; a.dZ = dZ; a.A = A; a.lda = lda; a.dA = dA;
  a.ldda = ldda; a.T = T; a.K = K; a.R = R; a.TW = tw; a.delta = delta;
  a.slab = slab; a.cnt = cnt;
  // slab with cnt: in-kernel last-arriver sums; slab without cnt: dxa3_reduce_kernel after
  if (slab != nullptr && (ldda & 1)) return hipErrorInvalidValue;
  const bool drop = thresh != 0;
  a.da_scale = drop ? drop_scale : 1.f;
  a.dx_scale = drop ? drop_scale : 1.f;
  a.drop = {static_cast<unsigned>(seed) ^ static_cast<unsigned>(seed >> 32), thresh, drop_scale,
            drop_ld, drop_col0};
  const dim3 grid((K + 127) / 128, (T + tw - 1) / tw), block(256);
#define LV3_DXA(TT, NJ)                                                                            \
  do {                                                                                           \
    if (drop) hipLaunchKernelGGL((lv3::dxa3_kernel<TT, true, NJ>), grid, block, 0, st, a);      \
    else hipLaunchKernelGGL((lv3::dxa3_kernel<TT, false, NJ>), grid, block, 0, st, a);          \
  } while (0)
#define LV3_DXA_NJ(TT)                                                                             \
  switch (R / 16) {                                                                              \
    case 1: LV3_DXA(TT, 1); break;                                                               \
    case 2: LV3_DXA(TT, 2); break;                                                               \
    case 3: LV3_DXA(TT, 3); break;                                                               \
    default: LV3_DXA(TT, 4); break;                                                              \
  }
  if (delta != nullptr) {  // o_proj (R = 16) with the attention delta hand-off
#define LV3_DXA_D(TT)                                                                              \
  do {                                                                                           \
    if (drop) hipLaunchKernelGGL((lv3::dxa3_kernel<TT, true, 1, true>), grid, block, 0, st, a);  \
    else hipLaunchKernelGGL((lv3::dxa3_kernel<TT, false, 1, true>), grid, block, 0, st, a);      \
  } while (0)
    if (dtype == kBF16) LV3_DXA_D(bf16);
    else if (dtype == kF16) LV3_DXA_D(fp16);
    else return hipErrorInvalidValue;
#undef LV3_DXA_D
  } else if (dtype == kBF16) { LV3_DXA_NJ(bf16) }
  else if (dtype == kF16) { LV3_DXA_NJ(fp16) }
  else return hipErrorInvalidValue;
  if (slab != nullptr && cnt == nullptr) {
    const long long n = (long long)R * (K / 2);
    hipLaunchKernelGGL(lv3::dxa3_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       st, (const float*)slab, dA, ldda, R, K, (int)grid.y, a.da_scale);
  }
#undef LV3_DXA_NJ
#undef LV3_DXA
  return hipGetLastError();
}
