// LoRA adapter products on the bf16/fp16 matrix cores (v_mfma_f32_16x16x32), gfx950.
//
// Reference behaviour: PEFT LoraLayer under fp16 autocast (training/train_baseline.py:131-141,
// r=16, alpha=32, dropout 0.05 on q/k/v/o): the adapter matmuls run in 16-bit with f32
// accumulation and f32 adapter parameters.  These kernels do the same -- the big activation
// operand streams through a swizzled LDS image, the small adapter-side operand is converted to
// 16-bit while staging -- and replace the exact-f32 MFMA kernel (lora.hip) for the four
// "reduction" products, whose f32-MFMA compute (~1.6 GFLOP each per q|k|v layer at 157 TF/s)
// made them compute-bound.  Two kernel shapes:
//
//   DOWN   out[t, j] += a * sum_k big[t, k] * small(j, k)       reduce over the feature axis
//          mode 1:  Z  = drop(x) A^T        big = x,  small = A  [R][K]   (k-major)
//          mode 2:  dZ = s dY_seg B_seg     big = dY, small = B  [N][r]   (n-major, transposed)
//   WGRAD  out[m, j] += a * sum_t big[t, m] * small[t, j]       reduce over tokens
//          mode 3:  dA = dZ^T drop(x)       big = x,  small = dZ, output [R][K]   (SWAP)
//          mode 4:  dB = s dY_seg^T Z_seg   big = dY, small = Z,  output [N][r]
//
// Both stage the big operand as [64 rows][128 cols] images (dropout applied in registers on the
// way in, so the backward regenerates the forward's mask from the same hash) and the small one
// as a padded bf16 LDS tile; each block owns a 128-wide slice of the non-reduced axis and a
// split of the reduced one, and lands its partial sums with 64-byte-coalesced f32 atomics.
#include "tile128.h"

namespace lumen {
namespace lv2 {

using namespace tile;

struct Drop {
  unsigned int seed, thresh;
  float scale;
  long long ld;   // logical row length of the dropout index (t * ld + feature)
};

struct Seg4 {
  long long big_off[4];    // element offset of the segment's first column in `big`
  long long small_off[4];  // element offset into `small`
  long long out_off[4];    // element offset into `out`
  int ncols[4];            // DOWN: reduced length (K / n_len); WGRAD: segment width M
  int nseg;
};

struct Args {
  const void* big;
  long long ldb;
  const float* small;
  long long lds;
  void* out;               // f32 (DOWN / WGRAD) or 16-bit (UP)
  long long cs0, cs1;      // DOWN: out[t*cs0 + j*cs1]; WGRAD: out[m*cs0 + j*cs1]; UP: row stride cs0
  float alpha;
  int T;                   // tokens
  int J;                   // small-operand width (R or r), multiple of 16, <= 64
  int split;               // reduction splits (grid.y)
  long long drop_col0;     // dropout feature index of big column 0 (segment offsets added)
  Drop drop;
  Seg4 seg;
  // UP only: rotary embedding fused into the write-back of the segments in rope_mask (q|k heads
  // of the fused QKV output, head dim 128): out = rope(out + delta) at position rope_pos[t]
  const float* rope_cos;   // [max_pos][64]
  const float* rope_sin;
  const int* rope_pos;     // [T]
  int rope_mask;
};

// ---- software-pipelined staging ------------------------------------------------------------
// Each stage moves a [64 rows][128 cols] 16-bit "big" tile and a small f32 tile into LDS.  The
// global loads for stage s+1 are issued into registers right after the barrier of stage s and
// land while the MFMAs of stage s run; LDS is double-buffered so only one barrier per stage is
// needed.

// big tile rows [r0, r0+64) x cols [c0, c0+128): 4 x 16 B per thread, zero outside the bounds
template <typename T>
__device__ __forceinline__ void load_big(uint4 (&v)[4], const T* base, long long ld, int r0, int rmax,
                                         int c0, int cmax) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int r = r0 + (idx >> 4), c = c0 + (idx & 15) * 8;
    v[i] = (r < rmax && c < cmax) ? *reinterpret_cast<const uint4*>(base + static_cast<long long>(r) * ld + c)
                                  : make_uint4(0, 0, 0, 0);
  }
}

// write the big tile into a swizzled image, applying the dropout MASK (index t * ld + dcol0 +
// col) as a bit mask on the packed 16-bit values; the 1 / (1 - p) keep-scale is linear and is
// applied once to the kernel's f32 output (drop_alpha) instead of per element -- the per-element
// unpack / multiply / repack made these stages VALU-bound (PMC: 0.4 VALU per wave-cycle)
template <typename T, bool DROP>
__device__ __forceinline__ void store_big(char* img, uint4 (&v)[4], int r0, int c0, const Drop& d,
                                          long long dcol0) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int row = idx >> 4, ch = idx & 15;
    uint4 u = v[i];
    if (DROP) {
      const unsigned long long i0 =
          static_cast<unsigned long long>(r0 + row) * d.ld + dcol0 + c0 + ch * 8;
      const uint32_t keep = dropout_keep8(d.seed, i0, d.thresh);
      // element 2w + h sits in 16-bit half h of word w
      const auto wmask = [keep](int w) {
        return ((keep >> (2 * w)) & 1u ? 0x0000FFFFu : 0u) |
               ((keep >> (2 * w + 1)) & 1u ? 0xFFFF0000u : 0u);
      };
      u = make_uint4(u.x & wmask(0), u.y & wmask(1), u.z & wmask(2), u.w & wmask(3));
    }
    *reinterpret_cast<uint4*>(img + img_off(row, ch)) = u;
  }
}

// output scale of a kernel whose big operand went through store_big<DROP>
template <bool DROP>
__device__ __forceinline__ float drop_alpha(const Args& a) {
  return DROP ? a.alpha * a.drop.scale : a.alpha;
}

constexpr int kSmallRegs = 8;  // float4 per thread for the small tile (J <= 64)

// ------------------------------------------------------------------------------------------
// DOWN
// ------------------------------------------------------------------------------------------
constexpr int kSK = 136;  // small-tile row stride (16-bit elements): 272 B -> conflict-free reads

template <bool SMALL_KMAJ>
__device__ __forceinline__ void down_load_small(float4 (&f)[kSmallRegs], const float* small,
                                                long long lds, int J, int k0, int kend) {
#pragma unroll
  for (int i = 0; i < kSmallRegs; ++i) {
    const int idx = threadIdx.x + i * 256;
    f[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (SMALL_KMAJ) {  // small(j, k) = small[j * lds + k]: [J][32 float4]
      const int j = idx >> 5, kk = (idx & 31) * 4;
      if (j < J && k0 + kk < kend) f[i] = *reinterpret_cast<const float4*>(small + (long long)j * lds + k0 + kk);
    } else {           // small(j, k) = small[k * lds + j]: [128][J/4 float4]
      const int jq = J >> 2;
      const int kk = idx / jq, j = (idx % jq) * 4;
      if (kk < 128 && k0 + kk < kend) f[i] = *reinterpret_cast<const float4*>(small + (long long)(k0 + kk) * lds + j);
    }
  }
}

template <typename T, bool SMALL_KMAJ>
__device__ __forceinline__ void down_store_small(T* sm, const float4 (&f)[kSmallRegs], int J) {
#pragma unroll
  for (int i = 0; i < kSmallRegs; ++i) {
    const int idx = threadIdx.x + i * 256;
    if (SMALL_KMAJ) {
      const int j = idx >> 5, kk = (idx & 31) * 4;
      if (j < J) *reinterpret_cast<uint2*>(sm + j * kSK + kk) = pack4<T>(f[i].x, f[i].y, f[i].z, f[i].w);
    } else {
      const int jq = J >> 2;
      const int kk = idx / jq, j = (idx % jq) * 4;
      if (kk < 128) {
        sm[(j + 0) * kSK + kk] = from_f32<T>(f[i].x);
        sm[(j + 1) * kSK + kk] = from_f32<T>(f[i].y);
        sm[(j + 2) * kSK + kk] = from_f32<T>(f[i].z);
        sm[(j + 3) * kSK + kk] = from_f32<T>(f[i].w);
      }
    }
  }
}

template <typename T, bool DROP, bool SMALL_KMAJ>
__global__ void __launch_bounds__(256) down_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char img[2][64 * 256];
  __shared__ __attribute__((aligned(16))) T sm[2][64 * kSK];
  const int seg = blockIdx.z;
  const int K = a.seg.ncols[seg];
  const int t0 = blockIdx.x * 64;
  int kchunk = (K + a.split - 1) / a.split;
  kchunk = (kchunk + 127) / 128 * 128;
  const int kbeg = blockIdx.y * kchunk, kend = min(K, kbeg + kchunk);
  if (kbeg >= kend || t0 >= a.T) return;
  const T* big = reinterpret_cast<const T*>(a.big) + a.seg.big_off[seg];
  const float* small = a.small + a.seg.small_off[seg];
  const long long dcol0 = a.drop_col0 + a.seg.big_off[seg];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = lane & 15, g = lane >> 4;
  const int J = a.J, NJ = J >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 bv[4];
  float4 sv[kSmallRegs];
  load_big<T>(bv, big, a.ldb, t0, a.T, kbeg, kend);
  down_load_small<SMALL_KMAJ>(sv, small, a.lds, J, kbeg, kend);
  int buf = 0;
  for (int k0 = kbeg; k0 < kend; k0 += 128, buf ^= 1) {
    store_big<T, DROP>(img[buf], bv, t0, k0, a.drop, dcol0);
    down_store_small<T, SMALL_KMAJ>(sm[buf], sv, J);
    __syncthreads();
    if (k0 + 128 < kend) {
      load_big<T>(bv, big, a.ldb, t0, a.T, k0 + 128, kend);
      down_load_small<SMALL_KMAJ>(sv, small, a.lds, J, k0 + 128, kend);
    }
    const char* im = img[buf];
    const T* s2 = sm[buf];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 av = row_read(im, wid * 16 + L, ks * 4 + g);
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        if (jt < NJ) {
          const uint4 b = *reinterpret_cast<const uint4*>(s2 + (jt * 16 + L) * kSK + ks * 32 + g * 8);
          acc[jt] = Mfma<T>::run(av, b, acc[jt]);
        }
      }
    }
  }
  float* out = reinterpret_cast<float*>(a.out) + a.seg.out_off[seg];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    if (jt >= NJ) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = t0 + wid * 16 + g * 4 + r;
      if (t < a.T) atomicAdd(out + (long long)t * a.cs0 + (long long)(jt * 16 + L) * a.cs1,
                             drop_alpha<DROP>(a) * acc[jt][r]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// WGRAD
// ------------------------------------------------------------------------------------------
constexpr int kST = 72;  // transposed small-tile row stride (16-bit): 144 B -> conflict-free

__device__ __forceinline__ void wg_load_small(float4 (&f)[kSmallRegs], const float* small,
                                              long long lds, int J, int tt, int tend) {
  const int jq = J >> 2;
#pragma unroll
  for (int i = 0; i < kSmallRegs; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int t = idx / jq, j = (idx % jq) * 4;
    f[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < 64 && tt + t < tend) f[i] = *reinterpret_cast<const float4*>(small + (long long)(tt + t) * lds + j);
  }
}

template <typename T>
__device__ __forceinline__ void wg_store_small(T* st, const float4 (&f)[kSmallRegs], int J) {
  const int jq = J >> 2;
#pragma unroll
  for (int i = 0; i < kSmallRegs; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int t = idx / jq, j = (idx % jq) * 4;
    if (t < 64) {
      st[(j + 0) * kST + t] = from_f32<T>(f[i].x);
      st[(j + 1) * kST + t] = from_f32<T>(f[i].y);
      st[(j + 2) * kST + t] = from_f32<T>(f[i].z);
      st[(j + 3) * kST + t] = from_f32<T>(f[i].w);
    }
  }
}

template <typename T, bool DROP, bool SWAP>
__global__ void __launch_bounds__(256) wgrad_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char img[2][64 * 256];
  __shared__ __attribute__((aligned(16))) T st[2][64 * kST];
  const int seg = blockIdx.z;
  const int M = a.seg.ncols[seg];
  const int m0 = blockIdx.x * 128;
  int tchunk = (a.T + a.split - 1) / a.split;
  tchunk = (tchunk + 63) / 64 * 64;
  const int tbeg = blockIdx.y * tchunk, tend = min(a.T, tbeg + tchunk);
  if (tbeg >= tend || m0 >= M) return;
  const T* big = reinterpret_cast<const T*>(a.big) + a.seg.big_off[seg];
  const float* small = a.small + a.seg.small_off[seg];
  const long long dcol0 = a.drop_col0 + a.seg.big_off[seg];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = lane & 15, g = lane >> 4;
  const int J = a.J, NJ = J >> 4;
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 bv[4];
  float4 sv[kSmallRegs];
  load_big<T>(bv, big, a.ldb, tbeg, tend, m0, M);
  wg_load_small(sv, small, a.lds, J, tbeg, tend);
  int buf = 0;
  for (int tt = tbeg; tt < tend; tt += 64, buf ^= 1) {
    store_big<T, DROP>(img[buf], bv, tt, m0, a.drop, dcol0);
    wg_store_small<T>(st[buf], sv, J);
    __syncthreads();
    if (tt + 64 < tend) {
      load_big<T>(bv, big, a.ldb, tt + 64, tend, m0, M);
      wg_load_small(sv, small, a.lds, J, tt + 64, tend);
    }
    const char* im = img[buf];
    const T* s2 = st[buf];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 bigv[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) bigv[mt] = tr_read_img(im, ks * 32, wid * 32 + mt * 16, lane);
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        if (jt < NJ) {
          const uint4 sv2 = *reinterpret_cast<const uint4*>(s2 + (jt * 16 + L) * kST + ks * 32 + g * 8);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
            acc[mt][jt] = SWAP ? Mfma<T>::run(sv2, bigv[mt], acc[mt][jt])
                               : Mfma<T>::run(bigv[mt], sv2, acc[mt][jt]);
        }
      }
    }
  }
  float* out = reinterpret_cast<float*>(a.out) + a.seg.out_off[seg];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      if (jt >= NJ) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // accumulator lane holds row 4g + r, column L of the 16x16 tile
        const int m = m0 + wid * 32 + mt * 16 + (SWAP ? L : g * 4 + r);
        const int j = jt * 16 + (SWAP ? g * 4 + r : L);
        if (m < M)
          atomicAdd(out + (long long)m * a.cs0 + (long long)j * a.cs1, drop_alpha<DROP>(a) * acc[mt][jt][r]);
      }
    }
}

// ------------------------------------------------------------------------------------------
// UP:  out[t, c] += a * sum_j small1[t, j] * small2(c, j)    (16-bit read-modify-write output)
//      mode 6:  y  += s Z_seg B_seg^T      small1 = Z,  small2(c, j) = B[c][j]   (FLAG = true)
//      mode 5:  dx += drop'(dZ A)          small1 = dZ, small2(c, j) = A[j][c]   (FLAG = false)
// Block = 128 output columns x RT row tiles of 64; the small2 slice [128][J] is staged once as
// bf16 in LDS; each wave computes 16 rows x 128 columns (8 MFMA n-tiles), stages the f32 tile
// through its LDS scratch and updates the output with 16-byte row vectors.
// ------------------------------------------------------------------------------------------
constexpr int kUpRT = 4;            // row tiles (of 64) per block
constexpr int kUS = 72;             // small2 LDS row stride (16-bit): 144 B, conflict-free
constexpr int kUC = 132;            // f32 scratch row stride

template <typename T, bool DROP, bool FLAG>
__global__ void __launch_bounds__(256) up_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) T s2[128 * kUS];
  __shared__ __attribute__((aligned(16))) float scr[4][16 * kUC];
  const int seg = blockIdx.z;
  const int NC = a.seg.ncols[seg];
  const int c0 = blockIdx.x * 128;
  if (c0 >= NC) return;
  const int J = a.J, KJ = J > 32 ? 64 : 32;
  const float* small1 = a.small + a.seg.small_off[seg];       // [T][lds] f32, J columns
  const float* small2 = reinterpret_cast<const float*>(a.big) + a.seg.big_off[seg];  // f32
  T* out = reinterpret_cast<T*>(a.out) + a.seg.out_off[seg];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int L = lane & 15, g = lane >> 4;

  // stage small2(c, j) for c in [c0, c0+128), j in [0, KJ) (zero beyond J / NC) as [c][j]
  for (int idx = threadIdx.x; idx < 128 * (KJ / 4); idx += 256) {
    int c, j;
    if (FLAG) { c = idx / (KJ / 4); j = (idx % (KJ / 4)) * 4; }   // B[c][j..j+4]: j contiguous
    else { j = idx / 32; c = (idx % 32) * 4; }                  // A[j][c..c+4]: c contiguous
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (FLAG) {
      if (c0 + c < NC && j < J) f = *reinterpret_cast<const float4*>(small2 + (long long)(c0 + c) * a.ldb + j);
      *reinterpret_cast<uint2*>(s2 + c * kUS + j) = pack4<T>(f.x, f.y, f.z, f.w);
    } else {
      if (j < J && c0 + c < NC) f = *reinterpret_cast<const float4*>(small2 + (long long)j * a.ldb + c0 + c);
      s2[(c + 0) * kUS + j] = from_f32<T>(f.x);
      s2[(c + 1) * kUS + j] = from_f32<T>(f.y);
      s2[(c + 2) * kUS + j] = from_f32<T>(f.z);
      s2[(c + 3) * kUS + j] = from_f32<T>(f.w);
    }
  }
  __syncthreads();
  float* sc = scr[wid];
  const int row_blocks = (a.T + 63) / 64;
  for (int rt = 0; rt < kUpRT; ++rt) {
    const int t0 = (blockIdx.y * kUpRT + rt) * 64;
    if (t0 >= a.T) break;
    const int trow = t0 + wid * 16 + L;   // A-operand row of this lane
    f32x4 acc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks * 32 >= KJ) break;
      const int j = ks * 32 + g * 8;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = 0.f;
      if (trow < a.T && j < J) {
        const float4 u = *reinterpret_cast<const float4*>(small1 + (long long)trow * a.lds + j);
        const float4 v = *reinterpret_cast<const float4*>(small1 + (long long)trow * a.lds + j + 4);
        f[0] = u.x; f[1] = u.y; f[2] = u.z; f[3] = u.w; f[4] = v.x; f[5] = v.y; f[6] = v.z; f[7] = v.w;
      }
      const uint4 av = pack8<T>(f);
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const uint4 bv = *reinterpret_cast<const uint4*>(s2 + (n * 16 + L) * kUS + j);
        acc[n] = Mfma<T>::run(av, bv, acc[n]);
      }
    }
    // accumulator (row 4g+r, col L) of n-tile n -> scratch [16][128] f32
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[(g * 4 + r) * kUC + n * 16 + L] = acc[n][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scratch writes land before the reads
    // 16 rows x 128 cols = 256 vectors of 8; 4 per lane
    const bool rope = (a.rope_mask >> seg) & 1;
    // issue every global load of the write-back (4 output vectors per lane and, for RoPE
    // segments, their cos/sin) before any arithmetic, so one memory latency covers the tile
    uint4 yr[4];
    float4 cr[4][2], sr[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = lane + i * 64;
      const int rr = v >> 4, cc = (v & 15) * 8;
      const int t = t0 + wid * 16 + rr, c = c0 + cc;
      const bool ok = t < a.T && c < NC;
      yr[i] = ok ? *reinterpret_cast<const uint4*>(out + (long long)t * a.cs0 + c) : make_uint4(0, 0, 0, 0);
      if (rope) {
        const long long p = (ok ? a.rope_pos[t] : 0) * 64LL + (cc & 63);
        cr[i][0] = *reinterpret_cast<const float4*>(a.rope_cos + p);
        cr[i][1] = *reinterpret_cast<const float4*>(a.rope_cos + p + 4);
        sr[i][0] = *reinterpret_cast<const float4*>(a.rope_sin + p);
        sr[i][1] = *reinterpret_cast<const float4*>(a.rope_sin + p + 4);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = lane + i * 64;
      const int rr = v >> 4, cc = (v & 15) * 8;
      const int t = t0 + wid * 16 + rr, c = c0 + cc;
      const bool ok = t < a.T && c < NC;
      float y[8];
      unpack8<T>(yr[i], y);
      const uint32_t keep = DROP ? dropout_keep8(a.drop.seed,
                                                 (unsigned long long)t * a.drop.ld + a.drop_col0 + c,
                                                 a.drop.thresh)
                                 : 0xFFu;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float add = a.alpha * sc[rr * kUC + cc + e];
        if (DROP) add = (keep >> e) & 1u ? add * a.drop.scale : 0.f;
        y[e] += add;
      }
      if (rope) {  // block-uniform: the 128 columns of this block are one head
        // rotate_half partner of column cc is cc ^ 64, held by lane ^ 8 of the same 16-lane row
        const float sg = cc < 64 ? -1.f : 1.f;
        const float cs[8] = {cr[i][0].x, cr[i][0].y, cr[i][0].z, cr[i][0].w,
                             cr[i][1].x, cr[i][1].y, cr[i][1].z, cr[i][1].w};
        const float sn[8] = {sr[i][0].x, sr[i][0].y, sr[i][0].z, sr[i][0].w,
                             sr[i][1].x, sr[i][1].y, sr[i][1].z, sr[i][1].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float partner = __builtin_bit_cast(
              float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y[e]), 0x128, 0xF, 0xF, false));
          y[e] = y[e] * cs[e] + sg * partner * sn[e];
        }
      }
      if (ok) store8(out + (long long)t * a.cs0 + c, y);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's writes
  }
  (void)row_blocks;
}

template <typename T>
hipError_t launch(int kind, bool drop, bool flag, const Args& a, dim3 grid, hipStream_t st) {
  dim3 block(256);
  if (kind == 0) {
    if (drop) {
      if (flag) hipLaunchKernelGGL((down_kernel<T, true, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((down_kernel<T, true, false>), grid, block, 0, st, a);
    } else {
      if (flag) hipLaunchKernelGGL((down_kernel<T, false, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((down_kernel<T, false, false>), grid, block, 0, st, a);
    }
  } else if (kind == 2) {
    if (drop) {
      if (flag) hipLaunchKernelGGL((up_kernel<T, true, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((up_kernel<T, true, false>), grid, block, 0, st, a);
    } else {
      if (flag) hipLaunchKernelGGL((up_kernel<T, false, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((up_kernel<T, false, false>), grid, block, 0, st, a);
    }
  } else {
    if (drop) {
      if (flag) hipLaunchKernelGGL((wgrad_kernel<T, true, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((wgrad_kernel<T, true, false>), grid, block, 0, st, a);
    } else {
      if (flag) hipLaunchKernelGGL((wgrad_kernel<T, false, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((wgrad_kernel<T, false, false>), grid, block, 0, st, a);
    }
  }
  return hipGetLastError();
}

}  // namespace lv2
}  // namespace lumen

// kind 0 = DOWN (flag = small operand is k-major), kind 1 = WGRAD (flag = swapped output
// orientation: out[m*cs0 + j*cs1] with the 16 lanes of an accumulator row walking m),
// kind 2 = UP (flag = small2 is B[c][j] (mode 6) rather than A[j][c] (mode 5)); for UP `big` is
// the f32 small2 matrix (row stride ldb), `out` the 16-bit output (row stride cs0) and `split`
// is ignored.
// Host-checked requirements: J in {16,32,48,64}; ldb, big offsets, segment widths multiples of 8;
// lds and small offsets multiples of 4; 16-byte aligned bases.
extern "C" hipError_t lumen_lora2(int dtype, int kind, int flag, const void* big, long long ldb,
                                  const float* small, long long lds, void* out, long long cs0,
                                  long long cs1, float alpha, int T, int J, int split,
                                  unsigned long long seed, unsigned int drop_thresh,
                                  float drop_scale, long long drop_ld, long long drop_col0,
                                  int nseg, const long long* big_off, const long long* small_off,
                                  const long long* out_off, const int* ncols, const float* rope_cos,
                                  const float* rope_sin, const int* rope_pos, int rope_mask,
                                  hipStream_t st) {
  if (nseg < 1 || nseg > 4 || split < 1 || J < 16 || J > 64 || (J & 15) || T <= 0)
    return hipErrorInvalidValue;
  lumen::lv2::Args a;
  a.big = big; a.ldb = ldb; a.small = small; a.lds = lds; a.out = out; a.cs0 = cs0; a.cs1 = cs1;
  a.alpha = alpha; a.T = T; a.J = J; a.split = split; a.drop_col0 = drop_col0;
  a.drop.seed = static_cast<unsigned int>(seed) ^ static_cast<unsigned int>(seed >> 32);
  a.drop.thresh = drop_thresh; a.drop.scale = drop_scale; a.drop.ld = drop_ld;
  a.rope_cos = rope_cos; a.rope_sin = rope_sin; a.rope_pos = rope_pos;
  a.rope_mask = (kind == 2 && rope_cos && rope_sin && rope_pos) ? rope_mask : 0;
  a.seg.nseg = nseg;
  int maxc = 0;
  for (int i = 0; i < 4; ++i) {
    const bool v = i < nseg;
    a.seg.big_off[i] = v ? big_off[i] : 0; a.seg.small_off[i] = v ? small_off[i] : 0;
    a.seg.out_off[i] = v ? out_off[i] : 0; a.seg.ncols[i] = v ? ncols[i] : 0;
    if (v && ncols[i] > maxc) maxc = ncols[i];
  }
  if (maxc == 0) return hipSuccess;
  dim3 grid = kind == 0 ? dim3((T + 63) / 64, split, nseg)
             : kind == 2 ? dim3((maxc + 127) / 128, (T + 64 * lumen::lv2::kUpRT - 1) / (64 * lumen::lv2::kUpRT), nseg)
                         : dim3((maxc + 127) / 128, split, nseg);
  const bool drop = drop_thresh != 0;
  if (dtype == lumen::kBF16) return lumen::lv2::launch<lumen::bf16>(kind, drop, flag, a, grid, st);
  if (dtype == lumen::kF16) return lumen::lv2::launch<lumen::fp16>(kind, drop, flag, a, grid, st);
  return hipErrorInvalidValue;
}
