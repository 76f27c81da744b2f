// Decode-batch GEMM on the matrix cores: y[M, N] = x[M, K] @ W[N, K]^T for 2 <= M <= 256.
//
// Reference behaviour: vLLM's decode projections (the serving stack the reference declares,
// SURVEY D11 / CS6) run these as library GEMMs.  At decode batch sizes hipBLASLt (with the tuned
// table, profiles/r02_serve) leaves most of the chip idle: M = 256 o_proj runs 23.4 us for
// 33.5 MB of weights (1.4 TB/s, 0.37 PF/s), because its 256x256 / 64x64 tiles give 16-256
// workgroups at K = 4096.  The op is weight-streaming up to M ~ 300 (2M FLOP per weight
// element vs 2.5 PF/s : 8 TB/s), so the design target is HBM bandwidth on W.
//
// Design (gfx950, wave64, v_mfma_f32_32x32x16_bf16):
//  * one workgroup = NW waves (NW = ceil(M / 32) <= 4) = a 32*NW x 64 output tile; wave w owns
//    rows [32w, 32w + 32) of the M tile against all 64 weight rows (two 32x32 accumulators);
//  * W streams in 128-column stages through two separately declared LDS images (256-byte rows,
//    XOR-swizzled 16-byte chunks) filled by LDS-DMA (global_load_lds: no VGPRs, 1 KiB per wave
//    instruction), shared by the NW waves; stage s+1 is in flight while stage s is multiplied;
//  * x (L2-resident: <= 256 x K) goes straight to registers in the MFMA B layout (lane: row
//    m = lane & 31, k = 8 (lane >> 5) + 0..7), prefetched one stage ahead;
//  * W is the A operand, so the accumulator is y^T: each lane holds 4 consecutive n of one m
//    per register quad -> 8-byte stores;
//  * too few tiles to fill 256 CUs (o / down: 64 column tiles) are split over K; the splits
//    write f32 partials with agent-scope (sc1) stores and the last split of a tile to arrive
//    (arrival counter, self-resetting) sums them in fixed order -- deterministic, one launch;
//  * workgroup ids are remapped XCD-aware (hardware dispatch is round-robin over the 8 XCDs):
//    the M tiles of one (column tile, split) run on one XCD and share W through its L2.
#include "common.h"

namespace lumen {
namespace dg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma32;
template <> struct Mfma32<bf16> {
  static __device__ __forceinline__ f32x16 run(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mfma32<fp16> {
  static __device__ __forceinline__ f32x16 run(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * 256 + ((chunk ^ swz(row)) << 4);
}
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(p)));
}
// LDS reads as inline asm: the compiler cannot prove they do not alias the LDS-DMA in flight
// into the other image and would otherwise put vmcnt(0) in front of them (serialising the
// prefetch); completion is ordered explicitly by lgkm_wait's register operands.
template <int OFF>
__device__ __forceinline__ u32x4v ds_b128(unsigned a) {
  u32x4v r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
__device__ __forceinline__ void lgkm_wait(u32x4v& a, u32x4v& b, u32x4v& c, u32x4v& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void lgkm_wait(u32x4v& a, u32x4v& b, u32x4v& c, u32x4v& d,
                                          u32x4v& e, u32x4v& f, u32x4v& g, u32x4v& h) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
}
__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// s_waitcnt vmcnt(V) (gfx9 simm16: vmcnt [3:0] + [15:14], expcnt [6:4] = 7, lgkmcnt [11:8] = 15)
template <int V>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt(0xF70 | (V & 15) | ((V >> 4) << 14));
}
// 16-byte load through the global address space (a generic pointer lets the compiler pick flat
// loads, which also count on lgkmcnt and would be waited for by every LDS wait)
__device__ __forceinline__ uint4 gload16(const void* p) {
  return __builtin_bit_cast(uint4, *reinterpret_cast<const __attribute__((address_space(1))) u32x4v*>(
                                       reinterpret_cast<uintptr_t>(p)));
}
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Args {
  const void* x;
  const void* W;
  void* y;
  float* ws;           // split partials [S][MT * 32 NW][N] f32 (S > 1)
  unsigned* cnt;       // arrival counters [MT * N / 64], zero on entry and on exit (S > 1)
  long long ldx, ldy;  // row strides (elements)
  int M, N, K, S, MT;
};

template <typename T, int NW>
__global__ void __launch_bounds__(NW * 64) dgemm_kernel(Args a) {
  constexpr int BM = NW * 32;
  constexpr int NWD = 16 / NW;  // LDS-DMA instructions per wave per stage (64 rows x 256 B)
  __shared__ __attribute__((aligned(1024))) char imgA[64 * 256];
  __shared__ __attribute__((aligned(1024))) char imgB[64 * 256];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int NT = a.N >> 6;
  // XCD-aware tile order: the 8 XCDs each take a contiguous range of logical tiles, M tiles of
  // one (column tile, split) adjacent
  const int total = gridDim.x, id = blockIdx.x;
  const int L = (total & 7) == 0 ? (id & 7) * (total >> 3) + (id >> 3) : id;
  const int mt = L % a.MT, rest = L / a.MT;
  const int s = rest % a.S, nt = rest / a.S;
  const int n0 = nt * 64, m0 = mt * BM;
  const int nst = a.K >> 7;
  const int st0 = (s * nst) / a.S, st1 = ((s + 1) * nst) / a.S;

  const T* W = reinterpret_cast<const T*>(a.W);
  const T* x = reinterpret_cast<const T*>(a.x);
  const int mrow = m0 + wid * 32 + (lane & 31);
  const bool mok = mrow < a.M;
  // rows >= M load row 0 (always in bounds): output row m depends on x row m only, and rows
  // >= M are never stored, so no masking (and no divergent loads) is needed
  const T* xp = x + (long long)(mok ? mrow : 0) * a.ldx + 8 * (lane >> 5);

  // LDS-DMA of W rows [n0, n0 + 64) x cols [128 st, 128 st + 128) into img: wave-instruction i
  // fills image rows 4i..4i+3 (1 KiB, lane-linear on the LDS side; swizzle on the source side)
  auto stage_w = [&](int st, char* img) {
#pragma unroll
    for (int j = 0; j < NWD; ++j) {
      const int i = wid + j * NW;
      const int row = i * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ swz(row);
      __builtin_amdgcn_global_load_lds(
          (const void*)(W + (long long)(n0 + row) * a.K + st * 128 + ch * 8),
          (__attribute__((address_space(3))) void*)(img + i * 1024), 16, 0, 0);
    }
  };
  auto load_x = [&](int st, uint4 (&xr)[8]) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) xr[ks] = gload16(xp + st * 128 + ks * 16);
  };
  // per-lane image offsets of the A fragments: W row (lane & 31) [+32], chunk 2 ks + (lane >> 5)
  unsigned off[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) off[ks] = img_off(lane & 31, 2 * ks + (lane >> 5));

  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }

  auto compute = [&](const char* img, const uint4 (&xr)[8]) {
    const unsigned base = lds_addr(img);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      u32x4v w0[4], w1[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w0[q] = ds_b128<0>(base + off[4 * h + q]);
        w1[q] = ds_b128<8192>(base + off[4 * h + q]);
      }
      lgkm_wait(w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc0 = Mfma32<T>::run(__builtin_bit_cast(uint4, w0[q]), xr[4 * h + q], acc0);
        acc1 = Mfma32<T>::run(__builtin_bit_cast(uint4, w1[q]), xr[4 * h + q], acc1);
      }
    }
  };

  // Stage pairs (imgA, imgB) with no exit in the middle of an iteration: the in-flight count is
  // then the same on every path into each wait, so the compiler's own waits for the x
  // registers agree with wait_vm instead of degrading to vmcnt(0).  An odd last stage was
  // prefetched into imgA by the final pair (which otherwise re-issues it, harmlessly).
  uint4 xa[8], xb[8];
  stage_w(st0, imgA);
  load_x(st0, xa);
  for (int st = st0; st + 1 < st1; st += 2) {
    stage_w(st + 1, imgB);
    load_x(st + 1, xb);
    wait_vm<NWD + 8>();  // stage st (issued one round earlier) has landed
    barrier();
    compute(imgA, xa);
    barrier();  // every wave is done with imgA before it is refilled
    const int p2 = st + 2 < st1 ? st + 2 : st1 - 1;
    stage_w(p2, imgA);
    load_x(p2, xa);
    wait_vm<NWD + 8>();
    barrier();
    compute(imgB, xb);
    barrier();
  }
  wait_vm<0>();  // also: no LDS-DMA may be in flight when the workgroup's LDS is released
  if ((st1 - st0) & 1) {
    barrier();
    compute(imgA, xa);
  }

  // accumulator tile t: register 4j + i = (n = 32t + 8j + 4 (lane >> 5) + i, m = lane & 31)
  const int nb = n0 + 4 * (lane >> 5);
  if (a.S == 1) {
    if (mok) {
      T* yr = reinterpret_cast<T*>(a.y) + (long long)mrow * a.ldy;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        *reinterpret_cast<uint2*>(yr + nb + 8 * j) =
            make_uint2(pk2<T>(acc0[4 * j], acc0[4 * j + 1]), pk2<T>(acc0[4 * j + 2], acc0[4 * j + 3]));
        *reinterpret_cast<uint2*>(yr + nb + 32 + 8 * j) =
            make_uint2(pk2<T>(acc1[4 * j], acc1[4 * j + 1]), pk2<T>(acc1[4 * j + 2], acc1[4 * j + 3]));
      }
    }
    return;
  }
  // split-K: f32 partial of this split, then the last split to arrive reduces the tile
  const int Mp = a.MT * BM;
  float* wp = a.ws + ((long long)s * Mp + mrow) * a.N + nb;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st_agent(wp + 8 * j + i, acc0[4 * j + i]);
      st_agent(wp + 32 + 8 * j + i, acc1[4 * j + i]);
    }
  wait_vm<0>();  // this wave's partial stores are complete (written through to device scope)
  barrier();
  __shared__ int last;
  if (threadIdx.x == 0) {
    unsigned* cp = a.cnt + mt * NT + nt;
    const unsigned prev = __hip_atomic_fetch_add(cp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int l = prev == static_cast<unsigned>(a.S - 1);
    if (l) __hip_atomic_store(cp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = l;
  }
  barrier();
  if (!last) return;
  T* y = reinterpret_cast<T*>(a.y);
  for (int e = threadIdx.x; e < BM * 16; e += NW * 64) {  // 4 consecutive columns per item
    const int r = e >> 4, c = (e & 15) * 4;
    const int m = m0 + r;
    if (m >= a.M) continue;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < a.S; ++sp) {
      const float* p = a.ws + ((long long)sp * Mp + m) * a.N + n0 + c;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += ld_agent(p + i);
    }
    *reinterpret_cast<uint2*>(y + (long long)m * a.ldy + n0 + c) =
        make_uint2(pk2<T>(v[0], v[1]), pk2<T>(v[2], v[3]));
  }
}

template <typename T>
hipError_t launch(const Args& a, hipStream_t st) {
  const int nw = (a.M + 31) / 32 >= 4 ? 4 : (a.M + 31) / 32;
  const dim3 grid((a.N / 64) * a.MT * a.S);
  if (nw == 4) hipLaunchKernelGGL((dgemm_kernel<T, 4>), grid, dim3(256), 0, st, a);
  else if (nw == 2) hipLaunchKernelGGL((dgemm_kernel<T, 2>), grid, dim3(128), 0, st, a);
  else if (nw == 3) hipLaunchKernelGGL((dgemm_kernel<T, 4>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((dgemm_kernel<T, 1>), grid, dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace dg
}  // namespace lumen

// Workgroup rows per M tile for a given M (the host sizes MT and the split workspace with it).
extern "C" int lumen_dgemm_tile_m(int M) {
  const int nw = (M + 31) / 32;
  return nw >= 3 ? 128 : nw * 32;
}

// y[M, N] = x[M, K] @ W[N, K]^T; 1 <= M <= 256, N % 64 == 0, K % 128 == 0, x / y row strides
// multiples of 8 / 4 elements, 16-byte aligned bases.  S > 1 needs ws (S * MT * tile_m * N f32)
// and cnt (MT * N / 64 zeroed counters).
extern "C" hipError_t lumen_dgemm(int dtype, const void* x, const void* W, void* y, int M, int N,
                                  int K, long long ldx, long long ldy, int S, float* ws,
                                  unsigned* cnt, hipStream_t st) {
  if (M < 1 || M > 256 || N % 64 != 0 || K % 128 != 0 || S < 1 || S > K / 128 ||
      (S > 1 && (ws == nullptr || cnt == nullptr)))
    return hipErrorInvalidValue;
  lumen::dg::Args a;
  a.x = x; a.W = W; a.y = y; a.ws = ws; a.cnt = cnt; a.ldx = ldx; a.ldy = ldy;
  a.M = M; a.N = N; a.K = K; a.S = S;
  const int bm = lumen_dgemm_tile_m(M);
  a.MT = (M + bm - 1) / bm;
  if (dtype == lumen::kBF16) return lumen::dg::launch<lumen::bf16>(a, st);
  if (dtype == lumen::kF16) return lumen::dg::launch<lumen::fp16>(a, st);
  return hipErrorInvalidValue;
}
