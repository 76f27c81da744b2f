// Paged-KV decode attention + KV-cache write (serving half of the north star).
//
// Reference behaviour: the reference only declares vLLM 0.6.0 serving (README.md:10,16,
// requirements.txt:17-18); vLLM's PagedAttention v1/v2 reads K/V through per-sequence block
// tables and splits long contexts into partitions reduced by a second kernel.
//
// Cache layout (chosen for wave64 coalescing, not vLLM's x-packed key layout):
//     k_cache, v_cache : [num_blocks, num_kv_heads, block_size, D]
// so one (block, kv-head) is a contiguous block_size*D*2-byte run (4 KiB at 16 x 128 bf16).
//
// Decode kernel: one 256-thread workgroup per (sequence, kv-head, context partition) serves ALL
// query heads of that GQA group, so K/V bytes are read once per group (memory-bound: the only
// cost that matters at decode).  D/8 lanes cooperate on one cache row (16-byte loads), 256/(D/8)
// rows per step; q lives in LDS (f32, pre-scaled); scores for the partition stay in LDS; softmax
// is one wave per head; P.V accumulates per lane then reduces through LDS.  Contexts longer than
// one partition write unnormalised (m, l, o) partials that `pa_reduce_kernel` merges.
#include "common.h"

#include <type_traits>

namespace lumen {

constexpr int kMaxGroup = 8;

// fp8 KV cache (vLLM --kv-cache-dtype fp8): one OCP e4m3fn byte per element, converted with the
// gfx950 packed converts (v_cvt_pk_f32_fp8 / v_cvt_pk_fp8_f32), no scale (vLLM's uncalibrated
// default of 1.0).  Halves the K/V bytes every decode step streams.
using fp8 = unsigned char;

template <typename T, typename KT>
__device__ __forceinline__ void load8kv(const KT* __restrict__ p, float (&o)[8]) {
  if constexpr (std::is_same<KT, fp8>::value) {
    const uint2 r = *reinterpret_cast<const uint2*>(p);
    const auto a = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.x), false);
    const auto b = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.x), true);
    const auto c = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.y), false);
    const auto d = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.y), true);
    o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1];
    o[4] = c[0]; o[5] = c[1]; o[6] = d[0]; o[7] = d[1];
  } else {
    load8(p, o);
  }
}

// 8 elements already in registers (the raw row piece a lane loaded: uint2 of fp8, uint4 of T)
template <typename T, typename KT, typename R>
__device__ __forceinline__ void cvt8kv(const R& r, float (&o)[8]) {
  if constexpr (std::is_same<KT, fp8>::value) {
    const auto a = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.x), false);
    const auto b = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.x), true);
    const auto c = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.y), false);
    const auto d = __builtin_amdgcn_cvt_pk_f32_fp8(static_cast<int>(r.y), true);
    o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1];
    o[4] = c[0]; o[5] = c[1]; o[6] = d[0]; o[7] = d[1];
  } else {
    const T* e = reinterpret_cast<const T*>(&r);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = to_f32(e[j]);
  }
}

template <typename T, typename KT>
__device__ __forceinline__ void store8kv(KT* __restrict__ p, const float (&v)[8]) {
  if constexpr (std::is_same<KT, fp8>::value) {
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
    *reinterpret_cast<uint2*>(p) = make_uint2(static_cast<unsigned>(lo), static_cast<unsigned>(hi));
  } else {
    store8(p, v);
  }
}

template <int W>
__device__ __forceinline__ float wave_sum_width(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Row reduction over the 16 lanes of a DPP row (quad_perm xor1/xor2, half-mirror, mirror).
template <int CTRL>
__device__ __forceinline__ float pa_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
__device__ __forceinline__ float pa_red16(float v) {
  v += pa_dpp<0xB1>(v);
  v += pa_dpp<0x4E>(v);
  v += pa_dpp<0x141>(v);
  v += pa_dpp<0x140>(v);
  return v;
}

__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T, int D, int G>
__global__ void __launch_bounds__(256) pa_decode_kernel(
    T* __restrict__ out, const T* __restrict__ q, const T* __restrict__ kc,
    const T* __restrict__ vc, const int* __restrict__ block_tables,
    const int* __restrict__ context_lens, int nh, int qldh, int nkv, int BS, int max_blocks, int max_parts,
    float scale, float* __restrict__ tmp_m, float* __restrict__ tmp_l, float* __restrict__ tmp_o,
    int PART, unsigned* __restrict__ counters) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int LPT = D / 8;        // lanes per cache row (16-byte chunk each)
  constexpr int RPS = 256 / LPT;    // rows per workgroup step
  constexpr int U = 4;              // rows in flight per thread (memory-level parallelism)
  const int seq = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z;
  const int ctx = context_lens[seq];
  const int start = part * PART;
  if (start >= ctx) return;
  const int end = min(ctx, start + PART);
  const int n = end - start;
  float* sc = smem;                  // [G][PART] scores, then probabilities
  float* red = sc + G * PART;        // [4 waves][G][D] PV partials
  float* ml = red + 4 * G * D;       // [2][G] + scratch [8]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int rsub = tid / LPT, d0 = (tid % LPT) * 8;
  // this lane's 8 q values for each head of the group (f32, pre-scaled)
  float qv[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    load8(q + (static_cast<size_t>(seq) * qldh + kvh * G + h) * D + d0, qv[h]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[h][j] *= scale;
  }
  const int* bt = block_tables + static_cast<size_t>(seq) * max_blocks;
  const size_t head_off = static_cast<size_t>(kvh) * BS * D;
  const size_t blk_stride = static_cast<size_t>(nkv) * BS * D;
  // ---- scores: U independent 16-byte K loads in flight per thread ----
  for (int t0 = start + rsub; t0 < end; t0 += RPS * U) {
    float kv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * RPS;
      if (t < end) {
        const T* kr = kc + bt[t / BS] * blk_stride + head_off + (t % BS) * D + d0;
        load8(kr, kv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * RPS;
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += kv[u][j] * qv[h][j];
        s = LPT == 16 ? pa_red16(s) : wave_sum_width<LPT>(s);
        if (t < end && (tid % LPT) == 0) sc[h * PART + (t - start)] = s;
      }
    }
  }
  __syncthreads();
  // ---- softmax over the partition (every wave covers a slice of the scores) ----
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float m = -INFINITY;
    for (int i = tid; i < n; i += 256) m = fmaxf(m, sc[h * PART + i]);
    m = block_max<256>(m, ml + 2 * G);
    float l = 0.f;
    for (int i = tid; i < n; i += 256) {
      const float p = __expf(sc[h * PART + i] - m);
      sc[h * PART + i] = p;
      l += p;
    }
    l = block_sum<256>(l, ml + 2 * G);
    if (tid == 0) { ml[h] = m; ml[G + h] = l; }
  }
  __syncthreads();
  // ---- P.V: U independent V loads in flight ----
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  for (int t0 = start + rsub; t0 < end; t0 += RPS * U) {
    float vv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * RPS;
      if (t < end) {
        const T* vr = vc + bt[t / BS] * blk_stride + head_off + (t % BS) * D + d0;
        load8(vr, vv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * RPS;
      if (t < end) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
          const float p = sc[h * PART + (t - start)];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[h][j] += p * vv[u][j];
        }
      }
    }
  }
  // reduce the 64/LPT row groups of each wave, then the 4 waves through LDS
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = acc[h][j];
#pragma unroll
      for (int o = LPT; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
      acc[h][j] = x;
    }
  if (lane < LPT) {
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(wid * G + h) * D + d0 + j] = acc[h][j];
  }
  __syncthreads();
  const int nparts = (ctx + PART - 1) / PART;
  for (int i = tid; i < G * D; i += 256) {
    const float o = red[i] + red[G * D + i] + red[2 * G * D + i] + red[3 * G * D + i];
    const int h = i / D, d = i % D;
    const int head = kvh * G + h;
    if (nparts == 1) {  // the whole context in this partition: final output directly
      out[(static_cast<size_t>(seq) * nh + head) * D + d] = from_f32<T>(o / ml[G + h]);
    } else {
      const size_t mi = (static_cast<size_t>(seq) * nh + head) * max_parts + part;
      st_agent(tmp_o + mi * D + d, o);
      if (d == 0) { st_agent(tmp_m + mi, ml[h]); st_agent(tmp_l + mi, ml[G + h]); }
    }
  }
  if (nparts == 1 || counters == nullptr) return;
  // Split context, fused merge: the last partition of this (sequence, kv-head) to arrive merges
  // all partials (no second launch).  Partitions run on different XCDs, whose L2s are not
  // coherent with each other: the partials go out as agent-scope stores (sc1, written through
  // to the coherent level) and are read back with agent-scope loads, and every store has
  // completed (vmcnt(0)) before the arrival count, so no L2 writeback / invalidate (the
  // buffer_wbl2 + buffer_inv of __threadfence(), measured 7x slower decode steps) is needed.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's partial stores are complete
  __syncthreads();
  int* flag = reinterpret_cast<int*>(ml + 2 * G);
  if (tid == 0) {
    unsigned* cp = counters + static_cast<size_t>(seq) * nkv + kvh;
    const unsigned prev = __hip_atomic_fetch_add(cp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == static_cast<unsigned>(nparts - 1);
    if (last)  // self-resetting for the next launch (next layer)
      __hip_atomic_store(cp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  for (int i = tid; i < G * D; i += 256) {
    const int h = i / D, d = i % D;
    const size_t base = (static_cast<size_t>(seq) * nh + kvh * G + h) * max_parts;
    float M = -INFINITY;
    for (int p = 0; p < nparts; ++p) M = fmaxf(M, ld_agent(tmp_m + base + p));
    float L = 0.f, o = 0.f;
    for (int p = 0; p < nparts; ++p) {
      const float w = __expf(ld_agent(tmp_m + base + p) - M);
      L += ld_agent(tmp_l + base + p) * w;
      o += ld_agent(tmp_o + (base + p) * D + d) * w;
    }
    out[(base / max_parts) * D + d] = from_f32<T>(o / L);
  }
}

// ---- single-pass variant (online softmax per row group) ------------------------------------
// The two-pass kernel above streams K, stops the memory pipe for a block-wide softmax, then
// streams V.  Here each 16-lane row group streams K AND V rows together (U of each in flight
// per lane) and keeps its own running (max, sum, P.V) state per head -- flash-decoding inside
// the workgroup -- so HBM traffic never pauses and no score buffer lives in LDS.  The 16 groups
// merge at the end: xor-16/32 exchanges inside a wave, then the 4 waves through LDS.  Output
// (and split partials for the merge kernel) have exactly the two-pass kernel's semantics.
__device__ __forceinline__ void pa_merge(float& m, float& l, float (&acc)[8], float m2, float l2,
                                         const float (&acc2)[8]) {
  const float M = fmaxf(m, m2);
  const float a1 = m == -INFINITY ? 0.f : __expf(m - M);
  const float a2 = m2 == -INFINITY ? 0.f : __expf(m2 - M);
  l = l * a1 + l2 * a2;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = acc[j] * a1 + acc2[j] * a2;
  m = M;
}

typedef unsigned int pa_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int pa_u32x2 __attribute__((ext_vector_type(2)));

// a K/V row piece read once per decode step: non-temporal (streamed past L2 / MALL retention)
template <typename R>
__device__ __forceinline__ R pa_ld_nt(const void* p) {
  R r;
  if constexpr (sizeof(R) == 16) {
    const pa_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const pa_u32x4*>(p));
    __builtin_memcpy(&r, &v, 16);
  } else {
    const pa_u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const pa_u32x2*>(p));
    __builtin_memcpy(&r, &v, 8);
  }
  return r;
}

// inline-asm form of pa_ld_nt (the PF kernel counts its own waits: see there)
template <typename R>
__device__ __forceinline__ R pa_ld_nt_asm(const void* p) {
  R r;
  if constexpr (sizeof(R) == 16) {
    pa_u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    __builtin_memcpy(&r, &v, 16);
  } else {
    pa_u32x2 v;
    asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    __builtin_memcpy(&r, &v, 8);
  }
  return r;
}

// orders every later use of these registers after the preceding asm wait
template <typename R>
__device__ __forceinline__ void pa_fence_reg(R& a, R& b) {
  if constexpr (sizeof(R) == 16) {
    pa_u32x4 x, y;
    __builtin_memcpy(&x, &a, 16);
    __builtin_memcpy(&y, &b, 16);
    asm volatile("" : "+v"(x), "+v"(y));
    __builtin_memcpy(&a, &x, 16);
    __builtin_memcpy(&b, &y, 16);
  } else {
    pa_u32x2 x, y;
    __builtin_memcpy(&x, &a, 8);
    __builtin_memcpy(&y, &b, 8);
    asm volatile("" : "+v"(x), "+v"(y));
    __builtin_memcpy(&a, &x, 8);
    __builtin_memcpy(&b, &y, 8);
  }
}

// UNI (block_size == rows per workgroup step, the launcher checks): row t = base + u * NGR + grp
// of an iteration lies in block (base / BS + u) at offset grp, so the block ids are
// workgroup-uniform -- scalar loads issued one iteration ahead -- instead of a per-lane block
// table load feeding every K / V address (a dependent L2 round trip per iteration); the K / V
// pieces are non-temporal loads.
// PF (with UNI): software-pipelined -- iteration i+1's K / V pieces are issued before iteration
// i's softmax / P.V work, so every wave keeps two iterations of loads in flight (a pure nt read
// stream reaches 7.1 TB/s on this chip with 8 x 16 B per lane in flight, profiles/r5_decode)
template <typename T, int D, int G, typename KT = T, bool UNI = false, bool PF = false>
__global__ void __launch_bounds__(256) pa_decode1_kernel(
    T* __restrict__ out, const T* __restrict__ q, const KT* __restrict__ kc,
    const KT* __restrict__ vc, const int* __restrict__ block_tables,
    const int* __restrict__ context_lens, int nh, int qldh, int nkv, int BS, int max_blocks, int max_parts,
    float scale, float* __restrict__ tmp_m, float* __restrict__ tmp_l, float* __restrict__ tmp_o,
    int PART) {
  constexpr int LPT = D / 8;        // lanes per cache row (8 elements each)
  constexpr int NGR = 256 / LPT;    // row groups per workgroup
  // K and V rows in flight per lane, loaded raw and converted at use: 4 of 16-bit rows (16 bytes
  // per lane each); 8 of fp8 rows (8 bytes each), so an fp8 cache keeps the same bytes in flight
  // (with 4 it streamed at ~3.9 TB/s against the bf16 cache's 5.9; 8 16-bit rows per lane
  // measured 26.9 vs 19.7 ms per 256-row decode step: the registers cost the occupancy)
  constexpr bool F8 = std::is_same<KT, fp8>::value;
  constexpr int U = F8 ? 8 : 4;
  using Raw = typename std::conditional<F8, uint2, uint4>::type;
  __shared__ float wst[4][G][D + 2];  // per-wave merged state: acc[D], m, l
  const int seq = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z;
  const int ctx = context_lens[seq];
  const int start = part * PART;
  if (start >= ctx) return;
  const int end = min(ctx, start + PART);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = tid / LPT, d0 = (tid % LPT) * 8;
  float qv[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    load8(q + (static_cast<size_t>(seq) * qldh + kvh * G + h) * D + d0, qv[h]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qv[h][j] *= scale;
  }
  const int* bt = block_tables + static_cast<size_t>(seq) * max_blocks;
  const size_t head_off = static_cast<size_t>(kvh) * BS * D;
  const size_t blk_stride = static_cast<size_t>(nkv) * BS * D;
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  }
  // one iteration's online-softmax update from its raw K / V pieces (rows t0 + u * NGR)
  const auto consume = [&](int t0, const Raw (&kraw)[U], const Raw (&vraw)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * NGR;
      float kr[8], vr[8];
      cvt8kv<T, KT>(kraw[u], kr);
      cvt8kv<T, KT>(vraw[u], vr);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += kr[j] * qv[h][j];
        s = LPT == 16 ? pa_red16(s) : wave_sum_width<LPT>(s);
        if (t < end) {  // uniform within the row group
          const float mn = fmaxf(m[h], s);
          const float al = __expf(m[h] - mn);  // m = -inf on the first row: al = 0
          const float p = __expf(s - mn);
          l[h] = l[h] * al + p;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[h][j] = acc[h][j] * al + p * vr[j];
          m[h] = mn;
        }
      }
    }
  };
  int nbid[U];
  if constexpr (UNI) {
#pragma unroll
    for (int u = 0; u < U; ++u) nbid[u] = start + u * NGR < end ? bt[start / NGR + u] : 0;
  }
  if constexpr (UNI && PF) {
    // Two register sets, the loop unrolled by two so they swap roles without copies (a copy of
    // the freshly issued set would wait for it); the loads are inline asm and the waits counted
    // by hand -- the compiler cannot see them, so it neither drains the set in flight before
    // the set being consumed nor waits before the branch joins.  Rows past the context read
    // their (allocated) block's slot or block 0; consume() skips them.
    const KT* kr0 = kc + head_off + static_cast<size_t>(grp) * D + d0;
    const KT* vr0 = vc + head_off + static_cast<size_t>(grp) * D + d0;
    constexpr int NL = 2 * U;  // loads per set
    const int step = NGR * U;
    const auto ids = [&](int b, int (&o)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) o[u] = b + u * NGR < end ? bt[b / NGR + u] : 0;
    };
    const auto issue = [&](const int (&id)[U], Raw (&kk)[U], Raw (&vv)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t off = static_cast<size_t>(id[u]) * blk_stride;
        kk[u] = pa_ld_nt_asm<Raw>(kr0 + off);
        vv[u] = pa_ld_nt_asm<Raw>(vr0 + off);
      }
    };
    // wait until the OLDER set landed (NEWER loads may stay in flight), then fence its registers
    const auto landed = [&](bool newer_in_flight, Raw (&kk)[U], Raw (&vv)[U]) {
      if (newer_in_flight) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) pa_fence_reg(kk[u], vv[u]);
    };
    // q must land before the first asm load issues: a later compiler-inserted wait for it
    // would be vmcnt(0) and drain the prefetched set too
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(qv[h][j]));
    Raw kA[U], vA[U], kB[U], vB[U];
    issue(nbid, kA, vA);
    ids(start + step, nbid);
    for (int base = start; base < end; base += 2 * step) {
      const int b1 = base + step;
      const bool more1 = b1 < end;
      if (more1) issue(nbid, kB, vB);
      ids(b1 + step, nbid);
      landed(more1, kA, vA);
      consume(base + grp, kA, vA);
      if (!more1) break;
      const int b2 = b1 + step;
      const bool more2 = b2 < end;
      if (more2) issue(nbid, kA, vA);
      ids(b2 + step, nbid);
      landed(more2, kB, vB);
      consume(b1 + grp, kB, vB);
    }
  } else
  for (int base = start; base < end; base += NGR * U) {
    const int t0 = base + grp;
    Raw kraw[U], vraw[U];
    if constexpr (UNI) {
      int bid[U];
#pragma unroll
      for (int u = 0; u < U; ++u) bid[u] = nbid[u];
      const int nb = base + NGR * U;
#pragma unroll
      for (int u = 0; u < U; ++u) nbid[u] = nb + u * NGR < end ? bt[nb / NGR + u] : 0;
      const KT* kr0 = kc + head_off + static_cast<size_t>(grp) * D + d0;
      const KT* vr0 = vc + head_off + static_cast<size_t>(grp) * D + d0;
      // unconditional (see the PF form): all 2U pieces in flight before the first use
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t off = static_cast<size_t>(bid[u]) * blk_stride;
        kraw[u] = pa_ld_nt<Raw>(kr0 + off);
        vraw[u] = pa_ld_nt<Raw>(vr0 + off);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 + u * NGR;
        if (t < end) {
          const size_t off = bt[t / BS] * blk_stride + head_off + (t % BS) * D + d0;
          kraw[u] = *reinterpret_cast<const Raw*>(kc + off);
          vraw[u] = *reinterpret_cast<const Raw*>(vc + off);
        }
      }
    }
    consume(t0, kraw, vraw);
  }
  // merge the 64 / LPT row groups of each wave (lanes d0-aligned at xor 16, 32, ...)
#pragma unroll
  for (int o = LPT; o < 64; o <<= 1) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float a2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a2[j] = __shfl_xor(acc[h][j], o, 64);
      const float m2 = __shfl_xor(m[h], o, 64), l2 = __shfl_xor(l[h], o, 64);
      pa_merge(m[h], l[h], acc[h], m2, l2, a2);
    }
  }
  if (lane < LPT) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
#pragma unroll
      for (int j = 0; j < 8; ++j) wst[wid][h][d0 + j] = acc[h][j];
      if (lane == 0) { wst[wid][h][D] = m[h]; wst[wid][h][D + 1] = l[h]; }
    }
  }
  __syncthreads();
  const int nparts = (ctx + PART - 1) / PART;
  for (int i = tid; i < G * D; i += 256) {
    const int h = i / D, d = i % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, wst[w][h][D]);
    float L = 0.f, o = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float mw = wst[w][h][D];
      const float a = mw == -INFINITY ? 0.f : __expf(mw - M);
      L += wst[w][h][D + 1] * a;
      o += wst[w][h][d] * a;
    }
    const int head = kvh * G + h;
    if (nparts == 1) {
      out[(static_cast<size_t>(seq) * nh + head) * D + d] = from_f32<T>(o / L);
    } else {
      const size_t mi = (static_cast<size_t>(seq) * nh + head) * max_parts + part;
      tmp_o[mi * D + d] = o;
      if (d == 0) { tmp_m[mi] = M; tmp_l[mi] = L; }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) pa_reduce_kernel(T* __restrict__ out,
                                                        const int* __restrict__ context_lens,
                                                        const float* __restrict__ tmp_m,
                                                        const float* __restrict__ tmp_l,
                                                        const float* __restrict__ tmp_o, int nh,
                                                        int D, int max_parts, int PART) {
  const int seq = blockIdx.x, head = blockIdx.y;
  const int nparts = (context_lens[seq] + PART - 1) / PART;
  if (nparts <= 1) return;  // written directly by the decode kernel
  const size_t base = (static_cast<size_t>(seq) * nh + head) * max_parts;
  float M = -INFINITY;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, tmp_m[base + p]);
  float L = 0.f;
  for (int p = 0; p < nparts; ++p) L += tmp_l[base + p] * __expf(tmp_m[base + p] - M);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float o = 0.f;
    for (int p = 0; p < nparts; ++p) o += tmp_o[(base + p) * D + d] * __expf(tmp_m[base + p] - M);
    out[(static_cast<size_t>(seq) * nh + head) * D + d] = from_f32<T>(o / L);
  }
}

// k, v: [ntok, nkv, D] rows with row strides k_stride / v_stride (elements), scattered to
// cache[block][head][slot][:] by slot_mapping (slot = block * BS + offset; < 0 = skip).
template <typename T, typename KT = T>
__global__ void __launch_bounds__(256) cache_write_kernel(
    const T* __restrict__ k, const T* __restrict__ v, KT* __restrict__ kc, KT* __restrict__ vc,
    const long long* __restrict__ slots, int ntok, int nkv, int D, int BS, long long k_stride,
    long long v_stride) {
  const int chunks = D / 8;
  const long long tid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= static_cast<long long>(ntok) * nkv * chunks) return;
  const int c = static_cast<int>(tid % chunks);
  const int h = static_cast<int>((tid / chunks) % nkv);
  const int t = static_cast<int>(tid / (static_cast<long long>(chunks) * nkv));
  const long long slot = slots[t];
  if (slot < 0) return;
  const long long blk = slot / BS, off = slot % BS;
  const size_t dst = ((static_cast<size_t>(blk) * nkv + h) * BS + off) * D + c * 8;
  if constexpr (std::is_same<KT, fp8>::value) {
    float a[8], b[8];
    load8(k + t * k_stride + static_cast<long long>(h) * D + c * 8, a);
    load8(v + t * v_stride + static_cast<long long>(h) * D + c * 8, b);
    store8kv<T, KT>(kc + dst, a);
    store8kv<T, KT>(vc + dst, b);
  } else {
    *reinterpret_cast<uint4*>(kc + dst) =
        *reinterpret_cast<const uint4*>(k + t * k_stride + static_cast<long long>(h) * D + c * 8);
    *reinterpret_cast<uint4*>(vc + dst) =
        *reinterpret_cast<const uint4*>(v + t * v_stride + static_cast<long long>(h) * D + c * 8);
  }
}

// RoPE of the q and k heads of the fused token-major QKV rows AND the paged KV-cache write of
// the rotated k and of v, in one pass (serving: prefill and decode).  Replaces rope_inplace +
// cache_write: at batch-1 decode each of those was a ~5 us launch per layer for a few KB.
// Thread = (token, head of q|k|v, 16-element chunk pair i0 / i0 + D/2).
template <typename T, typename KT = T>
__global__ void __launch_bounds__(256) rope_cache_kernel(
    T* __restrict__ qkv, long long ld, const int* __restrict__ pos,
    const float* __restrict__ cos_t, const float* __restrict__ sin_t, KT* __restrict__ kc,
    KT* __restrict__ vc, const long long* __restrict__ slots, int ntok, int nh, int nkv, int D,
    int BS) {
  const int half = D / 2, chunks = D / 16, H = nh + 2 * nkv;
  const long long tid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= static_cast<long long>(ntok) * H * chunks) return;
  const int c = static_cast<int>(tid % chunks);
  const int h = static_cast<int>((tid / chunks) % H);
  const int t = static_cast<int>(tid / (static_cast<long long>(chunks) * H));
  const int i0 = c * 8;
  T* row = qkv + static_cast<long long>(t) * ld + static_cast<long long>(h) * D;
  const long long slot = slots[t];
  const int hk = h - nh - (h >= nh + nkv ? nkv : 0);  // kv head index for k / v heads
  const size_t dst = slot >= 0 ? ((static_cast<size_t>(slot / BS) * nkv + hk) * BS + slot % BS) * D
                               : 0;
  if (h < nh + nkv) {
    const int p = pos[t];
    float cs[8], sn[8], a[8], b[8], oa[8], ob[8];
    load8(cos_t + static_cast<size_t>(p) * half + i0, cs);
    load8(sin_t + static_cast<size_t>(p) * half + i0, sn);
    load8(row + i0, a);
    load8(row + i0 + half, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // explicit fmas: bit-identical to rope_inplace (kernels/rope.hip), whatever the contraction
      oa[j] = fmaf(a[j], cs[j], -(b[j] * sn[j]));
      ob[j] = fmaf(b[j], cs[j], a[j] * sn[j]);
    }
    store8(row + i0, oa);
    store8(row + i0 + half, ob);
    if (h >= nh && slot >= 0) {
      store8kv<T, KT>(kc + dst + i0, oa);
      store8kv<T, KT>(kc + dst + i0 + half, ob);
    }
  } else if (slot >= 0) {
    if constexpr (std::is_same<KT, fp8>::value) {
      float a[8], b[8];
      load8(row + i0, a);
      load8(row + i0 + half, b);
      store8kv<T, KT>(vc + dst + i0, a);
      store8kv<T, KT>(vc + dst + i0 + half, b);
    } else {
      *reinterpret_cast<uint4*>(vc + dst + i0) = *reinterpret_cast<const uint4*>(row + i0);
      *reinterpret_cast<uint4*>(vc + dst + i0 + half) =
          *reinterpret_cast<const uint4*>(row + i0 + half);
    }
  }
}

// fp8 cache -> 16-bit scratch for the prefill flash-attention kernel (whose LDS-DMA staging
// moves raw 16-bit rows): block b of prefill sequence s (while b * BS < kv_len[s]) is copied,
// converted, to scratch block s * maxb + b; the kernel then reads the scratch through the
// identity table.  grid (nseq, maxb, 2 = K / V), block 256.
template <typename T>
__global__ void __launch_bounds__(256) kv_dequant_kernel(
    const fp8* __restrict__ kc, const fp8* __restrict__ vc, T* __restrict__ ks,
    T* __restrict__ vs, const int* __restrict__ tables, int tstride, const int* __restrict__ kv_lens,
    int maxb, int nkv, int BS, int D) {
  const int s = blockIdx.x, b = blockIdx.y;
  if (b * BS >= kv_lens[s]) return;
  const fp8* src = (blockIdx.z == 0 ? kc : vc) +
                   static_cast<size_t>(tables[static_cast<size_t>(s) * tstride + b]) * nkv * BS * D;
  T* dst = (blockIdx.z == 0 ? ks : vs) + (static_cast<size_t>(s) * maxb + b) * nkv * BS * D;
  const int n8 = nkv * BS * D / 8;
  for (int i = threadIdx.x; i < n8; i += 256) {
    float f[8];
    load8kv<T, fp8>(src + i * 8, f);
    store8(dst + i * 8, f);
  }
}

// The PF kernel's inline-asm K / V loads are invisible to hipcc's register allocator, so a spill
// or copy of a result before its counted wait would read stale data (scripts/tools/
// check_asm_loads.py audits the code object).  The audit passes for D = 128 (every G) and G = 1
// (every D); under the register pressure of D = 32 / 64 / 256 with G > 1 hipcc spills the loaded
// registers right after the issue, so those shapes run the compiler-visible UNI kernel -- and
// the PF form is not even instantiated for them.
template <int D, int G>
constexpr bool pa_pf_ok() { return D == 128 || G == 1; }

template <typename T, int D, int G, typename KT>
static void launch_pa_uni(bool pf, dim3 grid, hipStream_t st, void* out, const void* q,
                          const void* kc, const void* vc, const int* bt, const int* cl, int nh,
                          int qldh, int nkv, int BS, int max_blocks, int max_parts, float scale,
                          float* tm, float* tl, void* to, int PART) {
  if constexpr (pa_pf_ok<D, G>()) {
    if (pf) {
      hipLaunchKernelGGL((pa_decode1_kernel<T, D, G, KT, true, true>), grid, dim3(256), 0, st,
                         (T*)out, (const T*)q, (const KT*)kc, (const KT*)vc, bt, cl, nh, qldh, nkv,
                         BS, max_blocks, max_parts, scale, tm, tl, (float*)to, PART);
      return;
    }
  }
  hipLaunchKernelGGL((pa_decode1_kernel<T, D, G, KT, true>), grid, dim3(256), 0, st, (T*)out,
                     (const T*)q, (const KT*)kc, (const KT*)vc, bt, cl, nh, qldh, nkv, BS,
                     max_blocks, max_parts, scale, tm, tl, (float*)to, PART);
}

template <typename T, int D>
static void launch_pa_g(int G, dim3 grid, size_t smem, hipStream_t st, void* out, const void* q,
                        const void* kc, const void* vc, const int* bt, const int* cl, int nh,
                        int qldh, int nkv, int BS, int max_blocks, int max_parts, float scale,
                        float* tm,
                        float* tl, void* to, int PART, unsigned* cnt, int one_pass, bool fp8kv) {
  // one_pass 2: the uniform-block-id variant where the block size equals the rows per step
  const bool uni = one_pass >= 2 && BS == 256 / (D / 8) && PART % BS == 0;
  const bool pf = uni && one_pass == 3;
#define LUMEN_PA_G(GG)                                                                         \
  if (fp8kv && uni)                                                                             \
    launch_pa_uni<T, D, GG, fp8>(pf, grid, st, out, q, kc, vc, bt, cl, nh, qldh, nkv, BS,        \
                                 max_blocks, max_parts, scale, tm, tl, to, PART);                \
  else if (fp8kv)                                                                               \
    hipLaunchKernelGGL((pa_decode1_kernel<T, D, GG, fp8>), grid, dim3(256), 0, st, (T*)out,     \
                       (const T*)q, (const fp8*)kc, (const fp8*)vc, bt, cl, nh, qldh, nkv, BS,        \
                       max_blocks, max_parts, scale, tm, tl, (float*)to, PART);                 \
  else if (uni)                                                                                 \
    launch_pa_uni<T, D, GG, T>(pf, grid, st, out, q, kc, vc, bt, cl, nh, qldh, nkv, BS,          \
                               max_blocks, max_parts, scale, tm, tl, to, PART);                  \
  else if (one_pass)                                                                            \
    hipLaunchKernelGGL((pa_decode1_kernel<T, D, GG>), grid, dim3(256), 0, st, (T*)out,          \
                       (const T*)q, (const T*)kc, (const T*)vc, bt, cl, nh, qldh, nkv, BS, max_blocks, \
                       max_parts, scale, tm, tl, (float*)to, PART);                             \
  else                                                                                          \
    hipLaunchKernelGGL((pa_decode_kernel<T, D, GG>), grid, dim3(256), smem, st, (T*)out,       \
                       (const T*)q, (const T*)kc, (const T*)vc, bt, cl, nh, qldh, nkv, BS, max_blocks, \
                       max_parts, scale, tm, tl, (float*)to, PART, cnt)
  if (G == 1) LUMEN_PA_G(1);
  else if (G == 2) LUMEN_PA_G(2);
  else if (G == 4) LUMEN_PA_G(4);
  else LUMEN_PA_G(8);
#undef LUMEN_PA_G
}

template <typename T>
static hipError_t launch_pa(void* out, const void* q, const void* kc, const void* vc,
                            const int* bt, const int* cl, int nseq, int nh, int nkv, int D, int BS,
                            int max_blocks, int max_parts, float scale, float* tm, float* tl,
                            void* to, int PART, unsigned* cnt, int one_pass, int fp8kv,
                            int qldh, hipStream_t st) {
  const int G = nh / nkv;
  if (fp8kv && one_pass == 0) one_pass = 1;  // the fp8 cache: single-pass kernels only
  if (G != 1 && G != 2 && G != 4 && G != 8) return hipErrorInvalidValue;
  dim3 grid(nseq, nkv, max_parts);
  const size_t smem = (static_cast<size_t>(G) * PART + 4 * G * D + 2 * G + 8) * sizeof(float);
  if (D == 128) launch_pa_g<T, 128>(G, grid, smem, st, out, q, kc, vc, bt, cl, nh, qldh, nkv, BS, max_blocks, max_parts, scale, tm, tl, to, PART, cnt, one_pass, fp8kv != 0);
  else if (D == 64) launch_pa_g<T, 64>(G, grid, smem, st, out, q, kc, vc, bt, cl, nh, qldh, nkv, BS, max_blocks, max_parts, scale, tm, tl, to, PART, cnt, one_pass, fp8kv != 0);
  else if (D == 256) launch_pa_g<T, 256>(G, grid, smem, st, out, q, kc, vc, bt, cl, nh, qldh, nkv, BS, max_blocks, max_parts, scale, tm, tl, to, PART, cnt, one_pass, fp8kv != 0);
  else if (D == 32) launch_pa_g<T, 32>(G, grid, smem, st, out, q, kc, vc, bt, cl, nh, qldh, nkv, BS, max_blocks, max_parts, scale, tm, tl, to, PART, cnt, one_pass, fp8kv != 0);
  else return hipErrorInvalidValue;
  if (max_parts > 1 && (cnt == nullptr || one_pass)) {  // unfused merge: second kernel
    dim3 g2(nseq, nh), b2(128);
    hipLaunchKernelGGL(pa_reduce_kernel<T>, g2, b2, 0, st, (T*)out, cl, tm, tl,
                       (const float*)to, nh, D, max_parts, PART);
  }
  return hipGetLastError();
}

}  // namespace lumen

extern "C" hipError_t lumen_paged_attention_decode(int dtype, void* out, const void* q,
                                                   const void* kc, const void* vc,
                                                   const int* block_tables,
                                                   const int* context_lens, int nseq, int nh,
                                                   int nkv, int D, int BS, int max_blocks,
                                                   int max_parts, float scale, float* tmp_m,
                                                   float* tmp_l, void* tmp_o, int PART,
                                                   unsigned* counters, int one_pass,
                                                   int fp8kv, int qldh, hipStream_t st) {
  // counters: nullptr = merge split contexts in a second kernel; else >= nseq * nkv zeroed
  // arrival counters (left zeroed again) and the last partition to finish merges in place.
  if (nseq == 0) return hipSuccess;
  // qldh: q row stride in heads (nh for a contiguous [nseq, nh, D] q; the fused qkv row's
  // head count when q is read in place from it)
  if (nh % nkv != 0 || nh / nkv > lumen::kMaxGroup || PART <= 0 || qldh < nh)
    return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::launch_pa<lumen::bf16>(out, q, kc, vc, block_tables, context_lens, nseq, nh,
                                         nkv, D, BS, max_blocks, max_parts, scale, tmp_m, tmp_l,
                                         tmp_o, PART, counters, one_pass, fp8kv, qldh, st);
  if (dtype == lumen::kF16)
    return lumen::launch_pa<lumen::fp16>(out, q, kc, vc, block_tables, context_lens, nseq, nh,
                                         nkv, D, BS, max_blocks, max_parts, scale, tmp_m, tmp_l,
                                         tmp_o, PART, counters, one_pass, fp8kv, qldh, st);
  return hipErrorInvalidValue;
}

extern "C" hipError_t lumen_reshape_and_cache(int dtype, const void* k, const void* v, void* kc,
                                              void* vc, const long long* slots, int ntok, int nkv,
                                              int D, int BS, long long k_stride,
                                              long long v_stride, int fp8kv,
                                              hipStream_t st) {
  if (ntok == 0) return hipSuccess;
  if (D % 8 != 0) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(ntok) * nkv * (D / 8);
  dim3 grid(static_cast<unsigned>((total + 255) / 256)), block(256);
  if (fp8kv && dtype == lumen::kBF16)
    hipLaunchKernelGGL((lumen::cache_write_kernel<lumen::bf16, lumen::fp8>), grid, block, 0, st,
                       (const lumen::bf16*)k, (const lumen::bf16*)v, (lumen::fp8*)kc,
                       (lumen::fp8*)vc, slots, ntok, nkv, D, BS, k_stride, v_stride);
  else if (fp8kv && dtype == lumen::kF16)
    hipLaunchKernelGGL((lumen::cache_write_kernel<lumen::fp16, lumen::fp8>), grid, block, 0, st,
                       (const lumen::fp16*)k, (const lumen::fp16*)v, (lumen::fp8*)kc,
                       (lumen::fp8*)vc, slots, ntok, nkv, D, BS, k_stride, v_stride);
  else if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::cache_write_kernel<lumen::bf16>, grid, block, 0, st,
                       (const lumen::bf16*)k, (const lumen::bf16*)v, (lumen::bf16*)kc,
                       (lumen::bf16*)vc, slots, ntok, nkv, D, BS, k_stride, v_stride);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::cache_write_kernel<lumen::fp16>, grid, block, 0, st,
                       (const lumen::fp16*)k, (const lumen::fp16*)v, (lumen::fp16*)kc,
                       (lumen::fp16*)vc, slots, ntok, nkv, D, BS, k_stride, v_stride);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t lumen_rope_cache(int dtype, void* qkv, long long ld, const int* pos,
                                       const float* cos_t, const float* sin_t, void* kc, void* vc,
                                       const long long* slots, int ntok, int nh, int nkv, int D,
                                       int BS, int fp8kv, hipStream_t st) {
  if (ntok == 0) return hipSuccess;
  if (D % 16 != 0) return hipErrorInvalidValue;
  const long long n = static_cast<long long>(ntok) * (nh + 2 * nkv) * (D / 16);
  dim3 block(256), grid(static_cast<unsigned>((n + 255) / 256));
  if (fp8kv && dtype == lumen::kBF16)
    hipLaunchKernelGGL((lumen::rope_cache_kernel<lumen::bf16, lumen::fp8>), grid, block, 0, st,
                       (lumen::bf16*)qkv, ld, pos, cos_t, sin_t, (lumen::fp8*)kc,
                       (lumen::fp8*)vc, slots, ntok, nh, nkv, D, BS);
  else if (fp8kv && dtype == lumen::kF16)
    hipLaunchKernelGGL((lumen::rope_cache_kernel<lumen::fp16, lumen::fp8>), grid, block, 0, st,
                       (lumen::fp16*)qkv, ld, pos, cos_t, sin_t, (lumen::fp8*)kc,
                       (lumen::fp8*)vc, slots, ntok, nh, nkv, D, BS);
  else if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::rope_cache_kernel<lumen::bf16>, grid, block, 0, st,
                       (lumen::bf16*)qkv, ld, pos, cos_t, sin_t, (lumen::bf16*)kc,
                       (lumen::bf16*)vc, slots, ntok, nh, nkv, D, BS);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::rope_cache_kernel<lumen::fp16>, grid, block, 0, st,
                       (lumen::fp16*)qkv, ld, pos, cos_t, sin_t, (lumen::fp16*)kc,
                       (lumen::fp16*)vc, slots, ntok, nh, nkv, D, BS);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// fp8 cache blocks of the prefill sequences -> 16-bit scratch (see kv_dequant_kernel)
extern "C" hipError_t lumen_kv_dequant(int dtype, const void* kc, const void* vc, void* ks,
                                       void* vs, const int* tables, int tstride,
                                       const int* kv_lens, int nseq, int maxb, int nkv, int BS,
                                       int D, hipStream_t st) {
  if (nseq == 0 || maxb == 0) return hipSuccess;
  if ((nkv * BS * D) % 8) return hipErrorInvalidValue;
  const dim3 grid(nseq, maxb, 2), block(256);
  if (dtype == lumen::kBF16)
    hipLaunchKernelGGL(lumen::kv_dequant_kernel<lumen::bf16>, grid, block, 0, st,
                       (const lumen::fp8*)kc, (const lumen::fp8*)vc, (lumen::bf16*)ks,
                       (lumen::bf16*)vs, tables, tstride, kv_lens, maxb, nkv, BS, D);
  else if (dtype == lumen::kF16)
    hipLaunchKernelGGL(lumen::kv_dequant_kernel<lumen::fp16>, grid, block, 0, st,
                       (const lumen::fp8*)kc, (const lumen::fp8*)vc, (lumen::fp16*)ks,
                       (lumen::fp16*)vs, tables, tstride, kv_lens, maxb, nkv, BS, D);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
