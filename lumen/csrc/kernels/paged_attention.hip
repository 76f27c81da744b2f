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

namespace lumen {

constexpr int kMaxGroup = 8;

template <typename T, int D>
__global__ void __launch_bounds__(256) pa_decode_kernel(
    T* __restrict__ out, const T* __restrict__ q, const T* __restrict__ kc,
    const T* __restrict__ vc, const int* __restrict__ block_tables,
    const int* __restrict__ context_lens, int nh, int nkv, int BS, int max_blocks, int max_parts,
    float scale, float* __restrict__ tmp_m, float* __restrict__ tmp_l, float* __restrict__ tmp_o,
    int PART) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int LPT = D / 8;        // lanes per cache row
  constexpr int RPS = 256 / LPT;    // rows per step
  const int seq = blockIdx.x, kvh = blockIdx.y, part = blockIdx.z;
  const int ctx = context_lens[seq];
  const int start = part * PART;
  if (start >= ctx) return;
  const int end = min(ctx, start + PART);
  const int n = end - start;
  const int g = nh / nkv;
  float* q_s = smem;                  // [g][D]
  float* sc = q_s + kMaxGroup * D;    // [g][PART]
  float* ml = sc + kMaxGroup * PART;  // [2][g]
  float* red = ml + 2 * kMaxGroup;    // [4 waves][g][D]
  const int tid = threadIdx.x;
  for (int i = tid; i < g * D; i += 256) {
    const int h = i / D, d = i % D;
    q_s[i] = to_f32(q[(static_cast<size_t>(seq) * nh + kvh * g + h) * D + d]) * scale;
  }
  __syncthreads();
  const int rsub = tid / LPT, d0 = (tid % LPT) * 8;
  const int* bt = block_tables + static_cast<size_t>(seq) * max_blocks;
  // scores
  // groups of LPT lanes share t, so a group is entirely active or inactive and the xor-shuffle
  // reduction below never mixes groups
  for (int t = start + rsub; t < end; t += RPS) {
    float part_s[kMaxGroup];
    {
      const int blk = bt[t / BS], slot = t % BS;
      const T* kr = kc + ((static_cast<size_t>(blk) * nkv + kvh) * BS + slot) * D + d0;
      float kv[8];
      load8(kr, kv);
#pragma unroll
      for (int h = 0; h < kMaxGroup; ++h) {
        float s = 0.f;
        if (h < g) {
#pragma unroll
          for (int j = 0; j < 8; ++j) s += kv[j] * q_s[h * D + d0 + j];
        }
        part_s[h] = s;
      }
    }
#pragma unroll
    for (int h = 0; h < kMaxGroup; ++h) {
      float s = part_s[h];
#pragma unroll
      for (int o = LPT / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      part_s[h] = s;
    }
    if ((tid % LPT) == 0) {
#pragma unroll
      for (int h = 0; h < kMaxGroup; ++h)
        if (h < g) sc[h * PART + (t - start)] = part_s[h];
    }
  }
  __syncthreads();
  // softmax per head: one wave per head
  const int lane = tid & 63, wid = tid >> 6;
  for (int h = wid; h < g; h += 4) {
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, sc[h * PART + i]);
    m = wave_max(m);
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = __expf(sc[h * PART + i] - m);
      sc[h * PART + i] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) { ml[h] = m; ml[kMaxGroup + h] = l; }
  }
  __syncthreads();
  // P.V
  float acc[kMaxGroup][8];
#pragma unroll
  for (int h = 0; h < kMaxGroup; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  for (int t = start + rsub; t < end; t += RPS) {
    const int blk = bt[t / BS], slot = t % BS;
    const T* vr = vc + ((static_cast<size_t>(blk) * nkv + kvh) * BS + slot) * D + d0;
    float vv[8];
    load8(vr, vv);
#pragma unroll
    for (int h = 0; h < kMaxGroup; ++h) {
      if (h < g) {
        const float p = sc[h * PART + (t - start)];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[h][j] += p * vv[j];
      }
    }
  }
  // reduce the 64/LPT row groups of each wave with shuffles, then the 4 waves through LDS
#pragma unroll
  for (int h = 0; h < kMaxGroup; ++h) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = acc[h][j];
#pragma unroll
      for (int o = LPT; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
      acc[h][j] = a;
    }
  }
  if (lane < LPT) {
#pragma unroll
    for (int h = 0; h < kMaxGroup; ++h) {
      if (h < g) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[(wid * g + h) * D + d0 + j] = acc[h][j];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < g * D; i += 256) {
    float o = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) o += red[r * g * D + i];
    const int h = i / D, d = i % D;
    const int head = kvh * g + h;
    if (max_parts == 1) {
      out[(static_cast<size_t>(seq) * nh + head) * D + d] = from_f32<T>(o / ml[kMaxGroup + h]);
    } else {
      const size_t mi = (static_cast<size_t>(seq) * nh + head) * max_parts + part;
      tmp_o[mi * D + d] = o;
      if (d == 0) { tmp_m[mi] = ml[h]; tmp_l[mi] = ml[kMaxGroup + h]; }
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
template <typename T>
__global__ void __launch_bounds__(256) cache_write_kernel(
    const T* __restrict__ k, const T* __restrict__ v, T* __restrict__ kc, T* __restrict__ vc,
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
  *reinterpret_cast<uint4*>(kc + dst) =
      *reinterpret_cast<const uint4*>(k + t * k_stride + static_cast<long long>(h) * D + c * 8);
  *reinterpret_cast<uint4*>(vc + dst) =
      *reinterpret_cast<const uint4*>(v + t * v_stride + static_cast<long long>(h) * D + c * 8);
}

template <typename T>
static hipError_t launch_pa(void* out, const void* q, const void* kc, const void* vc,
                            const int* bt, const int* cl, int nseq, int nh, int nkv, int D, int BS,
                            int max_blocks, int max_parts, float scale, float* tm, float* tl,
                            void* to, int PART, hipStream_t st) {
  dim3 grid(nseq, nkv, max_parts), block(256);
  const size_t smem = (kMaxGroup * D + kMaxGroup * PART + 2 * kMaxGroup +
                       static_cast<size_t>(4) * (nh / nkv) * D) * sizeof(float);
#define LUMEN_PA(DD)                                                                           \
  hipLaunchKernelGGL((pa_decode_kernel<T, DD>), grid, block, smem, st, (T*)out, (const T*)q,     \
                     (const T*)kc, (const T*)vc, bt, cl, nh, nkv, BS, max_blocks, max_parts, scale, \
                     tm, tl, (float*)to, PART)
  if (D == 128) LUMEN_PA(128);
  else if (D == 64) LUMEN_PA(64);
  else if (D == 256) LUMEN_PA(256);
  else if (D == 32) LUMEN_PA(32);
  else return hipErrorInvalidValue;
#undef LUMEN_PA
  if (max_parts > 1) {
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
                                                   hipStream_t st) {
  if (nseq == 0) return hipSuccess;
  if (nh % nkv != 0 || nh / nkv > lumen::kMaxGroup || PART <= 0) return hipErrorInvalidValue;
  if (dtype == lumen::kBF16)
    return lumen::launch_pa<lumen::bf16>(out, q, kc, vc, block_tables, context_lens, nseq, nh,
                                         nkv, D, BS, max_blocks, max_parts, scale, tmp_m, tmp_l,
                                         tmp_o, PART, st);
  if (dtype == lumen::kF16)
    return lumen::launch_pa<lumen::fp16>(out, q, kc, vc, block_tables, context_lens, nseq, nh,
                                         nkv, D, BS, max_blocks, max_parts, scale, tmp_m, tmp_l,
                                         tmp_o, PART, st);
  return hipErrorInvalidValue;
}

extern "C" hipError_t lumen_reshape_and_cache(int dtype, const void* k, const void* v, void* kc,
                                              void* vc, const long long* slots, int ntok, int nkv,
                                              int D, int BS, long long k_stride,
                                              long long v_stride, int /*unused*/,
                                              hipStream_t st) {
  if (ntok == 0) return hipSuccess;
  if (D % 8 != 0) return hipErrorInvalidValue;
  const long long total = static_cast<long long>(ntok) * nkv * (D / 8);
  dim3 grid(static_cast<unsigned>((total + 255) / 256)), block(256);
  if (dtype == lumen::kBF16)
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
