// Flash attention forward + backward for gfx950, varlen + causal + GQA.
//
// Reference behaviour: torch SDPA inside transformers' Llama attention (the model loaded at
// training/train_baseline.py:122), preceded by a [B,S,H,D] -> [B,H,S,D] transpose of q/k/v and
// followed by the inverse transpose before o_proj.
//
// Here attention reads q/k/v IN PLACE from the fused token-major QKV GEMM output
// [T, (nh + 2 nkv) * D] (head h of q at column h*D, of k at (nh + h)*D, ...) and writes O
// token-major [T, nh*D] = exactly the o_proj input, so the split/transpose copies disappear.
// Sequences are packed back to back (cu_seqlens); the host passes the list of (sequence,
// row-start) tiles, heaviest causal tiles first.
//
// Tiling (D = 128, wave64, MFMA v_mfma_f32_16x16x32_{bf16,f16}):
//  fwd   workgroup = 4 waves x (16*MT) query rows; K/V tiles of 64 keys staged in LDS as
//        "dual-use" images (XOR-swizzled 256-byte rows: conflict-free ds_read_b128 row reads
//        for K^T operands AND ds_read_b64_tr_b16 transposed reads for V operands); online
//        softmax in exp2 domain on the MFMA accumulators; P goes through a small per-wave LDS
//        tile (8-byte writes, transposed reads) to become the A operand of P.V.
//  bwd   two kernels, no atomics: dK/dV per 64-key tile (each wave 16 keys, K and V fragments
//        in registers, loops over query tiles and the GQA group's heads), and dQ per 64-query
//        tile (loops over key tiles); the softmax row statistics come from the forward's LSE
//        and delta = rowsum(dO * O) (preprocess kernel).
#include "common.h"
#include <cstdlib>

namespace lumen {
namespace fa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int D = 128;     // head dim (Llama family)
constexpr int BN = 64;     // keys per tile
constexpr int IMG = BN * D * 2;  // bytes of one [64][128] 16-bit LDS image

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

// ---- LDS image of a [rows][128] 16-bit tile: 256-byte rows, 16-byte chunks XOR-swizzled ----
__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * 256 + ((chunk ^ swz(row)) << 4);
}
// Alternative swizzle (SW = 1) for images read by 16-row ds_read_b128 row reads AND the dK/dV
// kernel's ds_read_b64_tr_b16 reads of rows {32ks + 4g + 0..3}: the default swz maps rows r and
// r + 4 of those reads to the same bank pair (2-way conflict on both kinds: measured
// SQ_LDS_BANK_CONFLICT = 47% of SQ_LDS_IDX_ACTIVE in bwd_dkdv_kernel).  Reversing row bits 0..2
// into chunk bits 3..1 makes both access patterns conflict-free (exhaustive search over linear
// XOR swizzles against the gfx950 lane-group banking model, scripts/probes/fa_bank_model.py).
template <int SW>
__device__ __forceinline__ int swz_t(int row) {
  if constexpr (SW == 0) return swz(row);
  else return ((row & 1) << 3) | ((row & 2) << 1) | ((row & 4) >> 1);
}
__device__ __forceinline__ unsigned lds_off_g(const char* p) {
  return static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(p)));
}
template <int SW>
__device__ __forceinline__ int img_off_t(int row, int chunk) {
  return row * 256 + ((chunk ^ swz_t<SW>(row)) << 4);
}

// stage rows [r0, r0+64) x 128 cols of a token-major matrix (row stride ld elements) into img;
// rows >= rmax are zero-filled.  256 threads x 4 chunks of 16 bytes.
template <typename T>
__device__ __forceinline__ void stage64(char* img, const T* base, long long ld, int r0, int rmax) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + i * 256;
    const int row = idx >> 4, ch = idx & 15;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + row < rmax) v = *reinterpret_cast<const uint4*>(base + (long long)(r0 + row) * ld + ch * 8);
    *reinterpret_cast<uint4*>(img + img_off(row, ch)) = v;
  }
}

// Asynchronous variant: global_load_lds (LDS-DMA, 16 B per lane, no VGPRs) into the same
// swizzled image.  One wave-instruction fills 1 KiB = 4 image rows; wave w issues rows
// [16w, 16w+16) in 4 instructions.  The swizzle moves to the per-lane SOURCE address (the LDS side
// of an LDS-DMA is lane-linear).  Rows >= rmax are clamped to row rmax-1 (finite data; the
// softmax masks those keys).  Completion: the issuing wave's vmcnt, then a barrier.
template <typename T, int SW = 0>
__device__ __forceinline__ void stage64_async(char* img, const T* base, long long ld, int r0,
                                              int rmax) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ swz_t<SW>(row);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    __builtin_amdgcn_global_load_lds(
        (const void*)(base + (long long)gr * ld + ch * 8),
        (__attribute__((address_space(3))) void*)(img + (wid * 4 + i) * 1024), 16, 0, 0);
  }
}

// stage64_async with a wave-uniform 64-bit base (the tile's first row, SGPRs) and 32-bit per-lane
// byte offsets (< 64 rows x ld): the DMA takes the saddr + voffset form, one VGPR per address
// instead of a 64-bit VGPR pair -- fwd32_kernel's eight K / V addresses per tile otherwise pushed
// it over its 256-VGPR budget and spilled them to scratch inside the key loop.
template <typename T>
__device__ __forceinline__ void stage64_async_s(char* img, const T* base, long long ld, int r0,
                                                int rmax) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* tile = reinterpret_cast<const char*>(base + (long long)r0 * ld);
  const int last = rmax - 1 - r0;  // >= 0: callers stage only tiles that start inside the range
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ swz(row);
    const unsigned off = (unsigned)((row < last ? row : last) * (int)ld + ch * 8) * sizeof(T);
    __builtin_amdgcn_global_load_lds(
        (const void*)(tile + off),
        (__attribute__((address_space(3))) void*)(img + (wid * 4 + i) * 1024), 16, 0, 0);
  }
}

// Opaque LDS-DMA: the same global_load_lds as the builtin, as inline asm.  hipcc's wait
// insertion cannot tell an in-flight LDS-DMA into one ping-pong buffer from the ds_reads of the
// other and puts s_waitcnt vmcnt(0) before them (seen after the barrier of every step in the
// dK/dV and dQ-from-dS kernels, with builtin ds_read / ds_read_tr reads); hidden from it, the
// DMA is retired only by the kernels' own counted vmcnt waits.  Extra in-flight operations the
// compiler cannot see only make its own counted waits stricter (counters retire in order).
// M0 = wave-uniform LDS base of the lane-linear destination (+16 B per lane).
__device__ __forceinline__ void dma16_o(const void* g, const char* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_off_g(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(g), "s"(m0) : "memory", "m0");
}
__device__ __forceinline__ void dma4_o(const void* g, const char* lds_wave_base) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(lds_off_g(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
               :: "v"(g), "s"(m0) : "memory", "m0");
}
template <typename T, int SW>
__device__ __forceinline__ void stage64_async_o(char* img, const T* base, long long ld, int r0,
                                                int rmax) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ swz_t<SW>(row);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    dma16_o(base + (long long)gr * ld + ch * 8, img + (wid * 4 + i) * 1024);
  }
}

// 8-wave (512-thread) variant: wave w fills image rows [8w, 8w + 8) in 2 DMA instructions
template <typename T, int SW>
__device__ __forceinline__ void stage64_async8_o(char* img, const T* base, long long ld, int r0,
                                                 int rmax) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wid * 2 + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ swz_t<SW>(row);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    dma16_o(base + (long long)gr * ld + ch * 8, img + (wid * 2 + i) * 1024);
  }
}

// stage64_async for the paged KV cache: row r of the tile is key kv0 + r of the sequence, found
// in block bt[key / bs] at offset key % bs ([block][nkv][bs][D] layout: every (block, kv head)
// is one contiguous bs x D run, so a 64-key tile is 64 / bs contiguous runs).  Same LDS image
// and lane mapping as stage64_async.
template <typename T>
__device__ __forceinline__ void stage64_paged(char* img, const T* cache, int kvh, int nkv,
                                              const int* bt, int bs, int r0, int rmax) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ swz(row);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    const long long blk = bt[gr / bs];
    const T* src = cache + ((blk * nkv + kvh) * bs + gr % bs) * D + ch * 8;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + (wid * 4 + i) * 1024),
        16, 0, 0);
  }
}

// vmcnt waits as the s_waitcnt builtin (gfx9 simm16: vmcnt bits [3:0], expcnt [6:4] = 7,
// lgkmcnt [11:8] = 15 i.e. "don't care"), NOT inline asm: the compiler's wait-insertion pass
// sees the builtin, knows that every LDS-DMA older than the newest N has landed, and does not add
// its own vmcnt(0) in front of the ds_reads of the tile just waited for.
__device__ __forceinline__ void wait_vm_all() { __builtin_amdgcn_s_waitcnt(0xF70); }
__device__ __forceinline__ void wait_vm_8() { __builtin_amdgcn_s_waitcnt(0xF78); }
__device__ __forceinline__ void lds_fence_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 16-byte row read: 8 consecutive columns [8*chunk, 8*chunk+8) of `row`
template <int SW = 0>
__device__ __forceinline__ uint4 row_read(const char* img, int row, int chunk) {
  return *reinterpret_cast<const uint4*>(img + img_off_t<SW>(row, chunk));
}

__device__ __forceinline__ uint2 tr_read_raw(const char* p) {
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(uint2, r);
}

// B operand (k = rows, n = cols) of a 16x16x32 MFMA from an image whose rows are the k axis:
// lane (L = lane&15, g = lane>>4) gets col n0 + L, rows k0 + 8g + 0..7.
__device__ __forceinline__ uint4 tr_read_img(const char* img, int k0, int n0, int lane) {
  const int L = lane & 15, g = lane >> 4;
  const int col = n0 + 4 * (L & 3);
  const int ch = col >> 3, half = (col >> 2) & 1;
  const int r = k0 + 8 * g + (L >> 2);
  const uint2 lo = tr_read_raw(img + img_off(r, ch) + 8 * half);
  const uint2 hi = tr_read_raw(img + img_off(r + 4, ch) + 8 * half);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// Per-wave scratch Y[rows k][cols m] (plain row-major, `cols` 16-bit elements per row): C tiles are
// written transposed with 8-byte stores and read back as A operands (row m, 8 consecutive k).
// Y rows are padded by 4 elements (8 bytes) so the 16 rows of one 8-byte transposed store land on
// distinct banks.
__device__ __forceinline__ uint4 tr_read_y(const char* y, int cols, int k0, int m0, int lane) {
  const int L = lane & 15, g = lane >> 4;
  const int r = k0 + 8 * g + (L >> 2);
  const int c = m0 + 4 * (L & 3);
  const int ld = cols + 4;
  const uint2 lo = tr_read_raw(y + (r * ld + c) * 2);
  const uint2 hi = tr_read_raw(y + ((r + 4) * ld + c) * 2);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// write a 16x16 C tile (lane: col = lane&15, rows 4*(lane>>4)+0..3) transposed into Y at
// Y[k = k0 + col][m = m0 + 4*(lane>>4) .. +3] as one 8-byte store
template <typename T>
__device__ __forceinline__ void y_store(char* y, int cols, int k0, int m0, int lane, float v0,
                                        float v1, float v2, float v3) {
  T t[4] = {from_f32<T>(v0), from_f32<T>(v1), from_f32<T>(v2), from_f32<T>(v3)};
  *reinterpret_cast<uint2*>(y + ((k0 + (lane & 15)) * (cols + 4) + m0 + 4 * (lane >> 4)) * 2) =
      *reinterpret_cast<uint2*>(t);
}

template <typename T>
__device__ __forceinline__ uint4 gload16(const T* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
}

// Row reductions over the 16 lanes that share a 16x16 C-tile row, on the DPP cross-lane path
// (quad_perm xor1, xor2, row_half_mirror, row_mirror): 4 VALU ops instead of 4 LDS-routed
// ds_bpermute shuffles per reduction.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
__device__ __forceinline__ float red16_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp<0x141>(v));  // row_half_mirror
  v = fmaxf(v, dpp<0x140>(v));  // row_mirror
  return v;
}
__device__ __forceinline__ float red16_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}

// exp2 on the transcendental unit directly (v_exp_f32): the libm exp2f adds a denormal range
// fix-up (v_cmp + v_cndmask + v_ldexp per call) that a softmax does not need -- every input is
// <= 0 and results below 2^-126 are flushed to 0, far beneath bf16 resolution of the row sum.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

struct Args {
  const void* q; const void* k; const void* v;  // token-major bases (head 0)
  long long ldq, ldk, ldv;
  void* o; long long ldo;
  float* lse;                                     // [nh][T] (log2 domain)
  const int* cu;                                  // [nseq + 1]
  const int* tiles;                               // [ntiles][2] = (seq, row start)
  int nh, nkv, T;
  float scale, scale_log2;
  // backward
  const void* dout; long long lddo;
  void* dq; void* dk; void* dv; long long lddq, lddk, lddv;
  const float* delta;                             // [nh][T]
  // optional (backward dQ / dK epilogues): undo the rotary embedding the forward applied to q / k
  // -- write d(pre-RoPE) directly, so no separate inverse-rotation pass over dQKV is needed.
  // rope_pos [T] (token positions), rope_cos / rope_sin [max_pos][64]; nullptr = off
  const int* rope_pos;
  const float* rope_cos;
  const float* rope_sin;
  // optional (forward, PAGED): keys / values come from the serving KV cache
  // [num_blocks][nkv][block_size][D] (k / v point at the caches) through per-sequence block
  // tables; kv_lens[seq] = keys visible to the sequence (cached context + this chunk), and the
  // chunk's queries sit at positions kv_lens - q_len .. kv_lens - 1 (chunked / mixed prefill)
  const int* kv_lens;
  const int* block_tables;
  int bt_stride;
  int block_size;
  // optional (backward, dS hand-off): the dK/dV kernel stores dS (16-bit, the exact operand it
  // feeds its own dK product) per 64 x 64 (query tile, key tile) into ds; the dQ kernel then
  // forms dQ = dS K from it instead of recomputing S and dP.  Tile (head, seq, qt, kt) is
  // ds + (head * ds_total + ds_off[seq] + tri(qt, kt)) * 8 KiB, tri = qt(qt+1)/2 + kt (causal)
  // or qt * ntiles(seq) + kt.
  void* ds;
  const int* ds_off;
  int ds_total;
  // tiles3: 1-D grid over (seq, row start, head) triples (head = the kernel's head or kv head),
  // ordered on the host so that the tiles of one (sequence, head) land on one XCD together and
  // share its L2 (blocks go to XCDs round-robin by id; seq < 0 = padding); 0: pairs, head = y
  int tiles3;
  int nitems;  // > 0: persistent dK/dV launch over nitems = ntiles * nkv items (1-D grid)
  int snake;   // persistent item order: 1 snake rounds, 0 plain strided
};

struct Work { int seq, r0, head; };
__device__ __forceinline__ Work work_item(const Args& a) {
  if (a.tiles3) {
    const int* t = a.tiles + 3 * blockIdx.x;
    return Work{t[0], t[1], t[2]};
  }
  return Work{a.tiles[2 * blockIdx.x], a.tiles[2 * blockIdx.x + 1], (int)blockIdx.y};
}

// Inverse rotary embedding of one (x, x ^ 64) column pair: the forward rotation
// y1 = x1 c - x2 s, y2 = x2 c + x1 s has the transpose dx1 = dy1 c + dy2 s, dx2 = dy2 c - dy1 s.
__device__ __forceinline__ void rope_inv_pair(float& lo, float& hi, float c, float s) {
  const float l = lo, h = hi;
  lo = l * c + h * s;
  hi = h * c - l * s;
}

// V^T operand rows for the permuted key order (the dK/dV kernel): lane (L, g) gets column
// n0 + L of rows rlo + 0..3 (lo) and rhi + 0..3 (hi)
template <int SW = 0>
__device__ __forceinline__ uint4 tr_read_img2(const char* img, int rlo, int rhi, int n0, int lane) {
  const int L = lane & 15;
  const int col = n0 + 4 * (L & 3);
  const int ch = col >> 3, half = (col >> 2) & 1;
  const uint2 lo = tr_read_raw(img + img_off_t<SW>(rlo + (L >> 2), ch) + 8 * half);
  const uint2 hi = tr_read_raw(img + img_off_t<SW>(rhi + (L >> 2), ch) + 8 * half);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

template <typename T>
__device__ __forceinline__ uint4 pack_p(const f32x4& a, const f32x4& b) {
  return make_uint4(pk2<T>(a[0], a[1]), pk2<T>(a[2], a[3]), pk2<T>(b[0], b[1]), pk2<T>(b[2], b[3]));
}

// =============================================================================================
// backward: delta = rowsum(dO * O)
// =============================================================================================
// One wave per token row: lane l reads the 16-byte chunks l*8 + 512*i (coalesced 1 KiB per
// instruction); with D = 128 the 16 lanes of a row-group share one head per i, so a 16-lane
// butterfly finishes each head's sum.
template <typename T>
__global__ void __launch_bounds__(256) delta_kernel(Args a) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= a.T) return;
  const int H = a.nh * D;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (long long)t * a.lddo;
  const T* O = reinterpret_cast<const T*>(a.o) + (long long)t * a.ldo;
  for (int base = 0; base < H; base += 512) {
    const int e = base + lane * 8;
    float s = 0.f;
    if (e < H) {
      float x[8], y[8];
      load8(dO + e, x);
      load8(O + e, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[j] * y[j];
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 16);
    if ((lane & 15) == 0 && e < H) const_cast<float*>(a.delta)[(long long)(e / D) * a.T + t] = s;
  }
}

// =============================================================================================
// backward: dK, dV  (workgroup = 64 keys of one kv head; loops over q tiles and group heads)
// =============================================================================================
// dS hand-off layout inside one 8 KiB tile: block (wave w = key / 16, ks = query / 32) of 1 KiB
// holds 64 lanes' packed 16-byte P^T-order registers (queries 4m..4m+3 | 16+4m..16+4m+3 of the
// 32-query slice for key row lr) at slot m * 16 + (lr ^ 8 (m & 1)): the dK/dV kernel stores one
// coalesced KiB per instruction, and the dQ kernel's 8-byte transposed reads of one half are at
// most 2-way bank-conflicted (4 of its 36 LDS reads per key tile).
__device__ __forceinline__ int ds_slot(int m, int lr) { return (m * 16 + (lr ^ ((m & 1) << 3))) * 16; }
// seq_base = ds_off[seq], loaded once before the DMA ring starts (a load of it inside the loop
// would make the compiler drain every LDS-DMA in flight with vmcnt(0) before using it)
__device__ __forceinline__ long long ds_tile(const Args& a, int head, int seq_base, int qt, int kt,
                                             int ns, bool causal) {
  return ((long long)head * a.ds_total + seq_base + (causal ? qt * (qt + 1) / 2 + kt : qt * ns + kt)) * 8192;
}

template <typename T, bool CAUSAL, bool WDS = false>
__global__ void __launch_bounds__(256, 2) bwd_dkdv_kernel(Args a) {
  constexpr int STAGE = 2 * IMG + 512;  // Q image | dO image | lse[64] | delta[64]
  // two stages filled by LDS-DMA one (head, q-tile) step ahead.  S = Q K^T and dP = dO V^T are
  // computed with the queries as MFMA rows, so the accumulator lane (key L, queries 4g + r of each
  // 16-query tile) already holds P^T / dS^T rows in the permuted-k order of the fwd_t kernel:
  // they feed dV += P^T dO and dK += dS^T Q straight from registers (no LDS round trip).
  // two SEPARATE LDS objects, the loop unrolled by two (see fwd32_kernel): with one array indexed
  // by (j & 1) the compiler put s_waitcnt vmcnt(0) after the barrier of every step (it could not
  // tell the in-flight prefetch from the tile being read), serialising the DMA ring
  __shared__ __attribute__((aligned(16))) char bufA[STAGE];
  __shared__ __attribute__((aligned(16))) char bufB[STAGE];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  // persistent (a.nitems > 0): a grid of ~2 workgroups per CU walks the (key tile, kv head)
  // items in the host's heaviest-first order.  One workgroup's dK/dV stores (and dS flush) are
  // then still draining while its next item's K / V fragments and first Q / dO stage load,
  // instead of the workgroup slot idling on both latencies (prologue + epilogue alone measured
  // 35 us of a ~110 us call as one-shot workgroups, probe 128)
  auto run = [&](const int seq, const int k0, const int kvh) {
  const int grp = a.nh / a.nkv;
  const int s0 = a.cu[seq], L = a.cu[seq + 1] - s0;
  const T* K = reinterpret_cast<const T*>(a.k) + (long long)s0 * a.ldk + kvh * D;
  const T* V = reinterpret_cast<const T*>(a.v) + (long long)s0 * a.ldv + kvh * D;
  const int wk0 = k0 + wid * 16;  // this wave's 16 keys
  const int krow = wk0 + lr;      // the key of this lane's accumulator column
  const int qstart = CAUSAL ? (k0 / 64) * 64 : 0;
  const int nq = qstart < L ? (L - qstart + 63) / 64 : 0;
  const int nsteps = grp * nq;  // (group head, query tile) pairs
  // stage step j: Q / dO tiles via 8 DMA instructions per wave, lse / delta via one 4-byte DMA
  // instruction on waves 0 / 1 (the DMA ring stays the only in-loop global traffic, so the
  // counted vmcnt waits below stay exact: every wave keeps the same count per step, waves 0/1
  // issue one more, waited with vmcnt(0) on the last step only)
  auto stage = [&](int j, char* st) {
    const int hh = j / nq, q0 = qstart + (j % nq) * 64;
    const int head = kvh * grp + hh;
    stage64_async_o<T, 1>(st, reinterpret_cast<const T*>(a.q) + (long long)s0 * a.ldq + head * D, a.ldq,
                  q0, L);
    stage64_async_o<T, 1>(st + IMG, reinterpret_cast<const T*>(a.dout) + (long long)s0 * a.lddo + head * D,
                  a.lddo, q0, L);
    if (wid < 2) {
      const float* src = (wid == 0 ? a.lse : a.delta) + (long long)head * a.T + s0;
      int qr = q0 + lane;
      qr = qr < L ? qr : L - 1;
      dma4_o(src + qr, st + 2 * IMG + wid * 256);
    }
  };
  // WDS: step j's dS is held in registers and stored right after step j+1's wait, so the stores
  // are older than step j+2's DMA and retire under step j+1's compute: the counted vmcnt waits
  // stay exact and no step waits for a store it just issued
  uint4 pend[2];
  long long pend_off = -1;
  auto store_pend = [&]() {
    if (pend_off < 0) return;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      char* dst = reinterpret_cast<char*>(a.ds) + pend_off + (wid * 2 + ks) * 1024 + ds_slot(lg, lr);
      *reinterpret_cast<uint4*>(dst) = pend[ks];
    }
  };
  // stage 0's DMA and this wave's K / V fragment loads are in flight together (one latency,
  // not two, before the first step); the full drain below retires both
  if (nsteps > 0) stage(0, bufA);
  uint4 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = gload16(K + (long long)krow * a.ldk + (4 * ks + lg) * 8, krow < L);
    vf[ks] = gload16(V + (long long)krow * a.ldv + (4 * ks + lg) * 8, krow < L);
  }
  const int ds_base = WDS ? a.ds_off[seq] : 0;
  wait_vm_all();
  f32x4 dk[8], dv[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) { dk[n] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[n] = dk[n]; }
  auto step = [&](int j, char* st, char* nx) {
    char* qimg = st;
    char* oimg = st + IMG;
    const float* s_lse = reinterpret_cast<const float*>(st + 2 * IMG);
    const float* s_del = s_lse + 64;
    const int q0 = qstart + (j % nq) * 64;
    if (j + 1 < nsteps) {
      stage(j + 1, nx);
      if (wid < 2) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      wait_vm_all();
    }
    lds_fence_barrier();
    if constexpr (WDS) store_pend();
    // S = Q K^T and dP = dO V^T: [64 queries x 16 keys] per wave as 4 query tiles
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) { sc[nt] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[nt] = sc[nt]; }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        sc[nt] = Mfma<T>::run(row_read<1>(qimg, nt * 16 + lr, 4 * ks + lg), kf[ks], sc[nt]);
        dp[nt] = Mfma<T>::run(row_read<1>(oimg, nt * 16 + lr, 4 * ks + lg), vf[ks], dp[nt]);
      }
    }
    // lane: key krow, queries q0 + 16nt + 4lg + r
    // (WDS: keys past the end must also store dS = 0 -- dQ multiplies it by the clamped K rows;
    // without the hand-off those keys' dK / dV rows are simply never written)
    // wave-uniform (readfirstlane: an SGPR, so ONE scalar branch picks the masked or the plain
    // copy below); a per-element `if (need_mask && ...)` compiled to exec-mask save / branch /
    // restore around every element, ~200 scalar instructions per step on unmasked tiles
    const int need_mask = __builtin_amdgcn_readfirstlane(
        ((q0 + 64 > L) || (CAUSAL && wk0 + 15 > q0) || (WDS && k0 + 64 > L)) ? 1 : 0);
    float lq[4][4], dq4[4][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float4 l4 = *reinterpret_cast<const float4*>(s_lse + nt * 16 + 4 * lg);
      const float4 d4 = *reinterpret_cast<const float4*>(s_del + nt * 16 + 4 * lg);
      lq[nt][0] = l4.x; lq[nt][1] = l4.y; lq[nt][2] = l4.z; lq[nt][3] = l4.w;
      dq4[nt][0] = d4.x; dq4[nt][1] = d4.y; dq4[nt][2] = d4.z; dq4[nt][3] = d4.w;
    }
    if (need_mask) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qc = nt * 16 + 4 * lg + r;
          const bool out = (krow >= L) | (q0 + qc >= L) | (CAUSAL & (krow > q0 + qc));
          const float pv = out ? 0.f : fexp2(sc[nt][r] * a.scale_log2 - lq[nt][r]);
          sc[nt][r] = pv;
          dp[nt][r] = pv * (dp[nt][r] - dq4[nt][r]);
        }
    } else {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fexp2(sc[nt][r] * a.scale_log2 - lq[nt][r]);
          sc[nt][r] = pv;
          dp[nt][r] = pv * (dp[nt][r] - dq4[nt][r]);
        }
    }
    // dV += P^T dO ; dK += dS^T Q   (k = queries in the permuted order)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint4 pa = pack_p<T>(sc[2 * ks], sc[2 * ks + 1]);
      const uint4 da = pack_p<T>(dp[2 * ks], dp[2 * ks + 1]);
      if constexpr (WDS) pend[ks] = da;
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        dv[n] = Mfma<T>::run(pa, tr_read_img2<1>(oimg, 32 * ks + 4 * lg, 32 * ks + 16 + 4 * lg, n * 16, lane), dv[n]);
        dk[n] = Mfma<T>::run(da, tr_read_img2<1>(qimg, 32 * ks + 4 * lg, 32 * ks + 16 + 4 * lg, n * 16, lane), dk[n]);
      }
    }
    if constexpr (WDS)
      pend_off = ds_tile(a, kvh * grp + j / nq, ds_base, q0 / 64, k0 / 64, (L + 63) / 64, CAUSAL);
    lds_fence_barrier();  // stage buffer free for the DMA two steps ahead
  };
  for (int j = 0; j < nsteps; j += 2) {
    step(j, bufA, bufB);
    if (j + 1 < nsteps) step(j + 1, bufB, bufA);
  }
  if constexpr (WDS) store_pend();
  // write dK (x softmax scale), dV : rows wk0 + 4lg + r, cols 16n + lr.  (Staging these tiles
  // through LDS for whole-row stores, as the forward's O, measured slower here and in the dQ
  // kernel: 88.9 -> 92.8 us and 32.6 -> 33.7 us, profiles/r3d/fa)
  T* dK = reinterpret_cast<T*>(a.dk) + (long long)s0 * a.lddk + kvh * D;
  T* dV = reinterpret_cast<T*>(a.dv) + (long long)s0 * a.lddv + kvh * D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kr = wk0 + 4 * lg + r;
    if (kr >= L) continue;
    float kv[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) kv[n] = dk[n][r] * a.scale;
    if (a.rope_pos != nullptr) {  // column 16n + lr pairs with 16(n + 4) + lr: same lane
      const long long pb = (long long)a.rope_pos[s0 + kr] * 64 + lr;
#pragma unroll
      for (int n = 0; n < 4; ++n)
        rope_inv_pair(kv[n], kv[n + 4], a.rope_cos[pb + 16 * n], a.rope_sin[pb + 16 * n]);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      dK[(long long)kr * a.lddk + n * 16 + lr] = from_f32<T>(kv[n]);
      dV[(long long)kr * a.lddv + n * 16 + lr] = from_f32<T>(dv[n][r]);
    }
  }
  };
  if (a.nitems > 0) {
    // snake order over the heaviest-first item list: round r takes items r*G + w (even r) or
    // r*G + G-1-w (odd r), pairing heavy with light items per workgroup (static balance)
    const int G = gridDim.x, w = blockIdx.x;
    for (int base = 0; base < a.nitems; base += G) {
      const int it = (a.snake && ((base / G) & 1)) ? base + G - 1 - w : base + w;
      if (it >= a.nitems) continue;
      const int ti = it / a.nkv;
      run(a.tiles[2 * ti], a.tiles[2 * ti + 1], it - ti * a.nkv);
    }
  } else {
    const Work wk = work_item(a);
    if (wk.seq < 0) return;
    run(wk.seq, wk.r0, wk.head);
  }
}

// =============================================================================================
// 32x32x16 MFMA kernels (v_mfma_f32_32x32x16_{bf16,f16}): 32 queries (fwd, dQ) or 32 keys
// (dK/dV) per wave, 4 waves per workgroup.  Same swizzled K/V/Q/dO LDS images as above; every
// B fragment read from LDS now feeds a 32x32x16 product (32 KFLOP) instead of a 16x16x32 one
// (16 KFLOP), so the LDS traffic per FLOP halves.  Accumulator layout (verified by
// scripts/probes/mfma32_layout.hip): lane l, register r = 4j + i holds row 8j + 4(l>>5) + i,
// column l & 31; A/B lanes hold k = 8(l>>5) + 0..7.  With keys (or queries) on the accumulator
// ROWS, the registers 8s..8s+7 of a 32-row block are rows {16s + 4hi + 0..3, 16s + 8 + 4hi +
// 0..3} (hi = l>>5): read the other operand's rows in that order and P / dS feed the next
// product straight from registers.
// =============================================================================================
typedef float f32x16 __attribute__((ext_vector_type(16)));

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

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// 8 rows of an image, transposed, for a 32x32x16 operand whose k slots follow the register
// order above: lane (c = lane&31, hi) gets column n0 + c of rows r0 + 4hi + 0..3 and
// r0 + 8 + 4hi + 0..3 (each 16-lane group reads its own 16 columns).
__device__ __forceinline__ uint4 tr_read32(const char* img, int r0, int n0, int lane) {
  const int hi = lane >> 5;
  return tr_read_img2(img, r0 + 4 * hi, r0 + 8 + 4 * hi, n0 + 16 * ((lane >> 4) & 1), lane);
}

// registers 8s..8s+7 of a 32x32 accumulator -> 8 packed 16-bit values (a k=16 operand)
template <typename T>
__device__ __forceinline__ uint4 pack8(const f32x16& c, int s) {
  return make_uint4(pk2<T>(c[8 * s], c[8 * s + 1]), pk2<T>(c[8 * s + 2], c[8 * s + 3]),
                    pk2<T>(c[8 * s + 4], c[8 * s + 5]), pk2<T>(c[8 * s + 6], c[8 * s + 7]));
}

// ---- forward: S^T = K Q^T (keys on rows, lane = query), O^T += V^T P^T -----------------------
// Per-lane LDS byte offsets inside a K/V image, computed once: the swizzle depends only on
// row & 15, so the key block (kb * 32 rows) and the 16-key slice (16 rows) are immediates.
struct Off32 {
  int row[8];   // row_read of row (lane&31), chunk 2ks + hi        (ks = 0..7)
  int tr[8];    // tr_read32 lo / hi rows for output block n      (index 2n + lohi)
};
__device__ __forceinline__ void make_off32(Off32& o, int lane) {
  const int lq = lane & 31, hi = lane >> 5, L = lane & 15, g16 = (lane >> 4) & 1;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) o.row[ks] = img_off(lq, 2 * ks + hi);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int ch = 4 * n + 2 * g16 + ((L & 3) >> 1);
    const int r = 4 * hi + (L >> 2);
    o.tr[2 * n] = img_off(r, ch) + 8 * (L & 1);
    o.tr[2 * n + 1] = img_off(r + 8, ch) + 8 * (L & 1);
  }
}
__device__ __forceinline__ uint4 lds16(const char* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint4 tr32(const char* img, const Off32& o, int rowbase, int n) {
  const uint2 lo = tr_read_raw(img + rowbase * 256 + o.tr[2 * n]);
  const uint2 hi = tr_read_raw(img + rowbase * 256 + o.tr[2 * n + 1]);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// LDS reads as inline asm.  The compiler's wait insertion cannot tell that the LDS-DMA prefetch
// in flight targets the OTHER ping-pong buffer, so before any plain ds_read of the current tile
// it emits s_waitcnt vmcnt(0) -- waiting for the prefetch it was meant to overlap (seen in the
// ISA of every kernel in this file).  Inline asm is opaque to that pass; the tile code waits for
// its own reads with lgkm_wait(), whose register operands order every consumer after it.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned lds_off(const char* p) {
  return static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)(p)));
}
template <int OFF>
__device__ __forceinline__ u32x4v ds_b128(unsigned a) {
  u32x4v r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ u32x2v ds_tr64(unsigned a) {
  u32x2v r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
__device__ __forceinline__ void lgkm_wait(u32x4v& a, u32x4v& b, u32x4v& c, u32x4v& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ uint4 as_u4(u32x4v v) { return __builtin_bit_cast(uint4, v); }
// V^T / K^T operand of the 32x32x16 products (tr32 above) for key block rowbase = 16 * RB
template <int RB>
__device__ __forceinline__ u32x4v tr32a(unsigned img, const Off32& o, int n) {
  const u32x2v lo = ds_tr64<RB * 16 * 256>(img + o.tr[2 * n]);
  const u32x2v hi = ds_tr64<RB * 16 * 256>(img + o.tr[2 * n + 1]);
  return u32x4v{lo.x, lo.y, hi.x, hi.y};
}

// xor-32 lane exchange on the VALU (v_permlane32_swap, gfx950) instead of ds_bpermute through
// LDS: both operands must be distinct registers holding the value (the builtin, given the same
// value twice, gets them coalesced into one register and returns the lane's own value;
// scripts/probes/permlane_probe.hip).
__device__ __forceinline__ void xor32_pair(float v, float& a, float& b) {
  unsigned x = __builtin_bit_cast(unsigned, v), y = x;
  // s_nop padding: inline asm is invisible to the compiler's hazard recognizer, and the swap
  // reads VGPRs a VALU just wrote (and its results feed the next VALU)
  asm volatile("s_nop 4\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 4" : "+v"(x), "+v"(y));
  a = __builtin_bit_cast(float, x);
  b = __builtin_bit_cast(float, y);
}
__device__ __forceinline__ float xor32_max(float v) {
  float a, b;
  xor32_pair(v, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float xor32_sum(float v) {
  float a, b;
  xor32_pair(v, a, b);
  return a + b;
}

template <typename T, bool CAUSAL, bool MASK>
__device__ __forceinline__ void fwd32_tile(const char* kimg, const char* vimg, const Off32& off,
                                           const uint4 (&qf)[8], f32x16 (&acc)[4], float& m_i,
                                           float& l_i, int kv0, int L, int qrow, int hi,
                                           float scale_log2) {
  f32x16 st[2];
  st[0] = zero16();
  st[1] = zero16();
  {
    const unsigned kb0 = lds_off(kimg);
    u32x4v kr[2][8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      kr[0][ks] = ds_b128<0>(kb0 + off.row[ks]);
      kr[1][ks] = ds_b128<8192>(kb0 + off.row[ks]);
    }
    lgkm_wait(kr[0][0], kr[0][1], kr[0][2], kr[0][3]);
    lgkm_wait(kr[0][4], kr[0][5], kr[0][6], kr[0][7]);
    lgkm_wait(kr[1][0], kr[1][1], kr[1][2], kr[1][3]);
    lgkm_wait(kr[1][4], kr[1][5], kr[1][6], kr[1][7]);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) st[kb] = Mfma32<T>::run(as_u4(kr[kb][ks]), qf[ks], st[kb]);
    }
  }
  // V^T operands for the P V product, read while the S MFMAs drain and the softmax runs (they
  // take the K fragments' registers): the 32 transposed LDS reads' latency leaves the PV phase
  const unsigned vb = lds_off(vimg);
  u32x4v vr[4][4];  // [16-key slice kb * 2 + s][output block n]
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    vr[0][n] = tr32a<0>(vb, off, n);
    vr[1][n] = tr32a<1>(vb, off, n);
    vr[2][n] = tr32a<2>(vb, off, n);
    vr[3][n] = tr32a<3>(vb, off, n);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MASK) {
        const int kpos = kv0 + kb * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
        const bool out = (kpos >= L) | (CAUSAL & (kpos > qrow));
        st[kb][r] = out ? -INFINITY : st[kb][r];
      }
      mx = fmaxf(mx, st[kb][r]);
    }
  mx = xor32_max(mx) * scale_log2;
  // deferred rescale: the running max moves only when a row's new max exceeds it by more than
  // RESCALE (log2 units), so P stays <= 2^RESCALE and the O / l rescale (64 multiplies per lane)
  // runs on a handful of tiles per row instead of every tile
  constexpr float RESCALE = 8.f;
  const bool bump = mx > m_i + RESCALE;
  if (__any(bump)) {
    // lanes that do not move keep alpha = 1 (also when their m_i is still -inf: -inf - -inf)
    const float alpha = bump ? fexp2(m_i - mx) : 1.f;  // exp2(-inf) = 0 on a row's first tile
    const float m_new = bump ? mx : m_i;
    l_i *= alpha;
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] *= alpha;
    m_i = m_new;
  }
  const float mref = m_i == -INFINITY ? 0.f : m_i;
  float rs = 0.f;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = fexp2(fmaf(st[kb][r], scale_log2, -mref));
      st[kb][r] = p;
      rs += p;
    }
  l_i += xor32_sum(rs);
  // O^T[d][q] += V^T[d][key] P^T[key][q], keys in the register order
  const uint4 pb[4] = {pack8<T>(st[0], 0), pack8<T>(st[0], 1), pack8<T>(st[1], 0),
                       pack8<T>(st[1], 1)};
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    lgkm_wait(vr[sl][0], vr[sl][1], vr[sl][2], vr[sl][3]);
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = Mfma32<T>::run(as_u4(vr[sl][n]), pb[sl], acc[n]);
  }
}

// (Cost-split probe builds of this kernel -- key loop without the tile math, without the K / V
// loads, no key loop, no softmax -- produced profiles/r5_fa and were removed afterwards.)
template <typename T, bool CAUSAL, bool PAGED = false>
__global__ void __launch_bounds__(256, CAUSAL ? 2 : 1) fwd32_kernel(Args a) {
  constexpr int BM = 128;
  // Two SEPARATE LDS objects for the ping-pong K|V buffers, with the loop unrolled by two so
  // every LDS-DMA and every ds_read names its buffer statically: the compiler's wait insertion
  // tracks LDS-DMA per LDS object, and with one array indexed by (it & 1) it had to assume the
  // in-flight prefetch aliases the tile being read and put an s_waitcnt vmcnt(0) in front of the
  // first ds_read -- which serialised every prefetch against the compute it was meant to hide.
  __shared__ __attribute__((aligned(16))) char bufA[2 * IMG];  // [K | V]
  __shared__ __attribute__((aligned(16))) char bufB[2 * IMG];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lq = lane & 31, hi = lane >> 5;
  // persistent (a.nitems > 0, as bwd_dkdv_kernel): the workgroups walk the (query tile, head)
  // items, so one item's O / LSE stores drain under the next item's Q loads and first K / V DMA
  auto run = [&](const int seq, const int q0, const int head) {
  const int kvh = head / (a.nh / a.nkv);
  const int s0 = a.cu[seq], L = a.cu[seq + 1] - s0;  // L = this sequence's query rows
  // keys: self-attention over the same rows, or (PAGED) the cached context + this chunk, the
  // chunk's queries sitting at key positions qoff .. qoff + L - 1
  const int Lk = PAGED ? a.kv_lens[seq] : L;
  const int qoff = Lk - L;
  const T* Q = reinterpret_cast<const T*>(a.q) + (long long)s0 * a.ldq + head * D;
  const T* K = reinterpret_cast<const T*>(a.k) + (PAGED ? 0 : (long long)s0 * a.ldk + kvh * D);
  const T* V = reinterpret_cast<const T*>(a.v) + (PAGED ? 0 : (long long)s0 * a.ldv + kvh * D);
  const int* bt = PAGED ? a.block_tables + (long long)seq * a.bt_stride : nullptr;
  const int wq0 = q0 + wid * 32;
  const int qrow = wq0 + lq;
  const int qpos = qrow + qoff;  // key position of this lane's query (causal limit)
  Off32 off;
  make_off32(off, lane);
  f32x16 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = zero16();
  float m_i = -INFINITY, l_i = 0.f;
  const int kv_end = CAUSAL ? min(Lk, q0 + qoff + BM) : Lk;
  const int w_end = CAUSAL ? min(kv_end, wq0 + qoff + 32) : kv_end;  // keys this wave can see
  auto stage = [&](char* img, int r0) {
    if constexpr (PAGED) {
      stage64_paged(img, K, kvh, a.nkv, bt, a.block_size, r0, Lk);
      stage64_paged(img + IMG, V, kvh, a.nkv, bt, a.block_size, r0, Lk);
    } else {
      stage64_async_s(img, K, a.ldk, r0, L);
      stage64_async_s(img + IMG, V, a.ldv, r0, L);
    }
  };
  // Q tile by LDS-DMA into bufB (free until the first tile prefetches into it), in flight
  // together with the first K / V tile: one memory round trip before the key loop instead of
  // two, and whole 256-byte rows per wave-instruction instead of 32 strided 16-byte pieces.
  // Rows >= L are clamped duplicates (their outputs are never stored).
  uint4 qf[8];  // B operand of S^T: Q[qrow][16ks + 8hi .. +7]
  {
    const bool two = q0 + 64 < L;
    stage64_async_s(bufB, Q, a.ldq, q0, L);
    if (two) stage64_async_s(bufB + IMG, Q, a.ldq, q0 + 64, L);
    if (kv_end > 0) {
      stage(bufA, 0);
      wait_vm_8();  // this wave's Q pieces landed (the newest 8 are the K / V tile)
    } else {
      wait_vm_all();
    }
    __builtin_amdgcn_s_barrier();  // every wave's Q pieces landed
    asm volatile("" ::: "memory");
    const int r = 32 * wid + lq;   // row of the 128-row Q block
    const char* qi = bufB + (r >> 6) * IMG;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = row_read(qi, r & 63, 2 * ks + hi);
    lds_fence_barrier();  // bufB is the first prefetch target
  }
  // one K/V tile: prefetch the next into `nxt`, wait for `cur`, compute, release `cur`
  auto tile = [&](char* cur, char* nxt, int kv0) {
    if (kv0 + BN < kv_end) {
      stage(nxt, kv0 + BN);
      wait_vm_8();
    } else {
      wait_vm_all();
    }
    lds_fence_barrier();
    if (kv0 < w_end) {  // (causal: tiles entirely above this wave's rows are skipped)
      const bool need_mask = (kv0 + BN > Lk) || (CAUSAL && kv0 + BN - 1 > wq0 + qoff);
      if (need_mask)
        fwd32_tile<T, CAUSAL, true>(cur, cur + IMG, off, qf, acc, m_i, l_i, kv0, Lk, qpos,
                                           hi, a.scale_log2);
      else
        fwd32_tile<T, CAUSAL, false>(cur, cur + IMG, off, qf, acc, m_i, l_i, kv0, Lk, qpos,
                                            hi, a.scale_log2);
    }
    lds_fence_barrier();  // every wave is done with `cur` before it is refilled
  };
  for (int kv0 = 0; kv0 < kv_end; kv0 += 2 * BN) {
    tile(bufA, bufB, kv0);
    if (kv0 + BN < kv_end) tile(bufB, bufA, kv0 + BN);
  }
  // epilogue: lane holds O[qrow][32n + 8j + 4hi + i] in acc[n][4j + i].  The wave's 32 x 128
  // tile goes through LDS (bufA is free after the loop's last barrier; wave w owns 8 KiB of it)
  // and leaves as whole 256-byte rows: 8 wave-instructions of 4 rows each instead of 16 per-lane
  // 8-byte stores that touch 32 rows apiece.
  {
    // lane index made opaque here: the tile addresses below must not be hoisted above the key
    // loop (they would stay live across it and push it over the 256-VGPR budget)
    int ln = threadIdx.x;
    asm volatile("" : "+v"(ln));
    const int lq2 = ln & 31, hi2 = (ln >> 5) & 1;
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    char* ot = bufA + wid * 8192;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        struct alignas(8) O4 { T v[4]; } o4;
#pragma unroll
        for (int i = 0; i < 4; ++i) o4.v[i] = from_f32<T>(acc[n][4 * j + i] * inv);
        *reinterpret_cast<O4*>(ot + img_off(lq2, 4 * n + j) + 8 * hi2) = o4;
      }
    if (hi == 0 && a.lse && qrow < L)
      a.lse[(long long)head * a.T + s0 + qrow] = l_i > 0.f ? m_i + __log2f(l_i) : INFINITY;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back its own tile only
    T* O = reinterpret_cast<T*>(a.o) + (long long)s0 * a.ldo + head * D;
    const int ch = ln & 15;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int r = 4 * it + ((ln >> 4) & 3);
      const uint4 v = *reinterpret_cast<const uint4*>(ot + img_off(r, ch));
      if (wq0 + r < L) *reinterpret_cast<uint4*>(O + (long long)(wq0 + r) * a.ldo + ch * 8) = v;
    }
  }
  // the next item (persistent launch) refills bufA: every wave's read-back is done first
  if (a.nitems > 0) lds_fence_barrier();
  };
  if (a.nitems > 0) {
    // snake order over the heaviest-first item list: round r takes items r*G + w (even r) or
    // r*G + G-1-w (odd r), pairing heavy with light items per workgroup (static balance)
    const int G = gridDim.x, w = blockIdx.x;
    for (int base = 0; base < a.nitems; base += G) {
      const int it = (a.snake && ((base / G) & 1)) ? base + G - 1 - w : base + w;
      if (it >= a.nitems) continue;
      const int ti = it / a.nh;
      run(a.tiles[2 * ti], a.tiles[2 * ti + 1], it - ti * a.nh);
    }
  } else {
    const Work wk = work_item(a);
    if (wk.seq < 0) return;
    run(wk.seq, wk.r0, wk.head);
  }
}

// (A 256-query-tile forward -- 8 waves, one workgroup per CU, a 3-buffer K / V ring -- measured
// 48.5 vs 39.9 us per call and 90.30 vs 90.20 ms per step, profiles/r5_fa, and was removed: with
// one workgroup per CU the two waves of a SIMD run their MFMA and softmax phases in lockstep.)

template <typename T, bool CAUSAL, bool MASK>
__device__ __forceinline__ void dq32_tile(const char* kimg, const char* vimg, const Off32& off,
                                          const uint4 (&qf)[8], const uint4 (&of)[8],
                                          f32x16 (&dq)[4], int kv0, int L, int qrow, int hi,
                                          float lse_q, float del_q, float scale_log2) {
  // one 32-key block at a time: 32 accumulator registers live instead of 64, which keeps the
  // kernel at two waves per SIMD
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    f32x16 st = zero16(), dpt = zero16();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      st = Mfma32<T>::run(lds16(kimg + kb * 8192 + off.row[ks]), qf[ks], st);
      dpt = Mfma32<T>::run(lds16(vimg + kb * 8192 + off.row[ks]), of[ks], dpt);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float pv = fexp2(fmaf(st[r], scale_log2, -lse_q));
      if (MASK) {
        const int kpos = kv0 + kb * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
        const bool out = (kpos >= L) | (qrow >= L) | (CAUSAL & (kpos > qrow));
        pv = out ? 0.f : pv;
      }
      dpt[r] = pv * (dpt[r] - del_q);
    }
    // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint4 db = pack8<T>(dpt, s);
#pragma unroll
      for (int n = 0; n < 4; ++n)
        dq[n] = Mfma32<T>::run(tr32(kimg, off, kb * 32 + 16 * s, n), db, dq[n]);
    }
  }
}

// ---- backward dQ: 32 queries per wave, 128 per workgroup ------------------------------------
// S^T = K Q^T, dP^T = V dO^T (keys on rows, lane = query); dQ^T += K^T dS^T.  The recompute
// path, used when the dS hand-off buffer does not fit (LUMEN_FA_DS_MB).  (A variant that also
// formed delta from the rows it loads measured neutral and was removed.)
template <typename T, bool CAUSAL>
__global__ void __launch_bounds__(256, 2) bwd_dq32_kernel(Args a) {
  constexpr int BM = 128;
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lq = lane & 31, hi = lane >> 5;
  const Work wk = work_item(a);
  if (wk.seq < 0) return;
  const int seq = wk.seq, q0 = wk.r0;
  const int head = wk.head, kvh = head / (a.nh / a.nkv);
  const int s0 = a.cu[seq], L = a.cu[seq + 1] - s0;
  const T* Q = reinterpret_cast<const T*>(a.q) + (long long)s0 * a.ldq + head * D;
  const T* dO = reinterpret_cast<const T*>(a.dout) + (long long)s0 * a.lddo + head * D;
  const T* K = reinterpret_cast<const T*>(a.k) + (long long)s0 * a.ldk + kvh * D;
  const T* V = reinterpret_cast<const T*>(a.v) + (long long)s0 * a.ldv + kvh * D;
  const int wq0 = q0 + wid * 32;
  const int qrow = wq0 + lq;
  uint4 qf[8], of[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    qf[ks] = gload16(Q + (long long)qrow * a.ldq + 16 * ks + 8 * hi, qrow < L);
    of[ks] = gload16(dO + (long long)qrow * a.lddo + 16 * ks + 8 * hi, qrow < L);
  }
  const float lse_q = qrow < L ? a.lse[(long long)head * a.T + s0 + qrow] : INFINITY;
  const float del_q = qrow < L ? a.delta[(long long)head * a.T + s0 + qrow] : 0.f;
  f32x16 dq[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) dq[n] = zero16();
  const int kv_end = CAUSAL ? min(L, q0 + BM) : L;
  const int w_end = CAUSAL ? min(kv_end, wq0 + 32) : kv_end;
  wait_vm_all();
  if (kv_end > 0) {
    stage64_async(smem, K, a.ldk, 0, L);
    stage64_async(smem + IMG, V, a.ldv, 0, L);
  }
  Off32 off;
  make_off32(off, lane);
  int it = 0;
  for (int kv0 = 0; kv0 < kv_end; kv0 += BN, ++it) {
    char* kimg = smem + (it & 1) * 2 * IMG;
    char* vimg = kimg + IMG;
    if (kv0 + BN < kv_end) {
      char* nk = smem + ((it + 1) & 1) * 2 * IMG;
      stage64_async(nk, K, a.ldk, kv0 + BN, L);
      stage64_async(nk + IMG, V, a.ldv, kv0 + BN, L);
      wait_vm_8();
    } else {
      wait_vm_all();
    }
    lds_fence_barrier();
    if (kv0 < w_end) {
      // wave-uniform (the MFMAs read every lane's operands: never branch per lane around them)
      const bool need_mask = (kv0 + BN > L) || (wq0 + 32 > L) || (CAUSAL && kv0 + BN - 1 > wq0);
      if (need_mask)
        dq32_tile<T, CAUSAL, true>(kimg, vimg, off, qf, of, dq, kv0, L, qrow, hi, lse_q, del_q,
                                   a.scale_log2);
      else
        dq32_tile<T, CAUSAL, false>(kimg, vimg, off, qf, of, dq, kv0, L, qrow, hi, lse_q, del_q,
                                    a.scale_log2);
    }
    lds_fence_barrier();
  }
  if (qrow < L) {
    T* dQ = reinterpret_cast<T*>(a.dq) + (long long)s0 * a.lddq + head * D + (long long)qrow * a.lddq;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[n][r] *= a.scale;
    if (a.rope_pos != nullptr) {
      // column 32n + 8jj + 4hi + i pairs with n ^ 2 (64 columns on): same lane and register
      const float* cb = a.rope_cos + (long long)a.rope_pos[s0 + qrow] * 64 + 4 * hi;
      const float* sb = a.rope_sin + (long long)a.rope_pos[s0 + qrow] * 64 + 4 * hi;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float4 c4 = *reinterpret_cast<const float4*>(cb + 32 * n + 8 * jj);
          const float4 s4 = *reinterpret_cast<const float4*>(sb + 32 * n + 8 * jj);
          const float cs[4] = {c4.x, c4.y, c4.z, c4.w}, sn[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float lo = dq[n][4 * jj + i], hi2 = dq[n + 2][4 * jj + i];
            rope_inv_pair(lo, hi2, cs[i], sn[i]);
            dq[n][4 * jj + i] = lo;
            dq[n + 2][4 * jj + i] = hi2;
          }
        }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        struct alignas(8) O4 { T v[4]; } q4;
#pragma unroll
        for (int i = 0; i < 4; ++i) q4.v[i] = from_f32<T>(dq[n][4 * jj + i]);
        *reinterpret_cast<O4*>(dQ + 32 * n + 8 * jj + 4 * hi) = q4;
      }
  }
}

// ---- backward dQ from the dK/dV kernel's dS tiles (no recompute of S and dP) ----------------
// Workgroup = one 64-query tile of one head, wave v = queries 16v..16v+15 (16x16x32 MFMA).  Per
// key tile: the 8 KiB dS tile and the 16 KiB K tile arrive by LDS-DMA one tile ahead; dQ[16 x 128]
// += dS[16 x 64] K[64 x 128] is 16 MFMAs per wave with both operands read transposed
// (ds_read_b64_tr_b16): dS rows = keys in the hand-off layout (ds_slot), K in the SW = 1 image.
template <typename T, bool CAUSAL>
__global__ void __launch_bounds__(256) bwd_dq_ds_kernel(Args a) {
  constexpr int TILE = IMG + 8192;  // K image | dS tile
  __shared__ __attribute__((aligned(16))) char bufA[TILE];  // ping-pong as in bwd_dkdv_kernel
  __shared__ __attribute__((aligned(16))) char bufB[TILE];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  // persistent (a.nitems > 0, as bwd_dkdv_kernel) over (query tile, head) items
  auto run = [&](const int seq, const int q0, const int head) {
  const int kvh = head / (a.nh / a.nkv);
  const int s0 = a.cu[seq], L = a.cu[seq + 1] - s0;
  const int ns = (L + 63) / 64, qt = q0 / 64;
  const T* K = reinterpret_cast<const T*>(a.k) + (long long)s0 * a.ldk + kvh * D;
  const char* dsq = reinterpret_cast<const char*>(a.ds) + ds_tile(a, head, a.ds_off[seq], qt, 0, ns, CAUSAL);
  const int nkt = CAUSAL ? qt + 1 : ns;  // key tiles (contiguous in the hand-off buffer)
  // per-lane dS read offsets (tile-relative): source lane s = 4i + m of each 16-lane group g reads
  // keys 4g + i (+16 for the hi half) of the 32-key slice ks, queries 16 wid + 4m .. +3
  const int si = lr >> 2, sm = lr & 3;
  const int dso = ((wid >> 1) * 1024) + (wid & 1) * 8 + ds_slot(sm, 4 * lg + si);
  auto stage = [&](char* buf, int kt) {
    stage64_async_o<T, 1>(buf, K, a.ldk, kt * 64, L);
    const char* src = dsq + (long long)kt * 8192;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int off = (wid * 2 + i) * 1024;
      dma16_o(src + off + lane * 16, buf + IMG + off);
    }
  };
  f32x4 dq[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) dq[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nkt > 0) stage(bufA, 0);
  auto step = [&](int kt, char* buf, char* nx) {
    if (kt + 1 < nkt) {
      stage(nx, kt + 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      wait_vm_all();
    }
    lds_fence_barrier();
    const char* kimg = buf;
    const char* dsi = buf + IMG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // A = dS[query 16 wid + lr][keys 32ks + 4lg + 0..3 | 32ks + 16 + 4lg + 0..3]: the wave
      // w = key / 16 blocks 2ks and 2ks + 1 of the hand-off layout
      const uint2 lo = tr_read_raw(dsi + (2 * ks) * 2048 + dso);
      const uint2 hi = tr_read_raw(dsi + (2 * ks + 1) * 2048 + dso);
      const uint4 af = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
      for (int n = 0; n < 8; ++n)
        dq[n] = Mfma<T>::run(af, tr_read_img2<1>(kimg, 32 * ks + 4 * lg, 32 * ks + 16 + 4 * lg, n * 16, lane), dq[n]);
    }
    lds_fence_barrier();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, bufA, bufB);
    if (kt + 1 < nkt) step(kt + 1, bufB, bufA);
  }
  // lane: queries q0 + 16 wid + 4lg + r, columns 16n + lr
  T* dQ = reinterpret_cast<T*>(a.dq) + (long long)s0 * a.lddq + head * D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + wid * 16 + 4 * lg + r;
    if (qr >= L) continue;
    float qv[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) qv[n] = dq[n][r] * a.scale;
    if (a.rope_pos != nullptr) {  // column 16n + lr pairs with 16(n + 4) + lr: same lane
      const long long pb = (long long)a.rope_pos[s0 + qr] * 64 + lr;
#pragma unroll
      for (int n = 0; n < 4; ++n)
        rope_inv_pair(qv[n], qv[n + 4], a.rope_cos[pb + 16 * n], a.rope_sin[pb + 16 * n]);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) dQ[(long long)qr * a.lddq + n * 16 + lr] = from_f32<T>(qv[n]);
  }
  };
  if (a.nitems > 0) {
    // snake order over the heaviest-first item list: round r takes items r*G + w (even r) or
    // r*G + G-1-w (odd r), pairing heavy with light items per workgroup (static balance)
    const int G = gridDim.x, w = blockIdx.x;
    for (int base = 0; base < a.nitems; base += G) {
      const int it = (a.snake && ((base / G) & 1)) ? base + G - 1 - w : base + w;
      if (it >= a.nitems) continue;
      const int ti = it / a.nh;
      run(a.tiles[2 * ti], a.tiles[2 * ti + 1], it - ti * a.nh);
    }
  } else {
    const Work wk = work_item(a);
    if (wk.seq < 0) return;
    run(wk.seq, wk.r0, wk.head);
  }
}

// (An 8-wave, 128-key dK/dV variant with a 3-deep DMA ring measured slower than the 4-wave
// kernel above -- 117.6 vs 108.0 us at B=8 S=512, gpurun r2_36 -- and was removed.)

static int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <typename T>
static hipError_t launch(int which, int causal, int mt, int ntiles, const Args& a, hipStream_t st) {
  dim3 block(256);
  if (which == 0) {  // forward: 32x32x16 kernel, 128-row tiles
    if (mt != 20) return hipErrorInvalidValue;
    dim3 grid(ntiles, a.tiles3 ? 1 : a.nh);
    if (a.nitems > 0) grid = dim3(std::min(a.nitems, (causal ? 2 : 1) * cu_count()), 1);
    if (causal) hipLaunchKernelGGL((fwd32_kernel<T, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((fwd32_kernel<T, false>), grid, block, 0, st, a);
  } else if (which == 1) {
    dim3 grid((unsigned)((a.T + 3) / 4));
    hipLaunchKernelGGL(delta_kernel<T>, grid, block, 0, st, a);
  } else if (which == 2) {  // dK/dV (64-key tiles), dS recomputed by which 5
    dim3 grid(ntiles, a.tiles3 ? 1 : a.nkv);
    if (causal) hipLaunchKernelGGL((bwd_dkdv_kernel<T, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((bwd_dkdv_kernel<T, false>), grid, block, 0, st, a);
  } else if (which == 5) {  // dQ, 32x32x16 kernel, 128-query tiles
    dim3 grid(ntiles, a.tiles3 ? 1 : a.nh);
    if (causal) hipLaunchKernelGGL((bwd_dq32_kernel<T, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((bwd_dq32_kernel<T, false>), grid, block, 0, st, a);
  } else if (which == 7) {  // dK/dV (64-key tiles) + dS hand-off
    dim3 grid(ntiles, a.tiles3 ? 1 : a.nkv);
    if (a.nitems > 0) grid = dim3(std::min(a.nitems, 2 * cu_count()), 1);
    if (causal) hipLaunchKernelGGL((bwd_dkdv_kernel<T, true, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((bwd_dkdv_kernel<T, false, true>), grid, block, 0, st, a);
  } else if (which == 8) {  // dQ from the dS hand-off (64-query tiles)
    dim3 grid(ntiles, a.tiles3 ? 1 : a.nh);
    if (a.nitems > 0) grid = dim3(std::min(a.nitems, 3 * cu_count()), 1);  // 48 KiB LDS: 3 / CU
    if (causal) hipLaunchKernelGGL((bwd_dq_ds_kernel<T, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((bwd_dq_ds_kernel<T, false>), grid, block, 0, st, a);
  } else if (which == 6) {  // forward over the paged KV cache (32x32x16, 128-row tiles)
    dim3 grid(ntiles, a.nh);
    if (a.nitems > 0) grid = dim3(std::min(a.nitems, (causal ? 2 : 1) * cu_count()), 1);
    if (causal) hipLaunchKernelGGL((fwd32_kernel<T, true, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((fwd32_kernel<T, false, true>), grid, block, 0, st, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace fa
}  // namespace lumen

#include <algorithm>
#include <cstdlib>
// persistent launches (bit 0 dK/dV, 1 forward, 2 dQ-from-dS; bit 3 snake item order);
// LUMEN_FA_PERSIST overrides.
// Default 15 = all three, snake order.  dK/dV: 109.6 -> 91.6 us persistent (gpurun r2_51),
// snake 98.0 -> 96.3 (r2_55).  Forward: slower persistent with its round-2 prologue
// (52.4 -> 55.6), faster since Q arrives by LDS-DMA with the first K/V tile: 45.1 -> 41.0 us at
// B=8 S=512 and 128 -> 95 us at B=2 S=2048 causal.  dQ-from-dS: neutral at B=8 S=512, backward
// 338 -> 320 us at B=2 S=2048 causal (profiles/r3d/fa; round 2 measured it slower, 35.2 -> 39.4,
// before the dQ kernel's register fix).
static int fa_persist() {
  static int v = [] { const char* e = std::getenv("LUMEN_FA_PERSIST"); return e ? std::atoi(e) : 15; }();
  return v;
}

// which: 0 = forward (mt must be 20: the 32x32x16 kernel, 128-row tiles), 1 = delta,
//        2 = dK/dV (64-key tiles), 5 = dQ (32x32x16, 128-query tiles).  (Measured-slower
//        variants -- a 16x16x32 forward, the transposed-formulation forward, 16x16x32 dQ and a
//        32x32x16 dK/dV -- were removed, profiles/r02_fa and profiles/r2_fa.)
extern "C" hipError_t lumen_flash_attn(int dtype, int which, int causal, int mt,
                                       const void* q, const void* k, const void* v,
                                       long long ldq, long long ldk, long long ldv, void* o,
                                       long long ldo, float* lse, const int* cu,
                                       const int* tiles, int ntiles, int nh, int nkv, int T,
                                       float scale, const void* dout, long long lddo, void* dq,
                                       void* dk, void* dv, long long lddq, long long lddk,
                                       long long lddv, const float* delta, const int* rope_pos,
                                       const float* rope_cos, const float* rope_sin,
                                       hipStream_t st) {
  if (nkv <= 0 || nh % nkv != 0) return hipErrorInvalidValue;
  const int tiles3 = (which >> 8) & 1;  // 0x100: (seq, row, head) triples, 1-D grid
  which &= 0xff;
  if (tiles3 && which != 0 && which != 2 && which != 5) return hipErrorInvalidValue;
  // the fused inverse RoPE exists in the dK/dV kernel (which 2) and the 32x32 dQ kernel (which 5)
  if (rope_pos != nullptr && which != 2 && which != 5) return hipErrorInvalidValue;
  if (which != 1 && ntiles == 0) return hipSuccess;
  lumen::fa::Args a;
  a.q = q; a.k = k; a.v = v; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.o = o; a.ldo = ldo;
  a.lse = lse; a.cu = cu; a.tiles = tiles; a.nh = nh; a.nkv = nkv; a.T = T;
  a.scale = scale; a.scale_log2 = scale * 1.4426950408889634f;
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.dk = dk; a.dv = dv; a.lddq = lddq; a.lddk = lddk;
  a.lddv = lddv; a.delta = delta;
  a.rope_pos = rope_pos; a.rope_cos = rope_cos; a.rope_sin = rope_sin;
  a.kv_lens = nullptr; a.block_tables = nullptr; a.bt_stride = 0; a.block_size = 0;
  a.ds = nullptr; a.ds_off = nullptr; a.ds_total = 0; a.tiles3 = tiles3;
  a.nitems = (which == 0 && mt == 20 && !tiles3 && (fa_persist() & 2)) ? ntiles * nh : 0;
  a.snake = (fa_persist() >> 3) & 1;
  if (which == 6 || which == 7 || which == 8) return hipErrorInvalidValue;  // other entries
  if (dtype == lumen::kBF16) return lumen::fa::launch<lumen::bf16>(which, causal, mt, ntiles, a, st);
  if (dtype == lumen::kF16) return lumen::fa::launch<lumen::fp16>(which, causal, mt, ntiles, a, st);
  return hipErrorInvalidValue;
}

// Serving prefill (whole prompts, chunks of long prompts, or the prefill part of a mixed step):
// queries from the token-major q rows (cu_q: per-sequence row offsets), keys / values from the
// paged KV cache (this chunk's K/V already written there), kv_lens[s] = cached context + chunk.
extern "C" hipError_t lumen_flash_attn_paged(int dtype, int causal, const void* q, long long ldq,
                                             const void* k_cache, const void* v_cache, void* o,
                                             long long ldo, const int* cu_q, const int* kv_lens,
                                             const int* tiles, int ntiles,
                                             const int* block_tables, int bt_stride,
                                             int block_size, int nh, int nkv, int T, float scale,
                                             hipStream_t st) {
  if (nkv <= 0 || nh % nkv != 0 || block_size <= 0) return hipErrorInvalidValue;
  if (ntiles == 0) return hipSuccess;
  lumen::fa::Args a{};
  a.q = q; a.ldq = ldq; a.k = k_cache; a.v = v_cache; a.ldk = a.ldv = 0;
  a.o = o; a.ldo = ldo; a.lse = nullptr; a.cu = cu_q; a.tiles = tiles;
  a.nh = nh; a.nkv = nkv; a.T = T;
  a.scale = scale; a.scale_log2 = scale * 1.4426950408889634f;
  a.kv_lens = kv_lens; a.block_tables = block_tables; a.bt_stride = bt_stride;
  a.block_size = block_size;
  // one-shot grid: the persistent form measured neutral on the serving burst (7.54k / 7.51k vs
  // 7.55k / 7.53k tok/s, profiles/r3d/fa) and its item loop keeps a scratch reload per key tile
  // in this (PAGED) instantiation
  a.nitems = 0;
  if (dtype == lumen::kBF16) return lumen::fa::launch<lumen::bf16>(6, causal, 20, ntiles, a, st);
  if (dtype == lumen::kF16) return lumen::fa::launch<lumen::fp16>(6, causal, 20, ntiles, a, st);
  return hipErrorInvalidValue;
}

// Backward with the dS hand-off: which 7 = dK/dV + dS store (64-key tiles), 8 = dQ from dS
// (64-query tiles).  ds: [nh][ds_total][64 x 64] 16-bit, ds_off[seq] = the sequence's first tile.
extern "C" hipError_t lumen_flash_attn_ds(int dtype, int which, int causal, const void* q,
                                          const void* k, const void* v, long long ldq,
                                          long long ldk, long long ldv, const float* lse,
                                          const int* cu, const int* tiles, int ntiles, int nh,
                                          int nkv, int T, float scale, const void* dout,
                                          long long lddo, void* dq, void* dk, void* dv,
                                          long long lddq, long long lddk, long long lddv,
                                          const float* delta, const int* rope_pos,
                                          const float* rope_cos, const float* rope_sin, void* ds,
                                          const int* ds_off, int ds_total, hipStream_t st) {
  const int tiles3 = (which >> 8) & 1;
  which &= 0xff;
  if (nkv <= 0 || nh % nkv != 0 || (which != 7 && which != 8) || ds == nullptr ||
      ds_off == nullptr)
    return hipErrorInvalidValue;
  if (ntiles == 0) return hipSuccess;
  lumen::fa::Args a{};
  a.q = q; a.k = k; a.v = v; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv;
  a.lse = const_cast<float*>(lse); a.cu = cu; a.tiles = tiles; a.nh = nh; a.nkv = nkv; a.T = T;
  a.scale = scale; a.scale_log2 = scale * 1.4426950408889634f;
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.dk = dk; a.dv = dv; a.lddq = lddq; a.lddk = lddk;
  a.lddv = lddv; a.delta = delta;
  a.rope_pos = rope_pos; a.rope_cos = rope_cos; a.rope_sin = rope_sin;
  a.ds = ds; a.ds_off = ds_off; a.ds_total = ds_total; a.tiles3 = tiles3;
  a.snake = (fa_persist() >> 3) & 1;
  a.nitems = tiles3 ? 0 : (which == 7 && (fa_persist() & 1)) ? ntiles * nkv
                        : (which == 8 && (fa_persist() & 4)) ? ntiles * nh : 0;
  if (dtype == lumen::kBF16) return lumen::fa::launch<lumen::bf16>(which, causal, 1, ntiles, a, st);
  if (dtype == lumen::kF16) return lumen::fa::launch<lumen::fp16>(which, causal, 1, ntiles, a, st);
  return hipErrorInvalidValue;
}
