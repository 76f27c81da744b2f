// Shared LDS tile helpers for 16x16x32 bf16/fp16 MFMA kernels on gfx950.
//
// A "128-image" is a [rows][128] 16-bit tile in LDS: 256-byte rows split into 16-byte chunks
// whose chunk index is XOR-swizzled by the row, so both access patterns the MFMA operands need
// are bank-conflict free:
//   * row reads   : lane (L, g) reads 8 consecutive columns of row L        (k along columns)
//   * tr reads    : ds_read_b64_tr_b16 gathers 8 consecutive rows of a column (k along rows)
// Operand convention of v_mfma_f32_16x16x32_{bf16,f16}: lane (L = lane & 15, g = lane >> 4)
// supplies row/col L and k-elements [8g, 8g + 8); the accumulator lane holds rows 4g..4g+3 of
// column L.
#pragma once
#include "common.h"

namespace lumen {
namespace tile {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

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

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * 256 + ((chunk ^ swz(row)) << 4);
}

__device__ __forceinline__ uint4 row_read(const char* img, int row, int chunk) {
  return *reinterpret_cast<const uint4*>(img + img_off(row, chunk));
}

__device__ __forceinline__ uint2 tr_read_raw(const char* p) {
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(uint2, r);
}

// operand whose k axis runs along the image rows: lane (L, g) gets column n0 + L,
// rows k0 + 8g .. k0 + 8g + 7
__device__ __forceinline__ uint4 tr_read_img(const char* img, int k0, int n0, int lane) {
  const int L = lane & 15, g = lane >> 4;
  const int col = n0 + 4 * (L & 3);
  const int ch = col >> 3, half = (col >> 2) & 1;
  const int r = k0 + 8 * g + (L >> 2);
  const uint2 lo = tr_read_raw(img + img_off(r, ch) + 8 * half);
  const uint2 hi = tr_read_raw(img + img_off(r + 4, ch) + 8 * half);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// Alternative swizzle for images read BOTH by 16-row ds_read_b128 row reads (rows 16w + L,
// chunks 4i + g) and by tr_read_img (rows k0 + 8g + 0..7): the default swz is 2-way
// bank-conflicted on the row reads (dy3: 20% of LDS cycles); this one (row bits 0, 1, 3 ->
// chunk bits 3, 2, 1) is conflict-free on both (scripts/probes/fa_bank_model.py model).
__device__ __forceinline__ int swz_b(int row) {
  return ((row & 1) << 3) | ((row & 2) << 1) | (((row >> 3) & 1) << 1);
}
__device__ __forceinline__ int img_off_b(int row, int chunk) {
  return row * 256 + ((chunk ^ swz_b(row)) << 4);
}
__device__ __forceinline__ uint4 row_read_b(const char* img, int row, int chunk) {
  return *reinterpret_cast<const uint4*>(img + img_off_b(row, chunk));
}
__device__ __forceinline__ uint4 tr_read_img_b(const char* img, int k0, int n0, int lane) {
  const int L = lane & 15, g = lane >> 4;
  const int col = n0 + 4 * (L & 3);
  const int ch = col >> 3, half = (col >> 2) & 1;
  const int r = k0 + 8 * g + (L >> 2);
  const uint2 lo = tr_read_raw(img + img_off_b(r, ch) + 8 * half);
  const uint2 hi = tr_read_raw(img + img_off_b(r + 4, ch) + 8 * half);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}

// 8 floats -> 8 packed 16-bit values (round to nearest even)
template <typename T>
__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  return make_uint4(pk2<T>(v[0], v[1]), pk2<T>(v[2], v[3]), pk2<T>(v[4], v[5]),
                    pk2<T>(v[6], v[7]));
}

template <typename T>
__device__ __forceinline__ void unpack8(uint4 raw, float (&v)[8]) {
  const Vec8<T> e = __builtin_bit_cast(Vec8<T>, raw);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = to_f32(e.v[j]);
}

template <typename T>
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  struct alignas(8) P { T v[4]; } o;
  o.v[0] = from_f32<T>(a); o.v[1] = from_f32<T>(b);
  o.v[2] = from_f32<T>(c); o.v[3] = from_f32<T>(d);
  return __builtin_bit_cast(uint2, o);
}

}  // namespace tile
}  // namespace lumen
