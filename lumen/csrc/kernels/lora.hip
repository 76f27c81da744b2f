// LoRA low-rank adapter GEMMs, forward and backward (north-star kernel).
//
// Reference behaviour: PEFT 0.13 LoraLayer on q/k/v/o (training/train_baseline.py:131-141,
// LoraConfig r=16, alpha=32, dropout=0.05): y = W x + B(A(dropout(x))) * alpha/r, launched as
// dropout -> Linear(A) -> Linear(B) -> mul -> add (4-5 launches per adapted linear, plus the
// autograd of each).  Adapter weights are kept in f32 (PEFT autocast_adapter_dtype).
//
// All six products the adapters need are "skinny": one dimension is the rank (16, or 48 for the
// fused q|k|v adapters).  One templated kernel covers them: an LDS-staged MFMA tile loop on the
// exact-f32 matrix instruction v_mfma_f32_16x16x4_f32 (inputs converted to f32 while staging, so
// the adapter math is f32-exact on 16-bit activations).  Work per product is < 0.5 GFLOP, so the
// f32 MFMA rate (155 TF) keeps them memory/latency-bound; the kernel's job is coalesced 16-byte
// staging of the big operand, split-K for parallelism and an epilogue that lands the result
// where it is consumed (grad buffers by f32 atomics, the base GEMM output by an in-place add).
//
//   mode  product                                   X (M x K)            W (N x K)        C
//   1     Z  = drop(x) A^T          [T, R]          x   [T][Kf] kmaj     A  [R][Kf] kmaj   atomic f32
//   2     dZ = s dY_seg B_seg       [T, r]          dY  [T][N]  kmaj     B  [N][r] (nmaj)  atomic f32
//   3     dA = dZ^T drop(x)         [R, Kf]         dZ  [T][R] (mmaj)    x  [T][Kf] (nmaj) atomic f32
//   4     dB = s dY_seg^T Z_seg     [N, r]          dY  [T][N] (mmaj)    Z  [T][R] (nmaj)  atomic f32
//   5     dx += drop'(dZ A)         [T, Kf]         dZ  [T][R] kmaj      A  [R][Kf] (nmaj) 16-bit RMW
//   6     y  += s Z_seg B_seg^T     [T, N]          Z   [T][R] kmaj      B  [N][r] kmaj    16-bit RMW
//
// Tile: BM = 64 rows (4 waves x 16), BN = 16 or 64 columns, BK = 32; blockIdx.z enumerates
// (segment, K-split).  LDS rows are padded to 34 floats so the MFMA operand reads
// (lanes = 16 rows x 2 k) hit 32 distinct banks.
#include "common.h"

namespace lumen {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 64, kBK = 32, kLdsStride = kBK + 2;

struct SegArgs {
  long long x_off[4], w_off[4], c_off[4];
  int M[4], N[4], K[4];
  int nseg;
};

struct LoraGemmArgs {
  const void* X;
  const void* W;
  void* C;
  long long ldx, ldw;  // leading dims (elements)
  long long cs_m, cs_n;  // C strides
  float alpha;
  int ksplit;
  // dropout on the x operand (mode 1: X, mode 3: W); logical element (t, f) -> t * drop_ld + f
  unsigned int seed;          // host-premixed 32-bit seed
  unsigned int drop_thresh;  // 0 = no dropout
  float drop_scale;
  long long drop_ld;
  SegArgs seg;
};

template <typename T>
__device__ __forceinline__ void load8_any(const T* p, float (&o)[8]) { load8(p, o); }

// Stage a [rows x BK] operand tile (row = output index, col = k) into LDS as f32.
// KMAJ: element (r, k) at P[r * ld + k]; otherwise at P[k * ld + r].
// DROP_RK: dropout logical index; DROP_T_IS_ROW selects whether row or k is the token index.
template <typename T, bool KMAJ, int ROWS, bool DROP, bool DROP_T_IS_ROW>
__device__ __forceinline__ void stage_tile(float* __restrict__ lds, const T* __restrict__ P,
                                           long long ld, int r0, int rmax, int k0, int kmax,
                                           const LoraGemmArgs& a) {
  const int tid = threadIdx.x;
  if (KMAJ) {
    // ROWS rows x 32 k: 4 threads per row, 8 k each
    if (tid < ROWS * 4) {
      const int rr = tid >> 2, kk = (tid & 3) * 8;
      float v[8];
      const int r = r0 + rr, k = k0 + kk;
      if (r < rmax && k < kmax) {
        load8_any(P + static_cast<long long>(r) * ld + k, v);
        if (DROP) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const long long t = DROP_T_IS_ROW ? r : (k + j);
            const long long f = DROP_T_IS_ROW ? (k + j) : r;
            v[j] = dropout_keep(a.seed, t * a.drop_ld + f, a.drop_thresh) ? v[j] * a.drop_scale
                                                                           : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) lds[rr * kLdsStride + kk + j] = v[j];
    }
  } else {
    // 32 k-rows x ROWS contiguous: ROWS/8 threads per k-row
    constexpr int TPR = ROWS / 8;
    if (tid < 32 * TPR) {
      const int kk = tid / TPR, rr = (tid % TPR) * 8;
      float v[8];
      const int k = k0 + kk, r = r0 + rr;
      if (k < kmax && r < rmax) {
        load8_any(P + static_cast<long long>(k) * ld + r, v);
        if (DROP) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const long long t = DROP_T_IS_ROW ? (r + j) : k;
            const long long f = DROP_T_IS_ROW ? k : (r + j);
            v[j] = dropout_keep(a.seed, t * a.drop_ld + f, a.drop_thresh) ? v[j] * a.drop_scale
                                                                           : 0.f;
          }
        }
        // rows beyond rmax inside this 8-vector are never read by a valid output; zero them
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (r + j >= rmax) v[j] = 0.f;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) lds[(rr + j) * kLdsStride + kk] = v[j];
    }
  }
}

// EPI: 0 = f32 atomicAdd, 2 = 16-bit read-modify-write add (TC = 16-bit type)
template <typename TX, typename TW, typename TC, bool XK, bool WK, int EPI, int DROP, bool DROP_T_ROW,
          int BN>
__global__ void __launch_bounds__(256) lora_gemm_kernel(LoraGemmArgs a) {
  __shared__ float xs[kBM * kLdsStride];
  __shared__ float ws[BN * kLdsStride];
  const int nseg = a.seg.nseg;
  const int seg = blockIdx.z % nseg;
  const int split = blockIdx.z / nseg;
  const int M = a.seg.M[seg], N = a.seg.N[seg], K = a.seg.K[seg];
  const int m0 = blockIdx.x * kBM, n0 = blockIdx.y * BN;
  if (m0 >= M || n0 >= N) return;
  int kchunk = (K + a.ksplit - 1) / a.ksplit;
  kchunk = (kchunk + kBK - 1) / kBK * kBK;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);
  if (kbeg >= kend) return;
  const TX* X = reinterpret_cast<const TX*>(a.X) + a.seg.x_off[seg];
  const TW* W = reinterpret_cast<const TW*>(a.W) + a.seg.w_off[seg];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  f32x4 acc[BN / 16];
#pragma unroll
  for (int n = 0; n < BN / 16; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = kbeg; k0 < kend; k0 += kBK) {
    stage_tile<TX, XK, kBM, DROP == 1, DROP_T_ROW>(xs, X, a.ldx, m0, M, k0, kend, a);
    stage_tile<TW, WK, BN, DROP == 2, DROP_T_ROW>(ws, W, a.ldw, n0, N, k0, kend, a);
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < kBK / 4; ++kb) {
      const float av = xs[(wid * 16 + lr) * kLdsStride + kb * 4 + lk];
#pragma unroll
      for (int n = 0; n < BN / 16; ++n) {
        const float bv = ws[(n * 16 + lr) * kLdsStride + kb * 4 + lk];
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[n], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // C/D layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg
  if constexpr (EPI == 0) {
#pragma unroll
    for (int n = 0; n < BN / 16; ++n) {
      const int col = n0 + n * 16 + lr;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wid * 16 + lk * 4 + r;
        if (row >= M) continue;
        const long long off = a.seg.c_off[seg] + row * a.cs_m + col * a.cs_n;
        atomicAdd(reinterpret_cast<float*>(a.C) + off, a.alpha * acc[n][r]);
      }
    }
  } else {
    // 16-bit read-modify-write: stage the f32 tile through LDS, then each thread updates 8
    // consecutive columns of a row with one 16-byte load + one 16-byte store (requires
    // cs_n == 1, N % 8 == 0 and 16-byte aligned rows; checked on the host).
    constexpr int CST = BN + 4;
    __shared__ float cs[kBM * CST];
#pragma unroll
    for (int n = 0; n < BN / 16; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[(wid * 16 + lk * 4 + r) * CST + n * 16 + lr] = acc[n][r];
    __syncthreads();
    constexpr int TPR = BN / 8;              // threads per row
    constexpr int RPP = 256 / TPR;           // rows per pass
    const int tr = threadIdx.x / TPR, tc = (threadIdx.x % TPR) * 8;
#pragma unroll
    for (int pass = 0; pass < kBM / RPP; ++pass) {
      const int lrow = pass * RPP + tr;
      const int row = m0 + lrow, col = n0 + tc;
      if (row < M && col < N) {
        TC* c = reinterpret_cast<TC*>(a.C) + a.seg.c_off[seg] + row * a.cs_m + col;
        float v[8];
        load8(c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float add = a.alpha * cs[lrow * CST + tc + j];
          if (DROP == 3)  // mode 5: d/dx through drop(x); token = row, feature = col
            add = dropout_keep(a.seed, static_cast<long long>(row) * a.drop_ld + col + j,
                               a.drop_thresh) ? add * a.drop_scale : 0.f;
          v[j] += add;
        }
        store8(c, v);
      }
    }
  }
}

template <typename TA>
static hipError_t dispatch(int mode, int bn, const LoraGemmArgs& a, dim3 grid, hipStream_t st) {
  dim3 block(256);
#define LAUNCH(TX, TW, TC, XK, WK, EPI, DROP, DTR, BN) \
  hipLaunchKernelGGL((lora_gemm_kernel<TX, TW, TC, XK, WK, EPI, DROP, DTR, BN>), grid, block, 0, st, a)
#define BOTH_BN(TX, TW, TC, XK, WK, EPI, DROP, DTR) \
  if (bn == 16) LAUNCH(TX, TW, TC, XK, WK, EPI, DROP, DTR, 16); \
  else LAUNCH(TX, TW, TC, XK, WK, EPI, DROP, DTR, 64);
  switch (mode) {
    case 1:  // Z = drop(x) A^T
      if (a.drop_thresh) { BOTH_BN(TA, float, float, true, true, 0, 1, true) }
      else { BOTH_BN(TA, float, float, true, true, 0, 0, true) }
      break;
    case 2:  // dZ = s dY B
      BOTH_BN(TA, float, float, true, false, 0, 0, true)
      break;
    case 3:  // dA = dZ^T drop(x)   (x is the W operand, token index = k)
      if (a.drop_thresh) { BOTH_BN(float, TA, float, false, false, 0, 2, false) }
      else { BOTH_BN(float, TA, float, false, false, 0, 0, false) }
      break;
    case 4:  // dB = s dY^T Z
      BOTH_BN(TA, float, float, false, false, 0, 0, true)
      break;
    case 5:  // dx += drop'(dZ A)   (the x-gradient of the adapter path passes the dropout mask)
      if (a.drop_thresh) { BOTH_BN(float, float, TA, true, false, 2, 3, true) }
      else { BOTH_BN(float, float, TA, true, false, 2, 0, true) }
      break;
    case 6:  // y += s Z B^T
      BOTH_BN(float, float, TA, true, true, 2, 0, true)
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef BOTH_BN
#undef LAUNCH
  return hipGetLastError();
}

}  // namespace lumen

// Generic launcher.  Shapes per segment in `seg`; grid = (ceil(maxM/64), ceil(maxN/BN),
// nseg*ksplit).  Requirements (checked by the Python wrapper): every K-contiguous /
// M-contiguous / N-contiguous run and offset is a multiple of 8 elements and 16-byte aligned.
extern "C" hipError_t lumen_lora_gemm(int act_dtype, int mode, int bn, const void* X,
                                      const void* W, void* C, long long ldx, long long ldw,
                                      long long cs_m, long long cs_n, float alpha, int ksplit,
                                      unsigned long long seed, unsigned int drop_thresh,
                                      float drop_scale, long long drop_ld, int nseg,
                                      const long long* x_off, const long long* w_off,
                                      const long long* c_off, const int* Ms, const int* Ns,
                                      const int* Ks, hipStream_t st) {
  if (nseg < 1 || nseg > 4 || ksplit < 1) return hipErrorInvalidValue;
  if ((mode == 5 || mode == 6) && (ksplit != 1 || cs_n != 1)) return hipErrorInvalidValue;
  lumen::LoraGemmArgs a;
  a.X = X; a.W = W; a.C = C; a.ldx = ldx; a.ldw = ldw; a.cs_m = cs_m; a.cs_n = cs_n;
  a.alpha = alpha; a.ksplit = ksplit;
  a.seed = static_cast<unsigned int>(seed) ^ static_cast<unsigned int>(seed >> 32);
  a.drop_thresh = drop_thresh;
  a.drop_scale = drop_scale; a.drop_ld = drop_ld;
  a.seg.nseg = nseg;
  int maxM = 0, maxN = 0;
  for (int i = 0; i < 4; ++i) {
    const bool v = i < nseg;
    a.seg.x_off[i] = v ? x_off[i] : 0; a.seg.w_off[i] = v ? w_off[i] : 0;
    a.seg.c_off[i] = v ? c_off[i] : 0;
    a.seg.M[i] = v ? Ms[i] : 0; a.seg.N[i] = v ? Ns[i] : 0; a.seg.K[i] = v ? Ks[i] : 0;
    if (v) { maxM = Ms[i] > maxM ? Ms[i] : maxM; maxN = Ns[i] > maxN ? Ns[i] : maxN; }
  }
  if (maxM == 0 || maxN == 0) return hipSuccess;
  const int BN = bn == 16 ? 16 : 64;
  dim3 grid((maxM + lumen::kBM - 1) / lumen::kBM, (maxN + BN - 1) / BN, nseg * ksplit);
  if (act_dtype == lumen::kBF16) return lumen::dispatch<lumen::bf16>(mode, BN, a, grid, st);
  if (act_dtype == lumen::kF16) return lumen::dispatch<lumen::fp16>(mode, BN, a, grid, st);
  return hipErrorInvalidValue;
}
