// Token-embedding row gather: out[t, :] = W[ids[t], :] for the frozen embedding
// table (training forward; serving prefill / decode).  Reference: the embedding lookup inside
// LlamaForCausalLM / OPTForCausalLM (training/train_baseline.py:122).
//
// Pure bandwidth: each row is H 16-bit values moved as 16-byte vectors; a 256-thread block
// copies ROWS rows (one wave per row, 64 lanes x 16 B = 1 KiB per instruction), with every
// load of the block issued before the first store.  Out-of-range ids (padding / ignored
// positions) produce zero rows instead of faulting.
#include "common.h"

namespace lumen {

template <int VPL>  // 16-byte vectors per lane per row (H <= 64 * 8 * VPL)
__global__ void __launch_bounds__(256) embedding_kernel(const uint4* __restrict__ W,
                                                        const long long* __restrict__ ids,
                                                        uint4* __restrict__ out, int T, int V,
                                                        int hv) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const long long id = ids[t];
  const bool ok = id >= 0 && id < V;
  uint4 v[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    v[i] = (ok && c < hv) ? W[id * hv + c] : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < hv) out[(long long)t * hv + c] = v[i];
  }
}

}  // namespace lumen

// W [V, H] 16-bit contiguous, ids int64 [T], out [T, H]; H multiple of 8, H <= 16384
extern "C" hipError_t lumen_embedding(const void* W, const long long* ids, void* out, int T,
                                      int V, int H, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  if ((H & 7) || H > 16384 || V <= 0) return hipErrorInvalidValue;
  const int hv = H / 8;
  const dim3 grid((T + 3) / 4), block(256);
  const uint4* w = reinterpret_cast<const uint4*>(W);
  uint4* o = reinterpret_cast<uint4*>(out);
  if (hv <= 64) hipLaunchKernelGGL((lumen::embedding_kernel<1>), grid, block, 0, st, w, ids, o, T, V, hv);
  else if (hv <= 128) hipLaunchKernelGGL((lumen::embedding_kernel<2>), grid, block, 0, st, w, ids, o, T, V, hv);
  else if (hv <= 256) hipLaunchKernelGGL((lumen::embedding_kernel<4>), grid, block, 0, st, w, ids, o, T, V, hv);
  else if (hv <= 512) hipLaunchKernelGGL((lumen::embedding_kernel<8>), grid, block, 0, st, w, ids, o, T, V, hv);
  else if (hv <= 1024) hipLaunchKernelGGL((lumen::embedding_kernel<16>), grid, block, 0, st, w, ids, o, T, V, hv);
  else hipLaunchKernelGGL((lumen::embedding_kernel<32>), grid, block, 0, st, w, ids, o, T, V, hv);
  return hipGetLastError();
}
