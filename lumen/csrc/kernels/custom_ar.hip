// Custom all-reduce for tensor-parallel decode over xGMI peer memory (reference:
// vLLM csrc/custom_all_reduce.cu, declared through vllm==0.6.0 in requirements.txt).
//
// Why: a TP decode step does two all-reduces per layer on a few KB .. few MB. For messages
// that small, RCCL's ring latency dominates. RCCL also cannot sit inside the hipGraph of a
// decode bucket, so TP decode used to run eagerly. Here every rank maps every peer's staging
// buffer into its address space (hipIpcGetMemHandle / hipIpcOpenMemHandle; on MI355X these are
// direct loads over the point-to-point xGMI links) and one kernel does the whole collective:
//
//   one-shot  (small messages):  copy my input into my staging buffer  ->  barrier  ->
//             sum the same range of all W staging buffers  ->  barrier (buffers reusable)
//   two-shot  (larger):          copy  ->  barrier  ->  reduce my 1/W part from all peers, write
//             it back into my staging buffer  ->  barrier  ->  gather every part from its owner
//             ->  barrier
//
// One-shot reads (W-1)·n bytes over the links per rank. Two-shot reads 2(W-1)/W·n. Each rank
// has 7 links of ~153 GB/s, so one-shot wins below a few hundred KB.
//
// Synchronisation. Block b of every rank owns the same contiguous range of the message, so
// barriers are per block and no grid-wide sync is needed. A barrier is:
//   1. a system-scope release;
//   2. thread t < W writes the call's epoch into peer t's signal slot [b][my rank];
//   3. thread t spins until my slot [b][t] holds the epoch.
// Each block keeps its epoch counter in its own signal struct. Kernel arguments are therefore
// identical on every call, so the kernel can be captured in a hipGraph and replayed.
// Staging buffers and signals are allocated uncached (hipDeviceMallocUncached), so
// cross-device loads never see stale L2 lines.
//
// Every spin has a deadline (s_memrealtime, 100 MHz). A rank whose peer never arrives sets
// `err` and leaves, so a missing peer turns into a host-visible error instead of a hung GPU.
// The same timeout also sets a word in pinned, host-mapped memory (`host_err`), so the host
// can poll it after every step with a plain load -- no device sync, no copy -- and stop before
// it hands out tokens computed from a half-reduced tensor.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "common.h"

using namespace lumen;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 128;
constexpr int kThreads = 256;
constexpr int kBarriers = 3;

struct Signal {
  uint32_t bar[kBarriers][kMaxBlocks][kMaxRanks];
  uint32_t epoch[kMaxBlocks];
  uint32_t err;
  // diagnostics (read by the host after a timeout or at the end of a run, never per step):
  // err_info = the FIRST timed-out wait: 1<<31 | barrier << 24 | block << 16 | missing peer << 8
  // | low 8 bits of the epoch (= call count of that block); long_wait_us = the longest barrier
  // wait above kLongWaitTicks (1 ms), so a shared-device rehearsal shows how far ranks drift
  uint32_t err_info;
  uint32_t long_wait_us;
  uint32_t long_waits;
};

constexpr uint64_t kLongWaitTicks = 100000;  // 1 ms of the 100 MHz s_memrealtime clock

struct Peers {
  void* data[kMaxRanks];
  Signal* sig[kMaxRanks];
  uint32_t* host_err;  // pinned host-mapped error word (device view), or null
};

__device__ __forceinline__ void block_barrier(const Peers& P, Signal* self, int slot, int rank,
                                              int world, uint32_t epoch, uint64_t deadline_ticks) {
  __threadfence_system();  // this thread's staging writes reach memory before the flag
  __syncthreads();
  const int b = blockIdx.x;
  if (threadIdx.x < world) {
    const int t = threadIdx.x;
    // the fence above already released this block's writes (every thread ran it before the
    // __syncthreads), so the flag store and the polling loads can be relaxed: no L2
    // writeback/invalidate on each poll, one acquire fence after the loop
    __hip_atomic_store(&P.sig[t]->bar[slot][b][rank], epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = &self->bar[slot][b][t];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t waited = 0;
    while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      waited = __builtin_amdgcn_s_memrealtime() - t0;
      if (waited > deadline_ticks) {
        __hip_atomic_fetch_or(&self->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t expect = 0u;
        const uint32_t info = (1u << 31) | ((uint32_t)slot << 24) | ((uint32_t)b << 16) |
                              ((uint32_t)t << 8) | (epoch & 0xffu);
        __hip_atomic_compare_exchange_strong(&self->err_info, &expect, info, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (P.host_err)
          __hip_atomic_store(P.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (waited > kLongWaitTicks) {  // rare path: no extra atomic on a prompt barrier
      const uint64_t us = waited / 100;
      __hip_atomic_fetch_max(&self->long_wait_us, us > 0xffffffffull ? 0xffffffffu : (uint32_t)us,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_fetch_add(&self->long_waits, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
}

// W > 0: the peer count is a compile-time constant and every peer's load is issued before the
// first add, so W loads are in flight together (the link latency is paid once, not W times)
template <typename T, int W>
__device__ __forceinline__ void sum_peers(const Peers& P, int world, long long e, float (&acc)[8]) {
  if constexpr (W > 0) {
    float v[W][8];
#pragma unroll
    for (int q = 0; q < W; ++q) load8<T>(reinterpret_cast<const T*>(P.data[q]) + e, v[q]);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = v[0][i];
#pragma unroll
    for (int q = 1; q < W; ++q)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[q][i];
  } else {
    load8<T>(reinterpret_cast<const T*>(P.data[0]) + e, acc);
    for (int q = 1; q < world; ++q) {
      float v[8];
      load8<T>(reinterpret_cast<const T*>(P.data[q]) + e, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[i];
    }
  }
}

// n8 = numel / 8 ("units" of 8 elements: 16 B for 16-bit types, 32 B for f32)
template <typename T, bool TWO_SHOT, int W>
__global__ void __launch_bounds__(kThreads)
allreduce_kernel(Peers P, const T* __restrict__ in, T* __restrict__ out, long long n8, int rank,
                 int world, uint64_t deadline_ticks) {
  Signal* self = P.sig[rank];
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = self->epoch[blockIdx.x] + 1;
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const int G = gridDim.x;
  const long long lo = n8 * blockIdx.x / G, hi = n8 * (blockIdx.x + 1) / G;
  T* mine = reinterpret_cast<T*>(P.data[rank]);

  for (long long u = lo + threadIdx.x; u < hi; u += kThreads) {
    float v[8];
    load8<T>(in + u * 8, v);
    store8<T>(mine + u * 8, v);
  }
  block_barrier(P, self, 0, rank, world, epoch, deadline_ticks);

  if (!TWO_SHOT) {
    for (long long u = lo + threadIdx.x; u < hi; u += kThreads) {
      float acc[8];
      sum_peers<T, W>(P, world, u * 8, acc);
      store8<T>(out + u * 8, acc);
    }
  } else {
    const long long span = hi - lo;
    const long long plo = lo + span * rank / world, phi = lo + span * (rank + 1) / world;
    for (long long u = plo + threadIdx.x; u < phi; u += kThreads) {
      float acc[8];
      sum_peers<T, W>(P, world, u * 8, acc);
      store8<T>(mine + u * 8, acc);  // peers gather my reduced part from here
      store8<T>(out + u * 8, acc);
    }
    block_barrier(P, self, 1, rank, world, epoch, deadline_ticks);
    for (int q = 1; q < world; ++q) {
      const int src = (rank + q) % world;  // stagger so the ranks start on different links
      const long long qlo = lo + span * src / world, qhi = lo + span * (src + 1) / world;
      const T* theirs = reinterpret_cast<const T*>(P.data[src]);
      for (long long u = qlo + threadIdx.x; u < qhi; u += kThreads) {
        float v[8];
        load8<T>(theirs + u * 8, v);
        store8<T>(out + u * 8, v);
      }
    }
  }
  // nobody may overwrite a staging buffer (next call) while a peer still reads it
  block_barrier(P, self, 2, rank, world, epoch, deadline_ticks);
  if (threadIdx.x == 0) self->epoch[blockIdx.x] = epoch;
}

// All-gather of row-major shards: rank q holds in[R, Vs]; out[R, W*Vs] gets shard q in columns
// [q*Vs, (q+1)*Vs) on every rank (the vocab-parallel LM head's logits).  Same staging buffers
// and barriers as the all-reduce; the interleaving into `out` is done by the stores, so no
// separate concatenation pass is needed.  vs8 = Vs / 8.
template <typename T>
__global__ void __launch_bounds__(kThreads)
allgather_kernel(Peers P, const T* __restrict__ in, T* __restrict__ out, long long rows, int vs8,
                 int rank, int world, uint64_t deadline_ticks) {
  Signal* self = P.sig[rank];
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) s_epoch = self->epoch[blockIdx.x] + 1;
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const long long n8 = rows * vs8;
  const int G = gridDim.x;
  const long long lo = n8 * blockIdx.x / G, hi = n8 * (blockIdx.x + 1) / G;
  T* mine = reinterpret_cast<T*>(P.data[rank]);
  for (long long u = lo + threadIdx.x; u < hi; u += kThreads) {
    float v[8];
    load8<T>(in + u * 8, v);
    store8<T>(mine + u * 8, v);
  }
  block_barrier(P, self, 0, rank, world, epoch, deadline_ticks);
  const long long ld = (long long)world * vs8 * 8;
  for (int k = 0; k < world; ++k) {
    const int q = (rank + k) % world;
    const T* theirs = reinterpret_cast<const T*>(P.data[q]);
    for (long long u = lo + threadIdx.x; u < hi; u += kThreads) {
      const long long r = u / vs8, c = u - r * vs8;
      float v[8];
      load8<T>(theirs + u * 8, v);
      store8<T>(out + r * ld + (long long)q * vs8 * 8 + c * 8, v);
    }
  }
  block_barrier(P, self, 2, rank, world, epoch, deadline_ticks);
  if (threadIdx.x == 0) self->epoch[blockIdx.x] = epoch;
}

template <typename T, int W>
hipError_t launch_w(const Peers& P, const void* in, void* out, long long n8, int rank, int world,
                    int two_shot, int blocks, uint64_t ticks, hipStream_t st) {
  if (two_shot)
    hipLaunchKernelGGL((allreduce_kernel<T, true, W>), dim3(blocks), dim3(kThreads), 0, st, P,
                       (const T*)in, (T*)out, n8, rank, world, ticks);
  else
    hipLaunchKernelGGL((allreduce_kernel<T, false, W>), dim3(blocks), dim3(kThreads), 0, st, P,
                       (const T*)in, (T*)out, n8, rank, world, ticks);
  return hipGetLastError();
}

template <typename T>
hipError_t launch(const Peers& P, const void* in, void* out, long long numel, int rank, int world,
                  int two_shot, int blocks, double timeout_s, hipStream_t st) {
  const long long n8 = numel / 8;
  const uint64_t ticks = (uint64_t)(timeout_s * 1.0e8);
  switch (world) {
    case 2: return launch_w<T, 2>(P, in, out, n8, rank, world, two_shot, blocks, ticks, st);
    case 4: return launch_w<T, 4>(P, in, out, n8, rank, world, two_shot, blocks, ticks, st);
    case 8: return launch_w<T, 8>(P, in, out, n8, rank, world, two_shot, blocks, ticks, st);
    default: return launch_w<T, 0>(P, in, out, n8, rank, world, two_shot, blocks, ticks, st);
  }
}

}  // namespace

extern "C" {

long long lumen_car_signal_bytes() { return (long long)sizeof(Signal); }
int lumen_car_max_blocks() { return kMaxBlocks; }
int lumen_car_max_ranks() { return kMaxRanks; }

// device allocation for staging buffers and signals, zero-filled; uncached unless `cached`
// (cached staging relies on the barrier's system-scope L2 writeback / invalidate instead)
hipError_t lumen_car_alloc(long long bytes, int cached, void** ptr) {
  hipError_t e = cached ? hipMalloc(ptr, (size_t)bytes)
                        : hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  e = hipMemset(*ptr, 0, (size_t)bytes);
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

hipError_t lumen_car_free(void* ptr) { return hipFree(ptr); }

hipError_t lumen_car_get_handle(void* ptr, void* handle_out /* hipIpcMemHandle_t bytes */) {
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), ptr);
}

int lumen_car_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

hipError_t lumen_car_open_handle(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

hipError_t lumen_car_close_handle(void* ptr) { return hipIpcCloseMemHandle(ptr); }

// pinned host word the kernels raise on a barrier timeout; *dev is its device-side address
hipError_t lumen_car_host_flag_alloc(void** host, void** dev) {
  hipError_t e = hipHostMalloc(host, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return e;
  memset(*host, 0, 64);
  return hipHostGetDevicePointer(dev, *host, 0);
}

hipError_t lumen_car_host_flag_free(void* host) { return hipHostFree(host); }

hipError_t lumen_car_read_err(void* sig, unsigned int* err) {
  return hipMemcpy(err, &reinterpret_cast<Signal*>(sig)->err, sizeof(unsigned int),
                   hipMemcpyDeviceToHost);
}

// out[4] = err, err_info, long_wait_us, long_waits (synchronous: diagnostics only)
hipError_t lumen_car_read_diag(void* sig, unsigned int* out) {
  return hipMemcpy(out, &reinterpret_cast<Signal*>(sig)->err, 4 * sizeof(unsigned int),
                   hipMemcpyDeviceToHost);
}

// data[i] / sig[i]: rank i's staging buffer and signal as mapped in THIS process
hipError_t lumen_car_allreduce(int dtype, const long long* data, const long long* sig, int rank,
                               int world, const void* in, void* out, long long numel, int two_shot,
                               int blocks, double timeout_s, void* host_err, hipStream_t st) {
  if (world < 1 || world > kMaxRanks || blocks < 1 || blocks > kMaxBlocks || (numel & 7))
    return hipErrorInvalidValue;
  Peers P{};
  P.host_err = reinterpret_cast<uint32_t*>(host_err);
  for (int i = 0; i < world; ++i) {
    P.data[i] = reinterpret_cast<void*>(data[i]);
    P.sig[i] = reinterpret_cast<Signal*>(sig[i]);
  }
  switch (dtype) {
    case 0: return launch<float>(P, in, out, numel, rank, world, two_shot, blocks, timeout_s, st);
    case 1: return launch<fp16>(P, in, out, numel, rank, world, two_shot, blocks, timeout_s, st);
    case 2: return launch<bf16>(P, in, out, numel, rank, world, two_shot, blocks, timeout_s, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t lumen_car_allgather(int dtype, const long long* data, const long long* sig, int rank,
                               int world, const void* in, void* out, long long rows,
                               long long shard_cols, int blocks, double timeout_s, void* host_err,
                               hipStream_t st) {
  if (world < 1 || world > kMaxRanks || blocks < 1 || blocks > kMaxBlocks || (shard_cols & 7))
    return hipErrorInvalidValue;
  Peers P{};
  P.host_err = reinterpret_cast<uint32_t*>(host_err);
  for (int i = 0; i < world; ++i) {
    P.data[i] = reinterpret_cast<void*>(data[i]);
    P.sig[i] = reinterpret_cast<Signal*>(sig[i]);
  }
  const uint64_t ticks = (uint64_t)(timeout_s * 1.0e8);
  const int vs8 = (int)(shard_cols / 8);
  switch (dtype) {
    case 0:
      hipLaunchKernelGGL(allgather_kernel<float>, dim3(blocks), dim3(kThreads), 0, st, P,
                         (const float*)in, (float*)out, rows, vs8, rank, world, ticks);
      break;
    case 1:
      hipLaunchKernelGGL(allgather_kernel<fp16>, dim3(blocks), dim3(kThreads), 0, st, P,
                         (const fp16*)in, (fp16*)out, rows, vs8, rank, world, ticks);
      break;
    case 2:
      hipLaunchKernelGGL(allgather_kernel<bf16>, dim3(blocks), dim3(kThreads), 0, st, P,
                         (const bf16*)in, (bf16*)out, rows, vs8, rank, world, ticks);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // extern "C"
