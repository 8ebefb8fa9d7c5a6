// Shared helpers for the gfx950 kernels behind include/rpc_hip.h.
// Wave = 64 lanes (CDNA4); every block size here is a multiple of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rpc_hip.h"

#define RPC_CHECK(expr)                                   \
  do {                                                    \
    hipError_t _e = (expr);                               \
    if (_e != hipSuccess) return (int)RPC_ERR_HIP;        \
  } while (0)

#define RPC_LAUNCH_CHECK() RPC_CHECK(hipGetLastError())

namespace rpc {

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Last-arriving-block hand-off (cdna_hip_programming.md §5 "In-launch split-K
// reduction" / Guideline 16): every block has stored its partials with plain stores;
// each wave drains, the block meets at a barrier, lane 0 releases at agent scope and
// takes a ticket. The block that draws gridDim.x-1 acquires at agent scope before
// reading the other blocks' partials. `ticket` must be zero at launch (hipMemsetAsync
// by the launcher); the last block re-arms it to zero.
__device__ __forceinline__ bool last_block_arrive(unsigned* ticket, int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == gridDim.x - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// The same hand-off for a grid of `nblocks` blocks in any shape.
__device__ __forceinline__ bool last_block_arrive_2d(unsigned* ticket, int* lds_flag, int nblocks) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == (unsigned)nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// The same hand-off without the agent-scope release / acquire fences, for producers whose hand-off data is
// written with agent-scope atomic stores (st_agent: `global_store ... sc1`, coherent across the XCDs' L2s)
// and read back with agent-scope atomic loads (ld_agent: `... sc1`). The release fence of
// last_block_arrive_2d is a `buffer_wbl2`, which writes back every dirty line of the XCD's L2 — under a
// GEMM epilogue that is the block's whole output tile, once per block; here each block only waits for its
// own sc1 stores to complete (vmcnt(0)) before taking a ticket. Data not written with st_agent is not
// handed off.
__device__ __forceinline__ bool last_block_arrive_lite(unsigned* ticket, int* lds_flag, int nblocks) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int last = (t == (unsigned)nblocks - 1);
    if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fixed-order reduction of split-K slabs: dW[e] = sum_c part[c * total + e] (c ascending within
// each of 8 interleaved lanes, lanes combined as a fixed pairwise tree), in double. Block = 64
// outputs x 8 lanes, each lane with 8 loads in flight -> deterministic and latency-tolerant (the
// 64-channel head weight-gradient slabs of CenterPoint ran at 0.6 TB/s with 4 x 4). Predicated: a
// missing chunk reads a clamped address and adds 0.0 (r05: a remainder loop, one load per round trip,
// took every launch with fewer than 64 slabs — the sparse weight gradients' 28-56 — to ~1 TB/s)
template <int DUMMY = 0>
__global__ __launch_bounds__(512) void k_slab_reduce(const float* __restrict__ part, int chunks, long long total,
                                                     float* __restrict__ out) {
  __shared__ double sh[8][64];
  const int o = threadIdx.x & 63, q = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + o;
  double s = 0.0;
  if (e < total) {
    for (int c = q; c < chunks; c += 64) {
      float a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {   // clamped address + select (a conditional load waits for itself)
        const float v = part[(long long)min(c + 8 * k, chunks - 1) * total + e];
        a[k] = c + 8 * k < chunks ? v : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += (double)a[k];
    }
  }
  sh[q][o] = s;
  __syncthreads();
  if (q == 0 && e < total)
    out[e] = (float)((((sh[0][o] + sh[1][o]) + (sh[2][o] + sh[3][o])) + ((sh[4][o] + sh[5][o]) + (sh[6][o] + sh[7][o]))));
}

inline void slab_reduce(const float* part, int chunks, long long total, float* out, hipStream_t st) {
  hipLaunchKernelGGL(k_slab_reduce<0>, dim3((unsigned)((total + 63) / 64)), dim3(512), 0, st, part, chunks, total,
                     out);
}

inline int grid_for(long long n, int block, int cap) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace rpc
