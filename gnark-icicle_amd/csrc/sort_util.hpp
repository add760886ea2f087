// Block-level building blocks of the MSM bucket sort (msm_impl.hpp pass 1,
// msm_sort.hip pass 2): wave / block scans and an LDS counter increment that
// returns the entry's rank.  All assume 1024-thread blocks of wave64.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gm {

constexpr uint32_t S_THREADS = 1024;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += u;
  }
  return v;
}

// Exclusive scan of a[0, len) (LDS) by a 1024-thread block; returns the total.
// wsum: 17 words of LDS.  Synchronises on entry and exit.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t* a, uint32_t len, uint32_t* wsum) {
  __syncthreads();
  const uint32_t t = threadIdx.x;
  const uint32_t per = (len + S_THREADS - 1) / S_THREADS;
  const uint32_t lo = min(t * per, len), hi = min(lo + per, len);
  uint32_t s = 0;
  for (uint32_t q = lo; q < hi; q++) s += a[q];
  const uint32_t inc = wave_incl_scan(s);
  if ((t & 63) == 63) wsum[t >> 6] = inc;
  __syncthreads();
  if (t < 64) {
    const uint32_t v = t < S_THREADS / 64 ? wsum[t] : 0u;
    const uint32_t vi = wave_incl_scan(v);
    if (t < S_THREADS / 64) wsum[t] = vi - v;
    if (t == S_THREADS / 64 - 1) wsum[S_THREADS / 64] = vi;
  }
  __syncthreads();
  uint32_t run = wsum[t >> 6] + inc - s;
  for (uint32_t q = lo; q < hi; q++) {
    const uint32_t x = a[q];
    a[q] = run;
    run += x;
  }
  const uint32_t total = wsum[S_THREADS / 64];
  __syncthreads();
  return total;
}

// rank = hist[key]++ for the active lanes.  When every active lane of the wave
// has the same key (skewed scalars: one huge bucket) the wave does ONE atomic
// instead of 64 serialised same-address LDS atomics.
__device__ __forceinline__ uint32_t lds_rank_add(uint32_t* hist, uint32_t key) {
  const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
  const uint64_t active = __ballot(1);
  if (__ballot(key == k0) == active) {
    const uint32_t below = (uint32_t)__popcll(active & __lanemask_lt());
    uint32_t old = 0;
    if (below == 0) old = atomicAdd(&hist[k0], (uint32_t)__popcll(active));
    return __builtin_amdgcn_readfirstlane(old) + below;
  }
  return atomicAdd(&hist[key], 1u);
}

}  // namespace gm
