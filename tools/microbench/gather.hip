// FETCH_SIZE calibration for the MSM accumulation's access pattern (VERDICT r04
// item 6): how many bytes does rocprofv3's FETCH_SIZE report for
//   stream16   a coalesced streaming read, 16 B per lane (the guide's reference:
//              FETCH_SIZE = half the bytes on gfx950)
//   gather64   one 64-B record per thread at a pseudo-random index (the point
//              gather of k_msm_accum_seg: 4 x 16-B loads of one packed point)
// over tables larger than the 256 MiB Infinity Cache (1 GiB) and smaller (128
// MiB, the 2^21 GLV point set of the 2^20 bench MSM).  Known byte counts are
// printed; run each counter pass separately:
//   timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d OUT -o gather --output-format csv -- ./gather
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) k_fill(uint4* t, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) t[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 7), 0x9e3779b9u * (uint32_t)i, 7u);
}

__global__ void __launch_bounds__(256) k_stream16(const uint4* __restrict__ t, size_t n, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = t[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// nrec records of 64 B (4 uint4); thread i reads record mix(i) % nrec
__global__ void __launch_bounds__(256) k_gather64(const uint4* __restrict__ t, uint32_t nrec, uint32_t nthreads,
                                                  uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nthreads) return;
  const uint32_t r = mix(i) % nrec;
  const uint4* p = t + (size_t)r * 4;
  uint32_t acc = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 v = p[q];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[i] = acc;
}

int main() {
  const size_t big = size_t(1) << 30, small = size_t(128) << 20;  // bytes
  uint4* t;
  uint32_t* out;
  if (hipMalloc(&t, big) != hipSuccess || hipMalloc(&out, sizeof(uint32_t) << 24) != hipSuccess) return 1;
  k_fill<<<(big / 16 + 255) / 256, 256>>>(t, big / 16);
  // streaming read of the whole 1 GiB table and of the first 128 MiB
  for (size_t bytes : {big, small}) {
    k_stream16<<<8192, 256>>>(t, bytes / 16, out);
    printf("stream16 bytes=%zu\n", bytes);
  }
  // 2^24 gathers of 64 B from a 1 GiB table (2^24 records) and from 128 MiB (2^21 records)
  const uint32_t nthr = 1u << 24;
  for (size_t bytes : {big, small}) {
    k_gather64<<<nthr / 256, 256>>>(t, (uint32_t)(bytes / 64), nthr, out);
    printf("gather64 table=%zu records_read=%u bytes=%zu\n", bytes, nthr, (size_t)nthr * 64);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  hipFree(t);
  hipFree(out);
  return 0;
}
