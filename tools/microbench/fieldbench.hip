// Microbenchmark: Montgomery multiplication throughput on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
#include "mulvariants.hpp"
using namespace gm;

template <class P, int V>
__global__ void __launch_bounds__(256) k_mulchain(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<P> a, b;
#pragma unroll
  for (int i = 0; i < P::N; i++) { a.v[i] = io[(tid * P::N + i) % 4096] & 0x0fffffff; b.v[i] = (a.v[i] * 2654435761u) & 0x0fffffff; }
  Fe<P> c = a;
  for (int k = 0; k < iters; k++) { if (V==0) { a = fe_mul(a, b); c = fe_mul(c, a);} else { a = fe_mul_ps(a, b); c = fe_mul_ps(c, a);} }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) s ^= a.v[i] ^ c.v[i];
  if (s == 0x12345678) io[tid % 4096] = s;
}

__global__ void __launch_bounds__(256) k_mad(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[8]; uint64_t acc[8];
  for (int i = 0; i < 8; i++) { a[i] = io[(tid + i) % 4096]; acc[i] = a[i]; }
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (uint64_t)a[i] * (uint32_t)acc[(i + 1) & 7] + (acc[i] >> 32);
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  if (s == 0x12345678) io[tid % 4096] = (uint32_t)s;
}

__global__ void __launch_bounds__(256) k_mad_ind(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[8]; uint64_t acc[8];
  for (int i = 0; i < 8; i++) { a[i] = io[(tid + i) % 4096]; acc[i] = a[i]; }
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(acc[i]) : "v"(a[i]));
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  if (s == 0x12345678) io[tid % 4096] = (uint32_t)s;
}
__global__ void __launch_bounds__(256) k_addc_ind(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc[8];
  for (int i = 0; i < 8; i++) { acc[i] = io[(tid + i) % 4096]; }
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_addc_co_u32 %0, s[0:1], %0, 0, s[2:3]" : "+v"(acc[i]));
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  if (s == 0x12345678) io[tid % 4096] = (uint32_t)s;
}
__global__ void __launch_bounds__(256) k_mullo_ind(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc[8];
  for (int i = 0; i < 8; i++) { acc[i] = io[(tid + i) % 4096]; }
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("v_mul_hi_u32 %0, %0, %0" : "+v"(acc[i]));
  }
  uint64_t s = 0; for (int i = 0; i < 8; i++) s ^= acc[i];
  if (s == 0x12345678) io[tid % 4096] = (uint32_t)s;
}
template <class K>
double timeit(K kern, uint32_t* d, int blocks, int iters) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  kern<<<blocks, 256>>>(d, iters); hipDeviceSynchronize();
  hipEventRecord(e0);
  kern<<<blocks, 256>>>(d, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint32_t* d; hipMalloc(&d, 4096 * 4);
  uint32_t h[4096]; for (int i = 0; i < 4096; i++) h[i] = i * 2654435761u + 12345;
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  int blocks = 256 * 16, iters = 200;
  double threads = blocks * 256.0;
  double ms = timeit(k_mulchain<Bn254Fp,0>, d, blocks, iters);
  printf("bn254 fp mul CIOS-C: %.3f ms -> %.2f Gmul/s\n", ms, threads * iters * 2 / ms / 1e6);
  ms = timeit(k_mulchain<Bn254Fp,1>, d, blocks, iters);
  printf("bn254 fp mul FIPS-asm: %.3f ms -> %.2f Gmul/s\n", ms, threads * iters * 2 / ms / 1e6);
  ms = timeit(k_mulchain<Bls377Fp,0>, d, blocks, iters);
  printf("bls377 fp mul CIOS-C: %.3f ms -> %.2f Gmul/s\n", ms, threads * iters * 2 / ms / 1e6);
  ms = timeit(k_mulchain<Bls377Fp,1>, d, blocks, iters);
  printf("bls377 fp mul FIPS-asm: %.3f ms -> %.2f Gmul/s\n", ms, threads * iters * 2 / ms / 1e6);
  ms = timeit(k_mad_ind, d, blocks, iters * 16);
  printf("mad_u64_u32 indep: %.3f ms -> %.2f Tops/s\n", ms, threads * iters * 16 * 8 / ms / 1e9);
  ms = timeit(k_addc_ind, d, blocks, iters * 16);
  printf("addc indep: %.3f ms -> %.2f Tops/s\n", ms, threads * iters * 16 * 8 / ms / 1e9);
  ms = timeit(k_mullo_ind, d, blocks, iters * 16);
  printf("mul_hi_u32 indep: %.3f ms -> %.2f Tops/s\n", ms, threads * iters * 16 * 8 / ms / 1e9);
  return 0;
}
