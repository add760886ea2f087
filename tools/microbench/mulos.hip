// Microbenchmark: radix-2^29 Montgomery product, product scanning (gm::fe_mul,
// one serial 64-bit accumulator) vs operand scanning with N independent 64-bit
// column accumulators (ILP ~ 2N), at forced occupancies 1/2/4/8 waves per SIMD
// (occupancy set by dynamic LDS per 256-thread block).  Also checks that both
// variants agree on random inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../gnark-icicle_amd/csrc/field.hpp"
using namespace gm;

template <class P>
__device__ __forceinline__ Fe<P> mul_os(const Fe<P>& a, const Fe<P>& b) {
  constexpr int N = P::N;
  uint64_t t[N];
#pragma unroll
  for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j < N; j++) t[j] += (uint64_t)a.v[i] * b.v[j];
    const uint32_t m = ((uint32_t)t[0] * P::INV) & LIMB_MASK;
#pragma unroll
    for (int j = 0; j < N; j++) t[j] += (uint64_t)m * P::p(j);
    const uint64_t carry = t[0] >> RADIX;
#pragma unroll
    for (int j = 0; j < N - 1; j++) t[j] = t[j + 1];
    t[0] += carry;
    t[N - 1] = 0;
  }
  Fe<P> r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < N; j++) {
    c += t[j];
    r.v[j] = (uint32_t)c & LIMB_MASK;
    c >>= RADIX;
  }
  r.v[N - 1] |= (uint32_t)c << RADIX;  // top limb may exceed 29 bits before the final subtract
  fe_reduce_once(r);
  return r;
}

template <int V, class P>
__device__ __forceinline__ Fe<P> MUL(const Fe<P>& a, const Fe<P>& b) {
  if constexpr (V == 0) return fe_mul(a, b);
  else return mul_os(a, b);
}

template <int V>
__global__ void __launch_bounds__(256) kbench(uint32_t* io, int iters) {
  extern __shared__ uint32_t lds[];
  using P = Bn254Fp;
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<P> a, b;
  for (int i = 0; i < P::N; i++) {
    a.v[i] = io[(tid * 9 + i) % 4096] & 0x0fffffff;
    b.v[i] = (a.v[i] * 2654435761u) & 0x0fffffff;
  }
  Fe<P> c = a;
  for (int k = 0; k < iters; k++) {
    a = MUL<V>(a, b);
    c = MUL<V>(c, a);
  }
  uint32_t s = 0;
  for (int i = 0; i < P::N; i++) s ^= a.v[i] ^ c.v[i];
  if (s == 0x12345678) { lds[threadIdx.x] = s; io[tid % 4096] = lds[(threadIdx.x + 1) % 256]; }
}

__global__ void kcheck(const uint32_t* in, uint32_t* bad, int n) {
  using P = Bn254Fp;
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  Fe<P> a, b;
  for (int i = 0; i < P::N; i++) { a.v[i] = in[t * 18 + i] & LIMB_MASK; b.v[i] = in[t * 18 + 9 + i] & LIMB_MASK; }
  a.v[8] &= 0x1fffff; b.v[8] &= 0x1fffff;  // < 2^253 < p
  fe_reduce_once(a); fe_reduce_once(b);
  Fe<P> x = fe_mul(a, b), y = mul_os(a, b);
  if (!fe_eq(x, y)) atomicAdd(bad, 1u);
  Fe<P> z = fe_mul(x, y), w = mul_os(y, x);
  if (!fe_eq(z, w)) atomicAdd(bad, 1u);
}

template <int V>
float timeit(uint32_t* d, int blocks, int iters, size_t lds) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kbench<V>, dim3(blocks), dim3(256), lds, 0, d, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kbench<V>, dim3(blocks), dim3(256), lds, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 4096 * 4 * 18);
  static uint32_t h[4096 * 18];
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < 4096 * 18; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (uint32_t)s; }
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  uint32_t* bad;
  (void)hipMalloc(&bad, 4);
  (void)hipMemset(bad, 0, 4);
  kcheck<<<64, 64>>>(d, bad, 4096);
  uint32_t hb = 0;
  (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("os-vs-ps mismatches: %u of 8192\n", hb);
  const int iters = 100;
  // waves/SIMD w: blocks per CU = w (256 threads = 4 waves = 1 per SIMD)
  for (int w : {1, 2, 3, 4, 8}) {
    size_t lds = 0;
    int blocks = 256 * w;  // one round: w blocks (= w waves per SIMD) per CU
    double muls = (double)blocks * 256 * iters * 2;
    float t0 = timeit<0>(d, blocks, iters, lds);
    float t1 = timeit<1>(d, blocks, iters, lds);
    printf("occ~%d (lds %zu) PS %.3f ms %.1f Gmul/s | OS %.3f ms %.1f Gmul/s\n", w, lds, t0, muls / t0 / 1e6, t1,
           muls / t1 / 1e6);
  }
  return 0;
}
