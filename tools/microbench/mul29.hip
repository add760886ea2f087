// Microbenchmark: radix-2^29 unsaturated Montgomery multiplication vs 32-bit CIOS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../../gnark-icicle_amd/csrc/field.hpp"
using namespace gm;

struct F29 { uint32_t v[9]; };
__device__ __forceinline__ uint32_t P29(int i) {
  constexpr uint32_t a[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u, 0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  return a[i];
}
constexpr uint32_t INV29 = 0x04866389u;
constexpr uint32_t M29 = (1u << 29) - 1;

__device__ __forceinline__ F29 mul29(const F29& a, const F29& b) {
  uint64_t acc = 0;
  uint32_t m[9];
  F29 r;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k - 8 > 0 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) acc += (uint64_t)a.v[i] * b.v[k - i];
#pragma unroll
    for (int i = (k - 8 > 0 ? k - 8 : 0); i <= (k - 1 < 8 ? k - 1 : 8); i++) acc += (uint64_t)m[i] * P29(k - i);
    if (k < 9) {
      m[k] = ((uint32_t)acc * INV29) & M29;
      acc += (uint64_t)m[k] * P29(0);
    } else {
      r.v[k - 9] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

__global__ void __launch_bounds__(256) k29(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  F29 a, b;
  for (int i = 0; i < 9; i++) { a.v[i] = io[(tid * 9 + i) % 4096] & 0x0fffffff; b.v[i] = (a.v[i] * 2654435761u) & 0x0fffffff; }
  F29 c = a;
  for (int k = 0; k < iters; k++) { a = mul29(a, b); c = mul29(c, a); }
  uint32_t s = 0;
  for (int i = 0; i < 9; i++) s ^= a.v[i] ^ c.v[i];
  if (s == 0x12345678) io[tid % 4096] = s;
}
__global__ void __launch_bounds__(256) k32(uint32_t* io, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<Bn254Fp> a, b;
  for (int i = 0; i < 8; i++) { a.v[i] = io[(tid * 8 + i) % 4096] & 0x0fffffff; b.v[i] = (a.v[i] * 2654435761u) & 0x0fffffff; }
  Fe<Bn254Fp> c = a;
  for (int k = 0; k < iters; k++) { a = fe_mul(a, b); c = fe_mul(c, a); }
  uint32_t s = 0;
  for (int i = 0; i < 8; i++) s ^= a.v[i] ^ c.v[i];
  if (s == 0x12345678) io[tid % 4096] = s;
}
// correctness: compare mul29 against CIOS-32 on random inputs (convert via host)
__global__ void kcheck(const uint32_t* a32, const uint32_t* b32, uint32_t* o29, uint32_t* o32, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x; if (t >= n) return;
  F29 a, b;
  for (int i = 0; i < 9; i++) { a.v[i] = a32[t * 9 + i]; b.v[i] = b32[t * 9 + i]; }
  F29 r = mul29(a, b);
  for (int i = 0; i < 9; i++) o29[t * 9 + i] = r.v[i];
}

template <class K>
float timeit(K kern, uint32_t* d, int blocks, int iters) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  kern<<<blocks, 256>>>(d, iters); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  kern<<<blocks, 256>>>(d, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint32_t* d; (void)hipMalloc(&d, 4096 * 4);
  uint32_t h[4096]; for (int i = 0; i < 4096; i++) h[i] = i * 2654435761u + 12345;
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  int blocks = 256 * 16, iters = 200;
  double threads = blocks * 256.0;
  for (int rep = 0; rep < 2; rep++) {
    float ms = timeit(k32, d, blocks, iters);
    printf("CIOS-32 : %.3f ms -> %.2f Gmul/s\n", ms, threads * iters * 2 / ms / 1e6);
    ms = timeit(k29, d, blocks, iters);
    printf("radix-29: %.3f ms -> %.2f Gmul/s\n", ms, threads * iters * 2 / ms / 1e6);
  }
  // correctness vs host big-int: write inputs, read outputs, check in python later
  const int n = 1024;
  uint32_t *da, *db, *do29, *do32; (void)hipMalloc(&da, n*36); (void)hipMalloc(&db, n*36); (void)hipMalloc(&do29, n*36); (void)hipMalloc(&do32, n*36);
  static uint32_t ha[1024*9], hb[1024*9], ho[1024*9];
  uint64_t s = 88172645463325252ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
  for (int i = 0; i < n * 9; i++) { ha[i] = rnd() & M29; hb[i] = rnd() & M29; }
  for (int i = 0; i < n; i++) { ha[i*9+8] &= 0x1fffff; hb[i*9+8] &= 0x1fffff; }  // < 2^253 < 2p
  (void)hipMemcpy(da, ha, n*36, hipMemcpyHostToDevice); (void)hipMemcpy(db, hb, n*36, hipMemcpyHostToDevice);
  kcheck<<<n/64, 64>>>(da, db, do29, do32, n);
  (void)hipMemcpy(ho, do29, n*36, hipMemcpyDeviceToHost);
  FILE* f = fopen("mul29_check.bin", "wb"); fwrite(ha, 4, n*9, f); fwrite(hb, 4, n*9, f); fwrite(ho, 4, n*9, f); fclose(f);
  printf("wrote mul29_check.bin\n");
  return 0;
}
