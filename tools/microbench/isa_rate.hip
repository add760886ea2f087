// Microbenchmark: issue cost (cycles per wave64 instruction per SIMD) of the
// VALU instructions the radix-2^29 field product is made of, measured with 8
// independent dependency chains per wave at 8 waves/SIMD (throughput bound).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(X) X X X X X X X X
template <int OP, bool LAT = false>
__global__ void __launch_bounds__(256) kop(uint32_t* out, int iters) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = threadIdx.x * 3 + 1, y = threadIdx.x * 7 + 5;
  uint64_t fx = 0x3ff0000000000000ull + threadIdx.x, fy = 0x3ff0000000000001ull;  // doubles near 1.0
  for (int k = 0; k < iters; k++) {
#define BODY(A)                                                                                  \
  if constexpr (OP == 0) { uint64_t cc_; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(A), "=s"(cc_) : "v"(x), "v"(y)); } \
  if constexpr (OP == 1) asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(A));                      \
  if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(*(uint32_t*)&A) : "v"(y)); \
  if constexpr (OP == 3) asm volatile("v_and_b32 %0, %0, %1" : "+v"(*(uint32_t*)&A) : "v"(y));    \
  if constexpr (OP == 4) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(*(uint32_t*)&A) : "v"(x), "v"(y)); \
  if constexpr (OP == 5) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(A));                  \
  if constexpr (OP == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(*(uint32_t*)&A) : "v"(y));    \
  if constexpr (OP == 7) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(A) : "v"(fx), "v"(fy));      \
  if constexpr (OP == 8) asm volatile("v_add_f64 %0, %0, %1" : "+v"(A) : "v"(fx));                    \
  if constexpr (OP == 9) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(*(uint32_t*)&A) : "v"(y));     \
  if constexpr (OP == 10) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(*(uint32_t*)&A) : "v"(y));   \
  if constexpr (OP == 11) { uint64_t cc_; asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(*(uint32_t*)&A), "=s"(cc_) : "v"(y)); } \
  if constexpr (OP == 12) asm volatile("v_add_u32 %0, %0, %1" : "+v"(*(uint32_t*)&A) : "v"(y));
    if constexpr (LAT) {
      REP8(BODY(a0) BODY(a0) BODY(a0) BODY(a0) BODY(a0) BODY(a0) BODY(a0) BODY(a0))
    } else {
      REP8(BODY(a0) BODY(a1) BODY(a2) BODY(a3) BODY(a4) BODY(a5) BODY(a6) BODY(a7))
    }
  }
  uint64_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (s == 0x123456789ull) out[threadIdx.x] = (uint32_t)s;
}

static const char* NAMES[] = {"v_mad_u64_u32", "v_lshrrev_b64", "v_mul_lo_u32", "v_and_b32",
                              "v_add3_u32", "v_lshl_add_u64", "v_alignbit_b32", "v_fma_f64", "v_add_f64",
                              "v_mul_hi_u32", "v_mul_u32_u24", "v_add_co_u32", "v_add_u32"};

template <int OP, bool LAT = false>
void run(uint32_t* d, int cus, double ghz) {
  const int iters = 2000, waves_per_simd = LAT ? 1 : 8;
  const int blocks = cus * waves_per_simd;  // 256-thread block = 1 wave per SIMD
  hipLaunchKernelGGL((kop<OP, LAT>), dim3(blocks), dim3(256), 0, 0, d, 10);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((kop<OP, LAT>), dim3(blocks), dim3(256), 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double instr_per_simd = (double)waves_per_simd * iters * 64;  // wave-instructions per SIMD
  printf("%-16s %s %.3f ms  %.2f cycles/wave-instr/SIMD\n", NAMES[OP], LAT ? "dependent chain, 1 wave/SIMD" : "8 chains, 8 waves/SIMD", ms, ms * 1e-3 * ghz * 1e9 / instr_per_simd);
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 4096);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const double ghz = p.clockRate / 1e6;
  printf("CUs %d clock %.2f GHz\n", p.multiProcessorCount, ghz);
  run<0>(d, p.multiProcessorCount, ghz);
  run<1>(d, p.multiProcessorCount, ghz);
  run<2>(d, p.multiProcessorCount, ghz);
  run<3>(d, p.multiProcessorCount, ghz);
  run<4>(d, p.multiProcessorCount, ghz);
  run<5>(d, p.multiProcessorCount, ghz);
  run<6>(d, p.multiProcessorCount, ghz);
  run<7>(d, p.multiProcessorCount, ghz);
  run<8>(d, p.multiProcessorCount, ghz);
  run<9>(d, p.multiProcessorCount, ghz);
  run<10>(d, p.multiProcessorCount, ghz);
  run<11>(d, p.multiProcessorCount, ghz);
  run<12>(d, p.multiProcessorCount, ghz);
  run<7, true>(d, p.multiProcessorCount, ghz);
  run<0, true>(d, p.multiProcessorCount, ghz);
  run<1, true>(d, p.multiProcessorCount, ghz);
  run<3, true>(d, p.multiProcessorCount, ghz);
  run<4, true>(d, p.multiProcessorCount, ghz);
  return 0;
}
