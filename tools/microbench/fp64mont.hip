// Microbenchmark: BN254 Fp Montgomery product with 52-bit
// limbs held in doubles (exact 52x52 products from two v_fma_f64) against the
// radix-2^29 v_mad_u64_u32 product the kernels use (gm::fe_mul, lazy form).
//
// 52-bit product, f64 rounding toward zero (set once per wave in MODE):
//   h = fma(a, b, 2^104)            = 2^104 + H 2^52, H = floor(ab / 2^52)
//   s = (2^104 + 2^52) - h          = (1 - H) 2^52, exact
//   l = fma(a, b, s)                = 2^52 + L, L = ab mod 2^52, exact
// The bit patterns of h and l are EH + H and EL + L; the column accumulators add
// them as 64-bit integers and start from minus the offsets of every pattern they
// will receive, so no per-product fix-up is needed.  Every f64 instruction is
// inline asm: the compiler's mode-register pass would otherwise put the default
// rounding back in front of the first f64 instruction it sees.  (Round to nearest
// instead needs a fourth f64 op per product: L is then signed, and no single
// exact addend maps it into one binade.)
// Montgomery: product scanning over 5 limbs (R = 2^260 > 4p: inputs < 2p give
// outputs < 2p, no conditional subtraction), m_k = (t_k * -p^-1) mod 2^52 by the
// same exact product.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/fp64mont tools/microbench/fp64mont.hip
//   /tmp/fp64mont /tmp/fp64mont_dump.txt && python3 tools/microbench/fp64mont_check.py /tmp/fp64mont_dump.txt
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
#include "../../gnark-icicle_amd/csrc/field.hpp"

namespace {

constexpr double C1 = 0x1p104;
constexpr double C3 = 0x1p104 + 0x1p52;
constexpr uint64_t EH = 0x4670000000000000ull;  // bits of 2^104
constexpr uint64_t EL = 0x4330000000000000ull;  // bits of 2^52
constexpr uint64_t M52 = (1ull << 52) - 1;
constexpr uint64_t P52[5] = {0x8c16d87cfd47ull, 0x916871ca8d3c2ull, 0x181585d97816aull, 0xa029b85045b68ull,
                             0x30644e72e131ull};
constexpr uint64_t PINV52 = 0x20782e4866389ull;  // -p^-1 mod 2^52

struct F52 {
  double v[5];
};

constexpr int cnt(int k) { return k < 0 || k > 8 ? 0 : (k < 5 ? k + 1 : 9 - k); }

__device__ __forceinline__ void set_f64_round_toward_zero() {
  // MODE.FP_ROUND[3:2] (f64 / f16) = 3: toward zero
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3");
}
__device__ __forceinline__ double fma_f64(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ double sub_f64(double a, double b) {
  double r;
  asm("v_add_f64 %0, %1, -%2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// one asm block per product: the hazard recognizer pads every inline-asm
// boundary with s_nop, so fewer, larger blocks keep the count honest
__device__ __forceinline__ void pr(double a, double b, uint64_t& lo, uint64_t& hi) {
  double h, l;
  asm("v_fma_f64 %[h], %[a], %[b], %[c1]\n\t"
      "v_add_f64 %[l], %[c3], -%[h]\n\t"
      "v_fma_f64 %[l], %[a], %[b], %[l]\n\t"
      "v_lshl_add_u64 %[hi], %[h], 0, %[hi]\n\t"
      "v_lshl_add_u64 %[lo], %[l], 0, %[lo]"
      : [h] "=&v"(h), [l] "=&v"(l), [lo] "+v"(lo), [hi] "+v"(hi)
      : [a] "v"(a), [b] "v"(b), [c1] "s"(C1), [c3] "s"(C3));
}

// integer in [0, 2^52) -> double
__device__ __forceinline__ double to_d(uint64_t x) { return sub_f64(__longlong_as_double((long long)(x | EL)), 0x1p52); }

__device__ __forceinline__ F52 mont52(const F52& a, const F52& b) {
  uint64_t acc[10];
#pragma unroll
  for (int k = 0; k < 10; k++) acc[k] = 0ull - (uint64_t)(2 * cnt(k)) * EL - (uint64_t)(2 * cnt(k - 1)) * EH;
  double m[5];
  F52 r;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int lo = k - 4 > 0 ? k - 4 : 0, hi = k < 4 ? k : 4;
#pragma unroll
    for (int i = lo; i <= hi; i++) pr(a.v[i], b.v[k - i], acc[k], acc[k + 1]);
#pragma unroll
    for (int i = lo; i <= (k - 1 < 4 ? k - 1 : 4); i++) pr(m[i], (double)P52[k - i], acc[k], acc[k + 1]);
    if (k < 5) {
      // low 52 bits of the column (the pending m_k p_0 pattern's offset EL has
      // zero low bits); m_k = t (-p^-1) mod 2^52 by the same exact product
      const double t = to_d(acc[k] & M52);
      const double h = fma_f64(t, (double)PINV52, C1);
      m[k] = sub_f64(fma_f64(t, (double)PINV52, sub_f64(C3, h)), 0x1p52);
      pr(m[k], (double)P52[0], acc[k], acc[k + 1]);
    } else {
      r.v[k - 5] = to_d(acc[k] & M52);
    }
    acc[k + 1] += acc[k] >> 52;
  }
  r.v[4] = to_d(acc[9]);
  return r;
}

__global__ void __launch_bounds__(256) k_check52(const double* a, const double* b, double* out, int n) {
  set_f64_round_toward_zero();
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  F52 x, y;
  for (int i = 0; i < 5; i++) x.v[i] = a[5 * t + i], y.v[i] = b[5 * t + i];
  F52 z = mont52(x, y);
  z = mont52(z, y);  // chained: z = x y^2 / R^2, input < 2p exercised
  for (int i = 0; i < 5; i++) out[5 * t + i] = z.v[i];
}

// throughput: two dependent chains per thread, as tools/microbench/mul29.hip
__global__ void __launch_bounds__(256) k_rate52(const double* a, const double* b, double* out, int n, int iters) {
  set_f64_round_toward_zero();
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = t % n;
  F52 x, y;
  for (int i = 0; i < 5; i++) x.v[i] = a[5 * s + i], y.v[i] = b[5 * s + i];
  F52 c = y;
  for (int k = 0; k < iters; k++) {
    x = mont52(x, y);
    c = mont52(c, x);
  }
  uint64_t q = 0;
  for (int i = 0; i < 5; i++) q ^= (uint64_t)__double_as_longlong(x.v[i]) ^ (uint64_t)__double_as_longlong(c.v[i]);
  if (q == 1) out[0] = 1.0;
}

__global__ void __launch_bounds__(256) k_rate29(const uint32_t* a, uint32_t* out, int n, int iters) {
  using gm::Fe;
  using gm::Bn254Fp;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = t % n;
  Fe<Bn254Fp> x, y;
  for (int i = 0; i < Bn254Fp::N; i++) x.v[i] = a[(s * Bn254Fp::N + i) % 4096] & 0x0fffffff, y.v[i] = x.v[i] ^ 0x0abcdef;
  x.v[Bn254Fp::N - 1] &= 0xfffff, y.v[Bn254Fp::N - 1] &= 0xfffff;
  Fe<Bn254Fp> c = y;
  for (int k = 0; k < iters; k++) {
    x = gm::fe_mul<Bn254Fp, false>(x, y);
    c = gm::fe_mul<Bn254Fp, false>(c, x);
  }
  uint32_t q = 0;
  for (int i = 0; i < Bn254Fp::N; i++) q ^= x.v[i] ^ c.v[i];
  if (q == 0x12345678u) out[0] = q;
}

double to_double_limb(uint64_t x) { return (double)x; }

}  // namespace

int main(int argc, char** argv) {
  const char* dump = argc > 1 ? argv[1] : "/tmp/fp64mont_dump.txt";
  const int n = 4096;
  std::mt19937_64 rng(2026);
  std::vector<double> ha(5 * n), hb(5 * n), hout(5 * n);
  std::vector<uint32_t> h29(4096);
  for (auto& v : h29) v = (uint32_t)rng();
  for (int t = 0; t < n; t++)
    for (double* dst : {&ha[5 * t], &hb[5 * t]}) {
      uint64_t w[4] = {rng(), rng(), rng(), rng() & ((1ull << 61) - 1)};  // < 2^253 < p
      if (t < 4) {  // edge values: 0, 1, 2^253 - 1
        for (auto& x : w) x = 0;
        if (t == 1) w[0] = 1;
        if (t >= 2) w[0] = w[1] = w[2] = ~0ull, w[3] = (1ull << 61) - 1;
      }
      for (int i = 0; i < 5; i++) {
        const int bit = 52 * i, q = bit / 64, o = bit % 64;
        uint64_t x = w[q] >> o;
        if (o > 12 && q + 1 < 4) x |= w[q + 1] << (64 - o);
        dst[i] = to_double_limb(x & M52);
      }
    }
  double *da, *db, *dout;
  uint32_t *d29, *dsink;
  if (hipMalloc(&da, 8 * ha.size()) || hipMalloc(&db, 8 * hb.size()) || hipMalloc(&dout, 8 * hout.size()) ||
      hipMalloc(&d29, 4 * 4096) || hipMalloc(&dsink, 64))
    return 1;
  (void)hipMemcpy(da, ha.data(), 8 * ha.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb.data(), 8 * hb.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(d29, h29.data(), 4 * 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_check52, dim3(n / 256), dim3(256), 0, 0, da, db, dout, n);
  if (hipDeviceSynchronize()) return 2;
  (void)hipMemcpy(hout.data(), dout, 8 * hout.size(), hipMemcpyDeviceToHost);
  FILE* f = fopen(dump, "w");
  if (!f) return 3;
  for (int t = 0; t < n; t++) {
    for (const auto* v : {&ha, &hb, &hout}) {
      for (int i = 0; i < 5; i++) fprintf(f, "%s%llx", i ? "," : "", (unsigned long long)(*v)[5 * t + i]);
      fprintf(f, t >= 0 && v == &hout ? "\n" : " ");
    }
  }
  fclose(f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = 256 * 8 * 4, iters = 256;  // 8 waves per SIMD worth of threads per CU
  for (int rep = 0; rep < 3; rep++) {
    float ms52, ms29;
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate52, dim3(grid), dim3(256), 0, 0, da, db, dout, n, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms52, e0, e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate29, dim3(grid), dim3(256), 0, 0, d29, dsink, n, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms29, e0, e1);
    const double muls = 2.0 * iters * grid * 256;
    printf("fp64 52-bit Montgomery: %.3f ms  %.1f Gmul/s | radix-2^29 fe_mul (lazy): %.3f ms  %.1f Gmul/s\n", ms52,
           muls / ms52 / 1e6, ms29, muls / ms29 / 1e6);
  }
  return hipDeviceSynchronize() ? 4 : 0;
}
