// Device-side prime-field arithmetic for the MSM / NTT hot path (gfx950).
//
// Layout contract (SURVEY.md §8 preamble): elements are stored exactly as
// gnark-crypto stores fp.Element / fr.Element -- little-endian 64-bit limbs in
// Montgomery form x*R mod p with R = 2^(64*limbs).  Read as 32-bit words the
// same bytes are little-endian u32 limbs with the same R, so the kernels consume
// gnark's raw memory with zero conversion.
//
// Arithmetic is 32-bit-limb CIOS Montgomery multiplication built on
// v_mad_u64_u32.  All moduli here have a spare top bit (msw < 2^31 - 1), which
// allows the "no-carry" CIOS variant (no (N+1)-th accumulator word).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "field_constants.hpp"

namespace gm {

#define GM_DEV __device__ __forceinline__
#define GM_HD __host__ __device__ __forceinline__

// ---------------------------------------------------------------------------
// Field descriptors: N u32 limbs + constants returned by constexpr accessors so
// that fully-unrolled loops fold every modulus word into an instruction literal.
// ---------------------------------------------------------------------------
#define GM_DEFINE_FIELD(NAME, TAG, NLIMBS)                                        \
  struct NAME {                                                                   \
    static constexpr int N = NLIMBS;                                              \
    static constexpr int BITS = GM_##TAG##_BITS;                                  \
    static constexpr uint32_t INV = GM_##TAG##_INV32;                             \
    GM_HD static constexpr uint32_t p(int i) {                                    \
      constexpr uint32_t a[NLIMBS] = GM_##TAG##_P32;                              \
      return a[i];                                                                \
    }                                                                             \
    GM_HD static constexpr uint32_t one(int i) {                                  \
      constexpr uint32_t a[NLIMBS] = GM_##TAG##_ONE32;                            \
      return a[i];                                                                \
    }                                                                             \
    GM_HD static constexpr uint32_t r2(int i) {                                   \
      constexpr uint32_t a[NLIMBS] = GM_##TAG##_R2_32;                            \
      return a[i];                                                                \
    }                                                                             \
    /* limbs of p - 2 (Fermat exponent), borrow propagated */                     \
    GM_HD static constexpr uint32_t pm2(int i) {                                  \
      uint64_t borrow = 2;                                                        \
      for (int k = 0;; k++) {                                                     \
        const uint64_t v = (uint64_t)p(k) - borrow;                               \
        if (k == i) return (uint32_t)v;                                           \
        borrow = (v >> 63) & 1;                                                   \
      }                                                                           \
    }                                                                             \
  };

GM_DEFINE_FIELD(Bn254Fp, BN254_FP, 8)
GM_DEFINE_FIELD(Bn254Fr, BN254_FR, 8)
GM_DEFINE_FIELD(Bls377Fp, BLS12377_FP, 12)
GM_DEFINE_FIELD(Bls377Fr, BLS12377_FR, 8)

template <class P>
struct Fe {
  static constexpr int N = P::N;
  uint32_t v[P::N];
};

// --- carry helpers -----------------------------------------------------------
GM_DEV uint32_t add_cc(uint32_t a, uint32_t b, uint32_t& carry) {
  uint64_t s = (uint64_t)a + b + carry;
  carry = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
GM_DEV uint32_t sub_bb(uint32_t a, uint32_t b, uint32_t& borrow) {
  uint64_t d = (uint64_t)a - b - borrow;
  borrow = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

template <class P>
GM_DEV Fe<P> fe_zero() {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = 0;
  return r;
}
template <class P>
GM_DEV Fe<P> fe_one() {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = P::one(i);
  return r;
}
template <class P>
GM_DEV bool fe_is_zero(const Fe<P>& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) acc |= a.v[i];
  return acc == 0;
}
template <class P>
GM_DEV bool fe_eq(const Fe<P>& a, const Fe<P>& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) acc |= a.v[i] ^ b.v[i];
  return acc == 0;
}

// r = a - p if a >= p  (a < 2p)
template <class P>
GM_DEV void fe_reduce_once(Fe<P>& a) {
  Fe<P> t;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) t.v[i] = sub_bb(a.v[i], P::p(i), borrow);
  // borrow == 0  <=> a >= p  -> take t
#pragma unroll
  for (int i = 0; i < P::N; i++) a.v[i] = borrow ? a.v[i] : t.v[i];
}

template <class P>
GM_DEV Fe<P> fe_add(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = add_cc(a.v[i], b.v[i], c);
  fe_reduce_once(r);  // spare top bit: a+b < 2p < 2^(32N), no overflow word
  return r;
}

template <class P>
GM_DEV Fe<P> fe_sub(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = sub_bb(a.v[i], b.v[i], borrow);
  // if borrow, add p back
  uint32_t mask = 0u - borrow;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = add_cc(r.v[i], P::p(i) & mask, c);
  return r;
}

template <class P>
GM_DEV Fe<P> fe_dbl(const Fe<P>& a) {
  return fe_add(a, a);
}

template <class P>
GM_DEV Fe<P> fe_neg(const Fe<P>& a) {
  Fe<P> r;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = sub_bb(P::p(i), a.v[i], borrow);
  const bool z = fe_is_zero(a);
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = z ? 0u : r.v[i];
  return r;
}

// CIOS Montgomery multiplication, no-carry variant (requires p.msw < 2^31-1).
// Plain C: the compiler owns every carry and inserts the gfx950 VALU->carry
// hazard padding itself.
template <class P>
GM_DEV Fe<P> fe_mul(const Fe<P>& a, const Fe<P>& b) {
  constexpr int N = P::N;
  uint32_t t[N];
#pragma unroll
  for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint64_t acc = (uint64_t)a.v[0] * b.v[i] + t[0];
    t[0] = (uint32_t)acc;
    uint32_t C = (uint32_t)(acc >> 32);
#pragma unroll
    for (int j = 1; j < N; j++) {
      acc = (uint64_t)a.v[j] * b.v[i] + t[j] + C;
      t[j] = (uint32_t)acc;
      C = (uint32_t)(acc >> 32);
    }
    const uint32_t A = C;
    const uint32_t m = t[0] * P::INV;
    acc = (uint64_t)m * P::p(0) + t[0];
    C = (uint32_t)(acc >> 32);
#pragma unroll
    for (int j = 1; j < N; j++) {
      acc = (uint64_t)m * P::p(j) + t[j] + C;
      t[j - 1] = (uint32_t)acc;
      C = (uint32_t)(acc >> 32);
    }
    t[N - 1] = C + A;
  }
  Fe<P> r;
#pragma unroll
  for (int j = 0; j < N; j++) r.v[j] = t[j];
  fe_reduce_once(r);
  return r;
}

// acc(64) += a*b with the carry out of the 64-bit accumulator added to hi.
// v_mad_u64_u32 reports that carry in an SGPR pair; v_addc_co_u32 folds it in.
GM_DEV void mad_acc(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& hi) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
  asm("v_addc_co_u32 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(c) : "v"(hi), "s"(c));
}
GM_DEV void mad_acc_s(uint32_t a, uint32_t b_uniform, uint64_t& acc, uint32_t& hi) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "s"(b_uniform));
  asm("v_addc_co_u32 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(c) : "v"(hi), "s"(c));
}

// Finely-integrated product-scanning (FIPS) Montgomery multiplication:
// column k accumulates a_i*b_{k-i} and m_i*p_{k-i} into a 64-bit accumulator
// plus a carry word; 2N^2 v_mad_u64_u32 and no per-row carry propagation.
// EXPERIMENTAL / NOT USED: the carry hand-off between the two asm statements
// is a VALU-SGPR-write -> VALU-carry-read hazard that needs 2 wait states on
// gfx950, but hipcc only pads 1 around inline asm -> intermittent stale
// carries.  Kept for the microbenchmark until a hazard-safe form exists.
template <class P>
GM_DEV Fe<P> fe_mul_fips_asm(const Fe<P>& a, const Fe<P>& b) {
  constexpr int N = P::N;
  uint32_t m[N];
  Fe<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint32_t hi = 0;
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++)
      mad_acc(a.v[i], b.v[k - i], acc, hi);
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k - 1 < N - 1 ? k - 1 : N - 1); i++)
      mad_acc_s(m[i], P::p(k - i), acc, hi);
    if (k < N) {
      m[k] = (uint32_t)acc * P::INV;
      mad_acc_s(m[k], P::p(0), acc, hi);
    } else {
      r.v[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
  }
  r.v[N - 1] = (uint32_t)acc;
  fe_reduce_once(r);
  return r;
}

template <class P>
GM_DEV Fe<P> fe_sqr(const Fe<P>& a) {
  return fe_mul(a, a);
}

// Montgomery -> canonical integer (multiply by 1).
template <class P>
GM_DEV Fe<P> fe_from_mont(const Fe<P>& a) {
  Fe<P> one;
#pragma unroll
  for (int i = 0; i < P::N; i++) one.v[i] = (i == 0);
  return fe_mul(a, one);
}
// canonical -> Montgomery (multiply by R^2).
template <class P>
GM_DEV Fe<P> fe_to_mont(const Fe<P>& a) {
  Fe<P> r2;
#pragma unroll
  for (int i = 0; i < P::N; i++) r2.v[i] = P::r2(i);
  return fe_mul(a, r2);
}

// a^(p-2) (Fermat inversion; 0 -> 0).
template <class P>
GM_DEV Fe<P> fe_inv(const Fe<P>& a) {
  Fe<P> r = fe_one<P>();
  for (int i = P::N - 1; i >= 0; i--) {
    const uint32_t e = P::pm2(i);
    for (int b = 31; b >= 0; b--) {
      r = fe_sqr(r);
      if ((e >> b) & 1) r = fe_mul(r, a);
    }
  }
  return r;
}

// ---------------------------------------------------------------------------
// Quadratic extension Fp2 = Fp[u]/(u^2 - BETA).  BN254: BETA = -1;
// BLS12-377: BETA = -5 (gnark-crypto E2 layout: {A0, A1}).
// ---------------------------------------------------------------------------
template <class P, int BETA>
struct Fe2 {
  using Base = P;
  Fe<P> a0, a1;
};

template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_add(const Fe2<P, BETA>& a, const Fe2<P, BETA>& b) {
  return {fe_add(a.a0, b.a0), fe_add(a.a1, b.a1)};
}
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_sub(const Fe2<P, BETA>& a, const Fe2<P, BETA>& b) {
  return {fe_sub(a.a0, b.a0), fe_sub(a.a1, b.a1)};
}
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_dbl(const Fe2<P, BETA>& a) {
  return {fe_dbl(a.a0), fe_dbl(a.a1)};
}
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_neg(const Fe2<P, BETA>& a) {
  return {fe_neg(a.a0), fe_neg(a.a1)};
}
template <class P, int BETA>
GM_DEV bool fe_is_zero(const Fe2<P, BETA>& a) {
  return fe_is_zero(a.a0) && fe_is_zero(a.a1);
}
template <class P, int BETA>
GM_DEV Fe<P> mul_by_beta(const Fe<P>& x) {
  static_assert(BETA == -1 || BETA == -5, "unsupported non-residue");
  if constexpr (BETA == -1) {
    return fe_neg(x);
  } else {
    Fe<P> x2 = fe_dbl(x);
    Fe<P> x4 = fe_dbl(x2);
    return fe_neg(fe_add(x4, x));
  }
}
// Karatsuba: 3 base multiplications.
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_mul(const Fe2<P, BETA>& a, const Fe2<P, BETA>& b) {
  Fe<P> v0 = fe_mul(a.a0, b.a0);
  Fe<P> v1 = fe_mul(a.a1, b.a1);
  Fe<P> s = fe_mul(fe_add(a.a0, a.a1), fe_add(b.a0, b.a1));
  Fe2<P, BETA> r;
  r.a0 = fe_add(v0, mul_by_beta<P, BETA>(v1));
  r.a1 = fe_sub(fe_sub(s, v0), v1);
  return r;
}
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_sqr(const Fe2<P, BETA>& a) {
  // (a0 + a1 u)^2 = a0^2 + BETA a1^2 + 2 a0 a1 u
  Fe<P> v0 = fe_mul(a.a0, a.a0);
  Fe<P> v1 = fe_mul(a.a1, a.a1);
  Fe<P> c = fe_mul(a.a0, a.a1);
  Fe2<P, BETA> r;
  r.a0 = fe_add(v0, mul_by_beta<P, BETA>(v1));
  r.a1 = fe_dbl(c);
  return r;
}

template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_inv(const Fe2<P, BETA>& a) {
  // 1/(a0 + a1 u) = (a0 - a1 u) / (a0^2 - BETA a1^2)
  Fe<P> nrm = fe_sub(fe_sqr(a.a0), mul_by_beta<P, BETA>(fe_sqr(a.a1)));
  Fe<P> ni = fe_inv(nrm);
  return {fe_mul(a.a0, ni), fe_neg(fe_mul(a.a1, ni))};
}

}  // namespace gm
