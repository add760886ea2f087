// Device-side prime-field arithmetic for the MSM / NTT hot path (gfx950).
//
// Two representations of an element x of F_p:
//
//  * gnark layout (HBM, C-ABI): exactly gnark-crypto's fp.Element / fr.Element --
//    little-endian 64-bit limbs in Montgomery form x*Rg mod p, Rg = 2^(64*limbs).
//    Read as NG little-endian u32 words.  Points, scalars and NTT vectors cross
//    the boundary in this form, byte for byte.
//
//  * internal (registers / LDS / device scratch): N unsaturated 29-bit limbs
//    (radix 2^29, one limb per u32) in Montgomery form x*R' mod p,
//    R' = 2^(29N) (N = 9 for the 254/253-bit fields, 14 for BLS12-377 Fp).
//    Values are kept canonical (< p, every limb < 2^29).
//
// Why radix 2^29: a finely-integrated product-scanning Montgomery product then
// accumulates every column (<= 2N products of 58 bits) in one 64-bit register
// with v_mad_u64_u32 and no carry flags at all -- no VALU->VCC carry chains
// (which need 2 hazard wait states each on gfx950) and no 32-bit carry-word
// shuffling.  Measured 147-159 Gmul/s vs 87-96 for 32-bit CIOS on MI355X
// (tools/microbench/mul29.hip).
//
// Mixed-form identity used by the NTT: mul(a_gnark, w_internal) = a*w in gnark
// form (x*Rg * w*R' / R' = (x*w)*Rg), so NTT data never needs converting.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "field_constants.hpp"

namespace gm {

#define GM_DEV __device__ __forceinline__
#define GM_HD __host__ __device__ __forceinline__

constexpr int RADIX = 29;
constexpr uint32_t LIMB_MASK = (1u << RADIX) - 1;

#define GM_CONST_ARRAY_FN(FN, N, INIT)       \
  GM_HD static constexpr uint32_t FN(int i) { \
    constexpr uint32_t a[N] = INIT;           \
    return a[i];                              \
  }

#define GM_DEFINE_FIELD(NAME, TAG)                                              \
  struct NAME {                                                                 \
    static constexpr int N = GM_##TAG##_N29;  /* radix-2^29 limbs */            \
    static constexpr int NG = GM_##TAG##_NG;  /* gnark u32 words */             \
    static constexpr int BITS = GM_##TAG##_BITS;                                \
    static constexpr uint32_t INV = GM_##TAG##_INV29;                           \
    GM_CONST_ARRAY_FN(p, GM_##TAG##_N29, GM_##TAG##_P29)                        \
    GM_CONST_ARRAY_FN(one, GM_##TAG##_N29, GM_##TAG##_ONE29)                    \
    GM_CONST_ARRAY_FN(r2, GM_##TAG##_N29, GM_##TAG##_R229)                      \
    GM_CONST_ARRAY_FN(kin, GM_##TAG##_N29, GM_##TAG##_KIN29)                    \
    GM_CONST_ARRAY_FN(kout, GM_##TAG##_N29, GM_##TAG##_KOUT29)                  \
    GM_CONST_ARRAY_FN(kcan, GM_##TAG##_N29, GM_##TAG##_KCAN29)                  \
    GM_CONST_ARRAY_FN(kgn, GM_##TAG##_N29, GM_##TAG##_KGN29)                    \
    GM_CONST_ARRAY_FN(pg, GM_##TAG##_NG, GM_##TAG##_P32)                        \
    /* u32 words of p - 2 (Fermat exponent), borrow propagated */               \
    GM_HD static constexpr uint32_t pm2(int i) {                                \
      uint64_t borrow = 2;                                                      \
      for (int k = 0;; k++) {                                                   \
        const uint64_t v = (uint64_t)pg(k) - borrow;                            \
        if (k == i) return (uint32_t)v;                                         \
        borrow = (v >> 63) & 1;                                                 \
      }                                                                         \
    }                                                                           \
  };

GM_DEFINE_FIELD(Bn254Fp, BN254_FP)
GM_DEFINE_FIELD(Bn254Fr, BN254_FR)
GM_DEFINE_FIELD(Bls377Fp, BLS12377_FP)
GM_DEFINE_FIELD(Bls377Fr, BLS12377_FR)

template <class P>
struct Fe {
  static constexpr int N = P::N;
  uint32_t v[P::N];
};

// Packed gnark-layout words of one element (NG u32).
template <class P>
struct FeG {
  uint32_t w[P::NG];
};

#define GM_FE_CONST(P, FN)                                                    \
  ([]() {                                                                     \
    ::gm::Fe<P> r_;                                                           \
    _Pragma("unroll") for (int i_ = 0; i_ < P::N; i_++) r_.v[i_] = P::FN(i_); \
    return r_;                                                                \
  }())

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

// ---------------------------------------------------------------------------
// pack / unpack between NG x u32 (gnark words) and N x 29-bit limbs (same
// integer; no field conversion).  Fully unrolled bit plumbing.
// ---------------------------------------------------------------------------
template <class P>
GM_DEV Fe<P> fe_unpack(const FeG<P>& g) {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const int bit = RADIX * i, w = bit >> 5, s = bit & 31;
    const uint32_t lo = (w < P::NG) ? g.w[w] : 0u;
    const uint32_t hi = (w + 1 < P::NG) ? g.w[w + 1] : 0u;
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    r.v[i] = (uint32_t)(x >> s) & LIMB_MASK;
  }
  return r;
}
template <class P>
GM_DEV FeG<P> fe_pack(const Fe<P>& a) {
  FeG<P> g;
#pragma unroll
  for (int j = 0; j < P::NG; j++) {
    const int bit = 32 * j, i0 = bit / RADIX, s0 = bit % RADIX;
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int i = i0 + k;
      if (i < P::N) {
        const int sh = RADIX * k - s0;
        if (sh >= 0) x |= (uint64_t)a.v[i] << sh;
        else x |= (uint64_t)a.v[i] >> (-sh);
      }
    }
    g.w[j] = (uint32_t)x;
  }
  return g;
}

// vectorised loads / stores of gnark words (16 B, then an 8 B tail)
template <class P>
GM_DEV FeG<P> feg_load(const uint32_t* __restrict__ src) {
  FeG<P> g;
  static_assert(P::NG % 2 == 0, "gnark elements are whole u64 limbs");
#pragma unroll
  for (int q = 0; q < P::NG / 4; q++) {
    const uint4 v = reinterpret_cast<const uint4*>(src)[q];
    g.w[4 * q] = v.x;
    g.w[4 * q + 1] = v.y;
    g.w[4 * q + 2] = v.z;
    g.w[4 * q + 3] = v.w;
  }
  if constexpr (P::NG % 4 != 0) {
    const uint2 v = reinterpret_cast<const uint2*>(src)[P::NG / 2 - 1];
    g.w[P::NG - 2] = v.x;
    g.w[P::NG - 1] = v.y;
  }
  return g;
}
template <class P>
GM_DEV void feg_store(uint32_t* __restrict__ dst, const FeG<P>& g) {
#pragma unroll
  for (int q = 0; q < P::NG / 4; q++)
    reinterpret_cast<uint4*>(dst)[q] = make_uint4(g.w[4 * q], g.w[4 * q + 1], g.w[4 * q + 2], g.w[4 * q + 3]);
  if constexpr (P::NG % 4 != 0)
    reinterpret_cast<uint2*>(dst)[P::NG / 2 - 1] = make_uint2(g.w[P::NG - 2], g.w[P::NG - 1]);
}
// element idx of a gnark-layout array: unpacked, still in gnark form
template <class P>
GM_DEV Fe<P> fe_load_g(const void* base, size_t idx) {
  return fe_unpack<P>(feg_load<P>(reinterpret_cast<const uint32_t*>(base) + idx * P::NG));
}
template <class P>
GM_DEV void fe_store_g(void* base, size_t idx, const Fe<P>& a) {
  feg_store<P>(reinterpret_cast<uint32_t*>(base) + idx * P::NG, fe_pack(a));
}

// ---------------------------------------------------------------------------
// arithmetic on canonical internal elements
// ---------------------------------------------------------------------------
// a - p if a >= p (a < 2p, limbs < 2^29)
template <class P>
GM_DEV void fe_reduce_once(Fe<P>& a) {
  Fe<P> t;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const int32_t d = (int32_t)a.v[i] - (int32_t)P::p(i) + borrow;
    borrow = d >> RADIX;  // 0 or -1
    t.v[i] = (uint32_t)d & LIMB_MASK;
  }
  const bool ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) a.v[i] = ge ? t.v[i] : a.v[i];
}

template <class P>
GM_DEV Fe<P> fe_add(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = s & LIMB_MASK;
    c = s >> RADIX;
  }
  fe_reduce_once(r);  // a + b < 2p < R'
  return r;
}

template <class P>
GM_DEV Fe<P> fe_sub(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const int32_t d = (int32_t)a.v[i] - (int32_t)b.v[i] + borrow;
    borrow = d >> RADIX;
    r.v[i] = (uint32_t)d & LIMB_MASK;
  }
  // negative -> add p back
  const uint32_t msk = (uint32_t)borrow;  // 0 or 0xffffffff
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const uint32_t s = r.v[i] + (P::p(i) & msk) + c;
    r.v[i] = s & LIMB_MASK;
    c = s >> RADIX;
  }
  return r;
}

template <class P>
GM_DEV Fe<P> fe_dbl(const Fe<P>& a) {
  return fe_add(a, a);
}

template <class P>
GM_DEV Fe<P> fe_neg(const Fe<P>& a) {
  return fe_sub(fe_zero<P>(), a);
}

// Finely-integrated product-scanning Montgomery product in radix 2^29:
// column k accumulates a_i b_{k-i} + m_i p_{k-i} (< 2N * 2^58 < 2^64) in one
// 64-bit register; m_k = (acc * (-p^-1)) mod 2^29 zeroes the low limb.
// Inputs < p  ->  result < 2p -> one conditional subtraction -> canonical.
// CHAIN: every column starts from the carry of the previous one (an opaque
// register barrier stops the compiler from summing the next column separately
// and adding the carry with a 64-bit add, v_lshl_add_u64, per column).  One
// dependent mad chain per product: for kernels with several independent
// products in flight per thread (the radix-4 NTT rounds).
#ifndef GM_FE_CHAIN
#define GM_FE_CHAIN 0
#endif
// CHAIN levels of the products below: 0 -- the compiler's schedule; 1 -- one
// mad chain per column (a register barrier between columns); 2 -- strict: every
// mad takes the previous one's result as its addend (a barrier after each), so
// no column is summed in a second register pair and joined with a 64-bit add
// (v_lshl_add_u64), and squarings double an operand instead of shifting the
// cross sum.  Level 2 costs one wait state per dependent mad (s_nop 0, hidden by
// the other waves).
#define GM_STRICT_STEP(acc, CH) \
  do {                              \
    if constexpr ((CH) >= 2) __asm__ volatile("" : "+v"(acc)); \
  } while (0)
template <class P, bool REDUCE = true, int CHAIN = GM_FE_CHAIN>
GM_DEV Fe<P> fe_mul(const Fe<P>& a, const Fe<P>& b) {
  constexpr int N = P::N;
  uint32_t m[N];
  Fe<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    if constexpr (CHAIN) {
      if (k) __asm__ volatile("" : "+v"(acc));
    }
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      GM_STRICT_STEP(acc, CHAIN);
    }
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k - 1 < N - 1 ? k - 1 : N - 1); i++) {
      acc += (uint64_t)m[i] * P::p(k - i);
      GM_STRICT_STEP(acc, CHAIN);
    }
    if (k < N) {
      m[k] = ((uint32_t)acc * P::INV) & LIMB_MASK;
      acc += (uint64_t)m[k] * P::p(0);
    } else {
      r.v[k - N] = (uint32_t)acc & LIMB_MASK;
    }
    acc >>= RADIX;
  }
  r.v[N - 1] = (uint32_t)acc;
  if constexpr (REDUCE) fe_reduce_once(r);
  return r;
}

// Squaring: the symmetric products a_i a_j (i != j) are formed once and doubled.
template <class P, bool REDUCE = true, int CHAIN = GM_FE_CHAIN>
GM_DEV Fe<P> fe_sqr(const Fe<P>& a) {
  constexpr int N = P::N;
  uint32_t m[N];
  Fe<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    if constexpr (CHAIN) {
      if (k) __asm__ volatile("" : "+v"(acc));
    }
    if constexpr (CHAIN >= 2) {
      // 2 a_i a_j as a_i (2 a_j): 2 a_j < 2^30, the column stays below 2^64
#pragma unroll
      for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++) {
        const int j = k - i;
        if (i < j) {
          acc += (uint64_t)a.v[i] * (a.v[j] << 1);
          GM_STRICT_STEP(acc, CHAIN);
        }
      }
    } else {
      uint64_t cross = 0;
#pragma unroll
      for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++) {
        const int j = k - i;
        if (i < j) cross += (uint64_t)a.v[i] * a.v[j];
      }
      acc += cross << 1;
    }
    if ((k & 1) == 0) {
      acc += (uint64_t)a.v[k / 2] * a.v[k / 2];
      GM_STRICT_STEP(acc, CHAIN);
    }
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k - 1 < N - 1 ? k - 1 : N - 1); i++) {
      acc += (uint64_t)m[i] * P::p(k - i);
      GM_STRICT_STEP(acc, CHAIN);
    }
    if (k < N) {
      m[k] = ((uint32_t)acc * P::INV) & LIMB_MASK;
      acc += (uint64_t)m[k] * P::p(0);
    } else {
      r.v[k - N] = (uint32_t)acc & LIMB_MASK;
    }
    acc >>= RADIX;
  }
  r.v[N - 1] = (uint32_t)acc;
  if constexpr (REDUCE) fe_reduce_once(r);
  return r;
}

// ---------------------------------------------------------------------------
// Lazily reduced arithmetic (MSM bucket accumulation hot loop).
// Values are kept as representatives in [0, k p) with normalised 29-bit limbs
// instead of canonical [0, p): the Montgomery product returns
//   (ab + Mp) / R' < ab / R' + p,   M < R' = 2^(29N),
// so with ab < R' p its output is already < 2p and the final conditional
// subtraction (a third of the product's non-multiply instructions) can go.
// fe_sub_lz<K> adds K p instead of testing the sign.  The accumulation keeps
// x < 8p, y < 4p, zz, zzz < 2p and every product input pair satisfies
// ab <= 100 p^2 < R' p, which needs R' / p > 100 (static_assert in the caller:
// BITS + 7 <= 29 N, i.e. R' / p > 128; BN254 Fp: 254 + 7 = 261 = 29 * 9).
// ---------------------------------------------------------------------------
// limb i of K*p, normalised radix 2^29 (the top limb keeps any excess)
template <class P, int K>
GM_HD constexpr uint32_t kp_limb(int i) {
  uint64_t carry = 0;
  for (int j = 0; j < P::N; j++) {
    const uint64_t v = (uint64_t)P::p(j) * K + carry;
    if (j == i) return j == P::N - 1 ? (uint32_t)v : (uint32_t)(v & LIMB_MASK);
    carry = v >> RADIX;
  }
  return 0;
}
// top limb of j*p (j < 16)
template <class P>
GM_HD constexpr uint32_t kp_top(int j) {
  uint64_t carry = 0, v = 0;
  for (int i = 0; i < P::N; i++) {
    v = (uint64_t)P::p(i) * (uint64_t)j + carry;
    carry = v >> RADIX;
  }
  return (uint32_t)v;
}
template <class P>
GM_DEV Fe<P> fe_mul_lz(const Fe<P>& a, const Fe<P>& b) { return fe_mul<P, false>(a, b); }
template <class P>
GM_DEV Fe<P> fe_mul_lz_chain(const Fe<P>& a, const Fe<P>& b) { return fe_mul<P, false, true>(a, b); }
template <class P>
GM_DEV Fe<P> fe_sqr_lz(const Fe<P>& a) { return fe_sqr<P, false>(a); }
// Unsigned Montgomery reduction of x1*y1 + x2*y2 (radix 2^29 product scanning,
// one 64-bit column accumulator, no signs).  A difference x1 y1 - x y2 is
// computed as x1 y1 + (K p - x) y2 with the carry-free operand fe_negk_cf<K>(x):
// the G1 add's Y3 = R (Q - X3) - Y1 PPP (one reduction instead of two), and the
// lane-pair Fp2 product, whose two lanes then run the same instructions.  Column bound:
// N (2^58 + 2^59 + 2^58) < 2^64 for N <= 14 with x1, y1, y2 normalised and x2
// limbs < 2^30.  Output < (x1 y1 + x2 y2) / R' + p, limbs normalised.
template <class P, int CHAIN = GM_FE_CHAIN>
GM_DEV Fe<P> fe_mul2_redc_u(const Fe<P>& x1, const Fe<P>& y1, const Fe<P>& x2, const Fe<P>& y2) {
  constexpr int N = P::N;
  static_assert(N <= 14, "unsigned two-product column bound");
  uint32_t m[N];
  Fe<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    if constexpr (CHAIN) {
      if (k) __asm__ volatile("" : "+v"(acc));
    }
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++) {
      acc += (uint64_t)x1.v[i] * y1.v[k - i];
      GM_STRICT_STEP(acc, CHAIN);
      acc += (uint64_t)x2.v[i] * y2.v[k - i];
      GM_STRICT_STEP(acc, CHAIN);
    }
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k - 1 < N - 1 ? k - 1 : N - 1); i++) {
      acc += (uint64_t)m[i] * P::p(k - i);
      GM_STRICT_STEP(acc, CHAIN);
    }
    if (k < N) {
      m[k] = ((uint32_t)acc * P::INV) & LIMB_MASK;
      acc += (uint64_t)m[k] * P::p(0);
    } else {
      r.v[k - N] = (uint32_t)acc & LIMB_MASK;
    }
    acc >>= RADIX;
  }
  r.v[N - 1] = (uint32_t)acc;
  return r;
}

// a + b, no reduction (limbs normalised)
template <class P>
GM_DEV Fe<P> fe_add_lz(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = i == P::N - 1 ? s : (s & LIMB_MASK);
    c = s >> RADIX;
  }
  return r;
}
// a - b + K p  (requires b < K p; the result is < a + K p)
template <int K, class P>
GM_DEV Fe<P> fe_sub_lz(const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const int32_t d = (int32_t)(a.v[i] + kp_limb<P, K>(i)) - (int32_t)b.v[i] + c;
    c = d >> RADIX;
    r.v[i] = i == P::N - 1 ? (uint32_t)d : ((uint32_t)d & LIMB_MASK);
  }
  return r;
}
// a - K p if a >= K p
template <int K, class P>
GM_DEV void fe_reduce_k(Fe<P>& a) {
  Fe<P> t;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const int32_t d = (int32_t)a.v[i] - (int32_t)kp_limb<P, K>(i) + borrow;
    borrow = d >> RADIX;
    t.v[i] = (uint32_t)d & LIMB_MASK;
  }
  const bool ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) a.v[i] = ge ? t.v[i] : a.v[i];
}
// Limb i of 2p in "borrowed" form: each limb below the top takes 2^29 - 1 from
// its upper neighbour (limb 0: 2^29), so c_i >= s_i for every normalised s < 2p
// and c - s needs no carries.  Same integer as 2p.
template <class P>
GM_HD constexpr uint32_t p2_borrowed_limb(int i) {
  return i == 0 ? kp_limb<P, 2>(0) + (1u << RADIX)
                : (i == P::N - 1 ? kp_limb<P, 2>(i) - 1u : kp_limb<P, 2>(i) + (1u << RADIX) - 1u);
}
// Limb i of K p in borrowed form (as p2_borrowed_limb): every limb below the
// top is >= 2^29 - 1, so K p - s needs no carries for normalised s.
template <class P, int K>
GM_HD constexpr uint32_t kp_borrowed_limb(int i) {
  return i == 0 ? kp_limb<P, K>(0) + (1u << RADIX)
                : (i == P::N - 1 ? kp_limb<P, K>(i) - 1u : kp_limb<P, K>(i) + (1u << RADIX) - 1u);
}
// K p - s for s < (K - 1) p with normalised limbs, carry-free (one VOP2 per
// limb): limbs < 2^30, the top limb non-negative (s's top limb is at least p's
// top limb below K p's).  A product operand (fe_mul2_redc_u's x2), not a
// canonical value.
template <int K, class P>
GM_DEV Fe<P> fe_negk_cf(const Fe<P>& s) {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = kp_borrowed_limb<P, K>(i) - s.v[i];
  return r;
}
// a - b + K p as a product operand only, carry-free (two VOP2 per limb instead of
// fe_sub_lz's signed carry pass): a, b normalised, b < (K - 1) p.  The limbs are
// left unnormalised, < 3 2^29, which a Montgomery product's 64-bit columns
// absorb next to a normalised second operand (9 N 2^58 + N 2^58 < 2^64 for
// N <= 11); the value, < a + K p, is what fe_sub_lz<K> returns.
template <int K, class P>
GM_DEV Fe<P> fe_sub_cf(const Fe<P>& a, const Fe<P>& b) {
  static_assert(P::N <= 11, "unnormalised product operand column bound");
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = a.v[i] + (kp_borrowed_limb<P, K>(i) - b.v[i]);
  return r;
}
// neg ? 2p - s : s for s < 2p with normalised limbs, carry-free (2 VOP2 per limb
// instead of a borrow chain plus a masked add of p).  The limbs of 2p - s are left
// unnormalised (< 2^30; the top limb may read -1 as int32): the result may only
// feed fe_sub_lz / fe_sub2x_lz as their minuend, whose signed carry pass
// normalises it.  Value in (0, 2p].
template <class P>
GM_DEV Fe<P> fe_cneg2p_cf(const Fe<P>& s, bool neg) {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = neg ? p2_borrowed_limb<P>(i) - s.v[i] : s.v[i];
  return r;
}
// a - b - 2c + K p in one signed carry pass (b + 2c < K p; b, c normalised, a as
// fe_sub_lz accepts it).  Replaces sub_lz(sub_lz(a, b), add_lz(c, c)): one
// borrow chain instead of three.  The result is < a + K p.
template <int K, class P>
GM_DEV Fe<P> fe_sub2x_lz(const Fe<P>& a, const Fe<P>& b, const Fe<P>& c) {
  Fe<P> r;
  int32_t cy = 0;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    const int32_t d = (int32_t)(a.v[i] + kp_limb<P, K>(i)) - (int32_t)(b.v[i] + (c.v[i] << 1)) + cy;
    cy = d >> RADIX;
    r.v[i] = i == P::N - 1 ? (uint32_t)d : ((uint32_t)d & LIMB_MASK);
  }
  return r;
}
// canonical representative of a < 2^L p (L <= 4)
template <int L, class P>
GM_DEV Fe<P> fe_canon(Fe<P> a) {
  if constexpr (L >= 4) fe_reduce_k<8>(a);
  if constexpr (L >= 3) fe_reduce_k<4>(a);
  if constexpr (L >= 2) fe_reduce_k<2>(a);
  if constexpr (L >= 1) fe_reduce_k<1>(a);
  return a;
}
// Is a (< K p, K <= 16) congruent to 0?  a = j p forces a's top limb to be the
// top limb of j p, so that cheap filter decides almost always; the exact test
// runs only when the filter matches.
template <int K, class P>
GM_DEV bool fe_is_zero_lz(const Fe<P>& a) {
  static_assert(K <= 16, "fe_canon<4> covers a < 16p");
  const uint32_t top = a.v[P::N - 1];
  bool hit = false;
#pragma unroll
  for (int j = 0; j < K; j++) hit |= top == kp_top<P>(j);
  if (!hit) return false;
  return fe_is_zero(fe_canon<4>(a));
}

// form conversions (see header comment)
template <class P>
GM_DEV Fe<P> fe_to_internal(const Fe<P>& gnark_form) { return fe_mul(gnark_form, GM_FE_CONST(P, kin)); }
template <class P>
GM_DEV Fe<P> fe_to_gnark(const Fe<P>& internal) { return fe_mul(internal, GM_FE_CONST(P, kout)); }
template <class P>
GM_DEV Fe<P> fe_gnark_to_canonical(const Fe<P>& gnark_form) { return fe_mul(gnark_form, GM_FE_CONST(P, kcan)); }
template <class P>
GM_DEV Fe<P> fe_canonical_to_gnark(const Fe<P>& x) { return fe_mul(x, GM_FE_CONST(P, kgn)); }
template <class P>
GM_DEV Fe<P> fe_to_mont(const Fe<P>& x) { return fe_mul(x, GM_FE_CONST(P, r2)); }
template <class P>
GM_DEV Fe<P> fe_from_mont(const Fe<P>& internal) {
  Fe<P> o = fe_zero<P>();
  o.v[0] = 1;
  return fe_mul(internal, o);
}

// a^(p-2) (Fermat inversion; 0 -> 0), internal form in and out.
template <class P>
GM_DEV Fe<P> fe_inv(const Fe<P>& a) {
  Fe<P> r = fe_one<P>();
  for (int i = P::NG - 1; i >= 0; i--) {
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
// Complex squaring, 2 base multiplications:
//   a0^2 + BETA a1^2 = (a0 + a1)(a0 + BETA a1) - (1 + BETA) a0 a1,  2 a0 a1 u
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe_sqr(const Fe2<P, BETA>& a) {
  const Fe<P> c = fe_mul(a.a0, a.a1);
  Fe<P> t = fe_mul(fe_add(a.a0, a.a1), fe_add(a.a0, mul_by_beta<P, BETA>(a.a1)));
  if constexpr (BETA == -5) {
    const Fe<P> c2 = fe_dbl(c);
    t = fe_add(t, fe_dbl(c2));  // - (1 + BETA) c = + 4c
  } else {
    static_assert(BETA == -1, "unsupported non-residue");
  }
  Fe2<P, BETA> r;
  r.a0 = t;
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

// ---- lazily reduced Fp2 (G2 bucket accumulation) ---------------------------
// Components are normalised back below 2p after every product, so product
// inputs stay small: with components < IN p (IN <= 6 in the G2 mixed add) the
// Karatsuba term (a0 + a1)(b0 + b1) < 144 p^2 < R' p for BN254 (R' / p > 169);
// BLS12-377 Fp has R' / p ~ 2^29.
// x < M p  ->  x < 2p  (M <= 16)
template <int M, class P>
GM_DEV void fe_to2p(Fe<P>& x) {
  static_assert(M <= 16, "fe_to2p covers x < 16p");
  if constexpr (M > 8) fe_reduce_k<8>(x);
  if constexpr (M > 4) fe_reduce_k<4>(x);
  if constexpr (M > 2) fe_reduce_k<2>(x);
}
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe2_add_lz(const Fe2<P, BETA>& a, const Fe2<P, BETA>& b) {
  return {fe_add_lz(a.a0, b.a0), fe_add_lz(a.a1, b.a1)};
}
template <int K, class P, int BETA>
GM_DEV Fe2<P, BETA> fe2_sub_lz(const Fe2<P, BETA>& a, const Fe2<P, BETA>& b) {
  return {fe_sub_lz<K>(a.a0, b.a0), fe_sub_lz<K>(a.a1, b.a1)};
}
template <int M, class P, int BETA>
GM_DEV void fe2_to2p(Fe2<P, BETA>& x) {
  fe_to2p<M>(x.a0);
  fe_to2p<M>(x.a1);
}
// 5 x for x < 2p (< 10p)
template <class P>
GM_DEV Fe<P> fe_times5_lz(const Fe<P>& x) {
  const Fe<P> x2 = fe_add_lz(x, x);
  return fe_add_lz(fe_add_lz(x2, x2), x);
}
// Karatsuba product, result components < 2p.  Inputs: components < 6p (BN254).
template <class P, int BETA>
GM_DEV Fe2<P, BETA> fe2_mul_lz(const Fe2<P, BETA>& a, const Fe2<P, BETA>& b) {
  const Fe<P> v0 = fe_mul_lz(a.a0, b.a0);  // < 2p
  const Fe<P> v1 = fe_mul_lz(a.a1, b.a1);  // < 2p
  const Fe<P> s = fe_mul_lz(fe_add_lz(a.a0, a.a1), fe_add_lz(b.a0, b.a1));  // < 2p
  Fe2<P, BETA> r;
  if constexpr (BETA == -1) {
    r.a0 = fe_sub_lz<2>(v0, v1);  // < 4p
    fe_to2p<4>(r.a0);
  } else {
    static_assert(BETA == -5, "unsupported non-residue");
    r.a0 = fe_sub_lz<10>(v0, fe_times5_lz(v1));  // < 12p
    fe_to2p<12>(r.a0);
  }
  r.a1 = fe_sub_lz<4>(s, fe_add_lz(v0, v1));  // < 6p
  fe_to2p<6>(r.a1);
  return r;
}
// Complex squaring, result components < 2p.  Inputs: components < IN p.
template <int IN, class P, int BETA>
GM_DEV Fe2<P, BETA> fe2_sqr_lz(const Fe2<P, BETA>& a) {
  const Fe<P> c = fe_mul_lz(a.a0, a.a1);  // < 2p
  Fe2<P, BETA> r;
  if constexpr (BETA == -1) {
    // (a0 + a1)(a0 - a1): (2 IN p)^2 <= 144 p^2 for IN <= 6
    r.a0 = fe_mul_lz(fe_add_lz(a.a0, a.a1), fe_sub_lz<IN>(a.a0, a.a1));
  } else {
    static_assert(BETA == -5, "unsupported non-residue");
    // (a0 + a1)(a0 - 5 a1) + 4 a0 a1
    const Fe<P> a15 = fe_times5_lz(a.a1);  // < 5 IN p
    const Fe<P> t = fe_mul_lz(fe_add_lz(a.a0, a.a1), fe_sub_lz<5 * IN>(a.a0, a15));
    const Fe<P> c2 = fe_add_lz(c, c);
    r.a0 = fe_add_lz(t, fe_add_lz(c2, c2));  // < 10p
    fe_to2p<10>(r.a0);
  }
  r.a1 = fe_add_lz(c, c);  // < 4p
  fe_to2p<4>(r.a1);
  return r;
}

// gnark-layout <-> internal for a coordinate field (Fe or Fe2).
template <class F>
struct Coord;
template <class P>
struct Coord<Fe<P>> {
  static constexpr int WORDS = P::NG;  // u32 words in gnark layout
  GM_DEV static Fe<P> load_internal(const uint32_t* src) { return fe_to_internal(fe_unpack<P>(feg_load<P>(src))); }
  GM_DEV static void store_gnark(uint32_t* dst, const Fe<P>& a) { feg_store<P>(dst, fe_pack(fe_to_gnark(a))); }
  // "packed internal": the internal (x * 2^(29N) mod p) value in gnark's word
  // layout -- same byte size as gnark, no multiplication to convert.
  GM_DEV static Fe<P> load_packed(const uint32_t* src) { return fe_unpack<P>(feg_load<P>(src)); }
  GM_DEV static void store_packed(uint32_t* dst, const Fe<P>& a) { feg_store<P>(dst, fe_pack(a)); }
};
template <class P, int B>
struct Coord<Fe2<P, B>> {
  static constexpr int WORDS = 2 * P::NG;
  GM_DEV static Fe2<P, B> load_internal(const uint32_t* src) {
    return {Coord<Fe<P>>::load_internal(src), Coord<Fe<P>>::load_internal(src + P::NG)};
  }
  GM_DEV static void store_gnark(uint32_t* dst, const Fe2<P, B>& a) {
    Coord<Fe<P>>::store_gnark(dst, a.a0);
    Coord<Fe<P>>::store_gnark(dst + P::NG, a.a1);
  }
  GM_DEV static Fe2<P, B> load_packed(const uint32_t* src) {
    return {Coord<Fe<P>>::load_packed(src), Coord<Fe<P>>::load_packed(src + P::NG)};
  }
  GM_DEV static void store_packed(uint32_t* dst, const Fe2<P, B>& a) {
    Coord<Fe<P>>::store_packed(dst, a.a0);
    Coord<Fe<P>>::store_packed(dst + P::NG, a.a1);
  }
};

}  // namespace gm
