// TEST ORACLE ONLY -- CPU restatement of gnark-crypto field / curve arithmetic.
// Used by tests/, the fixture generator and bench.py's cpu_baseline leg; never
// linked into the product library.  64-bit limbs, CIOS Montgomery, gnark-crypto
// memory layout (little-endian u64 limbs, x*R mod p, R = 2^(64N)).
#pragma once
#include <cstdint>
#include <cstring>
#include "oracle_constants.h"

namespace orc {

typedef unsigned __int128 u128;

template <int N_, int ID>
struct FDesc {
  static constexpr int N = N_;
};

#define ORC_FIELD(NAME, TAG, NN)                              \
  struct NAME {                                               \
    static constexpr int N = NN;                              \
    static constexpr uint64_t P[NN] = O_##TAG##_P;            \
    static constexpr uint64_t ONE[NN] = O_##TAG##_ONE;        \
    static constexpr uint64_t R2[NN] = O_##TAG##_R2;          \
    static constexpr uint64_t INV = O_##TAG##_INV;            \
  };
ORC_FIELD(BnFp, BN254_FP, 4)
ORC_FIELD(BnFr, BN254_FR, 4)
ORC_FIELD(BlsFp, BLS12377_FP, 6)
ORC_FIELD(BlsFr, BLS12377_FR, 4)

template <class D>
struct Fe {
  uint64_t v[D::N];
};

template <class D>
inline bool geq_p(const uint64_t* a) {
  for (int i = D::N - 1; i >= 0; i--) {
    if (a[i] > D::P[i]) return true;
    if (a[i] < D::P[i]) return false;
  }
  return true;
}
template <class D>
inline void sub_p(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < D::N; i++) {
    u128 d = (u128)a[i] - D::P[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}

template <class D>
inline Fe<D> zero() {
  Fe<D> r;
  memset(r.v, 0, sizeof(r.v));
  return r;
}
template <class D>
inline Fe<D> one() {
  Fe<D> r;
  for (int i = 0; i < D::N; i++) r.v[i] = D::ONE[i];
  return r;
}
template <class D>
inline bool is_zero(const Fe<D>& a) {
  uint64_t x = 0;
  for (int i = 0; i < D::N; i++) x |= a.v[i];
  return x == 0;
}
template <class D>
inline bool eq(const Fe<D>& a, const Fe<D>& b) {
  return memcmp(a.v, b.v, sizeof(a.v)) == 0;
}
template <class D>
inline Fe<D> add(const Fe<D>& a, const Fe<D>& b) {
  Fe<D> r;
  uint64_t c = 0;
  for (int i = 0; i < D::N; i++) {
    u128 s = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq_p<D>(r.v)) sub_p<D>(r.v);
  return r;
}
template <class D>
inline Fe<D> sub(const Fe<D>& a, const Fe<D>& b) {
  Fe<D> r;
  uint64_t br = 0;
  for (int i = 0; i < D::N; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < D::N; i++) {
      u128 s = (u128)r.v[i] + D::P[i] + c;
      r.v[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  return r;
}
template <class D>
inline Fe<D> neg(const Fe<D>& a) {
  if (is_zero(a)) return a;
  return sub(zero<D>(), a);
}
template <class D>
inline Fe<D> dbl(const Fe<D>& a) {
  return add(a, a);
}

// CIOS Montgomery multiplication
template <class D>
inline Fe<D> mul(const Fe<D>& a, const Fe<D>& b) {
  constexpr int N = D::N;
  uint64_t t[N + 2];
  memset(t, 0, sizeof(t));
  for (int i = 0; i < N; i++) {
    uint64_t C = 0;
    for (int j = 0; j < N; j++) {
      u128 x = (u128)a.v[j] * b.v[i] + t[j] + C;
      t[j] = (uint64_t)x;
      C = (uint64_t)(x >> 64);
    }
    u128 x = (u128)t[N] + C;
    t[N] = (uint64_t)x;
    t[N + 1] = (uint64_t)(x >> 64);
    uint64_t m = t[0] * D::INV;
    x = (u128)m * D::P[0] + t[0];
    C = (uint64_t)(x >> 64);
    for (int j = 1; j < N; j++) {
      x = (u128)m * D::P[j] + t[j] + C;
      t[j - 1] = (uint64_t)x;
      C = (uint64_t)(x >> 64);
    }
    x = (u128)t[N] + C;
    t[N - 1] = (uint64_t)x;
    t[N] = t[N + 1] + (uint64_t)(x >> 64);
  }
  Fe<D> r;
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  if (t[N] || geq_p<D>(r.v)) sub_p<D>(r.v);
  return r;
}
template <class D>
inline Fe<D> sqr(const Fe<D>& a) {
  return mul(a, a);
}
template <class D>
inline Fe<D> from_mont(const Fe<D>& a) {
  Fe<D> o = zero<D>();
  o.v[0] = 1;
  return mul(a, o);
}
template <class D>
inline Fe<D> to_mont(const Fe<D>& a) {
  Fe<D> r2;
  for (int i = 0; i < D::N; i++) r2.v[i] = D::R2[i];
  return mul(a, r2);
}
template <class D>
inline Fe<D> from_u64(uint64_t x) {
  Fe<D> a = zero<D>();
  a.v[0] = x;
  return to_mont(a);
}
// a^e for a little-endian u64 exponent of length ne
template <class D>
inline Fe<D> pow(const Fe<D>& a, const uint64_t* e, int ne) {
  Fe<D> r = one<D>();
  for (int i = ne - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = sqr(r);
      if ((e[i] >> b) & 1) r = mul(r, a);
    }
  return r;
}
template <class D>
inline Fe<D> inv(const Fe<D>& a) {
  // Fermat: a^(p-2)
  uint64_t e[D::N];
  for (int i = 0; i < D::N; i++) e[i] = D::P[i];
  e[0] -= 2;  // p is odd and > 2, no borrow for these moduli (p[0] >= 2)
  return pow(a, e, D::N);
}

// ---------------------------------------------------------------------------
// Fp2 = Fp[u]/(u^2 - beta)
// ---------------------------------------------------------------------------
template <class D, int BETA>
struct Fe2 {
  Fe<D> a0, a1;
};
template <class D, int BETA>
inline Fe<D> mul_beta(const Fe<D>& x) {
  if (BETA == -1) return neg(x);
  Fe<D> x4 = dbl(dbl(x));
  return neg(add(x4, x));  // -5x
}

// generic ops used by the group code: overloads on Fe and Fe2
template <class D, int B>
inline Fe2<D, B> add(const Fe2<D, B>& a, const Fe2<D, B>& b) { return {add(a.a0, b.a0), add(a.a1, b.a1)}; }
template <class D, int B>
inline Fe2<D, B> sub(const Fe2<D, B>& a, const Fe2<D, B>& b) { return {sub(a.a0, b.a0), sub(a.a1, b.a1)}; }
template <class D, int B>
inline Fe2<D, B> neg(const Fe2<D, B>& a) { return {neg(a.a0), neg(a.a1)}; }
template <class D, int B>
inline Fe2<D, B> dbl(const Fe2<D, B>& a) { return {dbl(a.a0), dbl(a.a1)}; }
template <class D, int B>
inline bool is_zero(const Fe2<D, B>& a) { return is_zero(a.a0) && is_zero(a.a1); }
template <class D, int B>
inline bool eq(const Fe2<D, B>& a, const Fe2<D, B>& b) { return eq(a.a0, b.a0) && eq(a.a1, b.a1); }
template <class D, int B>
inline Fe2<D, B> mul(const Fe2<D, B>& a, const Fe2<D, B>& b) {
  Fe<D> v0 = mul(a.a0, b.a0), v1 = mul(a.a1, b.a1);
  Fe<D> s = mul(add(a.a0, a.a1), add(b.a0, b.a1));
  return {add(v0, mul_beta<D, B>(v1)), sub(sub(s, v0), v1)};
}
template <class D, int B>
inline Fe2<D, B> sqr(const Fe2<D, B>& a) { return mul(a, a); }
template <class D, int B>
inline Fe2<D, B> inv(const Fe2<D, B>& a) {
  // 1/(a0 + a1 u) = (a0 - a1 u) / (a0^2 - beta a1^2)
  Fe<D> n = sub(sqr(a.a0), mul_beta<D, B>(sqr(a.a1)));
  Fe<D> ni = inv(n);
  return {mul(a.a0, ni), neg(mul(a.a1, ni))};
}

template <class F>
struct FTraits;
template <class D>
struct FTraits<Fe<D>> {
  static Fe<D> zero() { return orc::zero<D>(); }
  static Fe<D> one() { return orc::one<D>(); }
};
template <class D, int B>
struct FTraits<Fe2<D, B>> {
  static Fe2<D, B> zero() { return {orc::zero<D>(), orc::zero<D>()}; }
  static Fe2<D, B> one() { return {orc::one<D>(), orc::zero<D>()}; }
};

// ---------------------------------------------------------------------------
// short Weierstrass, a = 0.  Affine (gnark layout {X, Y}, infinity = (0,0))
// and Jacobian (X/Z^2, Y/Z^3; infinity Z = 0).
// ---------------------------------------------------------------------------
template <class F>
struct Aff {
  F x, y;
};
template <class F>
struct Jac {
  F x, y, z;
};

template <class F>
inline bool aff_is_inf(const Aff<F>& p) {
  return is_zero(p.x) && is_zero(p.y);
}
template <class F>
inline Jac<F> jac_inf() {
  return {FTraits<F>::one(), FTraits<F>::one(), FTraits<F>::zero()};
}
template <class F>
inline Jac<F> to_jac(const Aff<F>& p) {
  if (aff_is_inf(p)) return jac_inf<F>();
  return {p.x, p.y, FTraits<F>::one()};
}
template <class F>
inline Aff<F> to_aff(const Jac<F>& p) {
  if (is_zero(p.z)) return {FTraits<F>::zero(), FTraits<F>::zero()};
  F zi = inv(p.z);
  F zi2 = sqr(zi);
  return {mul(p.x, zi2), mul(p.y, mul(zi2, zi))};
}

// dbl-2009-l
template <class F>
inline Jac<F> jdbl(const Jac<F>& p) {
  if (is_zero(p.z)) return p;
  F A = sqr(p.x), B = sqr(p.y), C = sqr(B);
  F t = add(p.x, B);
  F D = dbl(sub(sub(sqr(t), A), C));
  F E = add(dbl(A), A);
  F Fv = sqr(E);
  F X3 = sub(Fv, dbl(D));
  F C8 = dbl(dbl(dbl(C)));
  F Y3 = sub(mul(E, sub(D, X3)), C8);
  F Z3 = dbl(mul(p.y, p.z));
  return {X3, Y3, Z3};
}
// add-2007-bl
template <class F>
inline Jac<F> jadd(const Jac<F>& p, const Jac<F>& q) {
  if (is_zero(p.z)) return q;
  if (is_zero(q.z)) return p;
  F Z1Z1 = sqr(p.z), Z2Z2 = sqr(q.z);
  F U1 = mul(p.x, Z2Z2), U2 = mul(q.x, Z1Z1);
  F S1 = mul(p.y, mul(q.z, Z2Z2)), S2 = mul(q.y, mul(p.z, Z1Z1));
  if (eq(U1, U2)) {
    if (eq(S1, S2)) return jdbl(p);
    return jac_inf<F>();
  }
  F H = sub(U2, U1);
  F I = sqr(dbl(H));
  F J = mul(H, I);
  F r = dbl(sub(S2, S1));
  F V = mul(U1, I);
  F X3 = sub(sub(sqr(r), J), dbl(V));
  F Y3 = sub(mul(r, sub(V, X3)), dbl(mul(S1, J)));
  F Z3 = mul(sub(sub(sqr(add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}
// madd-2007-bl (q affine, not infinity)
template <class F>
inline Jac<F> jadd_mixed(const Jac<F>& p, const Aff<F>& q) {
  if (aff_is_inf(q)) return p;
  if (is_zero(p.z)) return to_jac(q);
  F Z1Z1 = sqr(p.z);
  F U2 = mul(q.x, Z1Z1);
  F S2 = mul(q.y, mul(p.z, Z1Z1));
  if (eq(U2, p.x)) {
    if (eq(S2, p.y)) return jdbl(p);
    return jac_inf<F>();
  }
  F H = sub(U2, p.x);
  F HH = sqr(H);
  F I = dbl(dbl(HH));
  F J = mul(H, I);
  F r = dbl(sub(S2, p.y));
  F V = mul(p.x, I);
  F X3 = sub(sub(sqr(r), J), dbl(V));
  F Y3 = sub(mul(r, sub(V, X3)), dbl(mul(p.y, J)));
  F Z3 = sub(sub(sqr(add(p.z, H)), Z1Z1), HH);
  return {X3, Y3, Z3};
}
template <class F>
inline Aff<F> aff_neg(const Aff<F>& p) {
  return {p.x, neg(p.y)};
}

// [k]P, k canonical little-endian u64 words
template <class F>
inline Jac<F> scalar_mul(const Jac<F>& p, const uint64_t* k, int nk) {
  Jac<F> r = jac_inf<F>();
  for (int i = nk - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = jdbl(r);
      if ((k[i] >> b) & 1) r = jadd(r, p);
    }
  return r;
}

}  // namespace orc
