// Host-side field / curve arithmetic used by the product library for the O(1)
// finishing work that follows the device kernels:
//   * Horner combination of per-window MSM sums  (sum_w 2^(c*w) W_w)
//   * Groth16 finishing adds (AddMixed alpha/beta, [r]delta, [s]Ar, ...:
//     backend/groth16/bn254/icicle/icicle.go:295-391, prove.go:195-305)
//   * XYZZ -> Jacobian / affine conversion of device results.
// 64-bit limbs, CIOS Montgomery, gnark-crypto layout.
#pragma once
#include <cstdint>
#include <cstring>
#include "field_constants.hpp"

namespace gm {
namespace host {

typedef unsigned __int128 u128;

#define GM_HOST_FIELD(NAME, TAG, NN)                        \
  struct NAME {                                             \
    static constexpr int N = NN;                            \
    static constexpr uint64_t P[NN] = GM_##TAG##_P64;       \
    static constexpr uint64_t ONE[NN] = GM_##TAG##_ONE64;   \
    static constexpr uint64_t R2[NN] = GM_##TAG##_R2_64;    \
    static constexpr uint64_t INV = GM_##TAG##_INV64;       \
  };
GM_HOST_FIELD(HBnFp, BN254_FP, 4)
GM_HOST_FIELD(HBnFr, BN254_FR, 4)
GM_HOST_FIELD(HBlsFp, BLS12377_FP, 6)
GM_HOST_FIELD(HBlsFr, BLS12377_FR, 4)

template <class D>
struct F {
  uint64_t v[D::N];
  static F zero() {
    F r;
    memset(r.v, 0, sizeof(r.v));
    return r;
  }
  static F one() {
    F r;
    memcpy(r.v, D::ONE, sizeof(r.v));
    return r;
  }
  bool is_zero() const {
    uint64_t x = 0;
    for (int i = 0; i < D::N; i++) x |= v[i];
    return x == 0;
  }
  bool operator==(const F& o) const { return memcmp(v, o.v, sizeof(v)) == 0; }
};

template <class D>
inline void cond_sub_p(uint64_t* a, uint64_t carry) {
  uint64_t t[D::N], br = 0;
  for (int i = 0; i < D::N; i++) {
    u128 d = (u128)a[i] - D::P[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
  }
  if (carry || !br) memcpy(a, t, sizeof(t));
}
template <class D>
inline F<D> operator+(const F<D>& a, const F<D>& b) {
  F<D> r;
  uint64_t c = 0;
  for (int i = 0; i < D::N; i++) {
    u128 s = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  cond_sub_p<D>(r.v, c);
  return r;
}
template <class D>
inline F<D> operator-(const F<D>& a, const F<D>& b) {
  F<D> r;
  uint64_t br = 0;
  for (int i = 0; i < D::N; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 127);
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
inline F<D> operator-(const F<D>& a) {
  return F<D>::zero() - a;
}
template <class D>
inline F<D> operator*(const F<D>& a, const F<D>& b) {
  constexpr int N = D::N;
  uint64_t t[N + 2] = {0};
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
  F<D> r;
  memcpy(r.v, t, sizeof(r.v));
  cond_sub_p<D>(r.v, t[N]);
  return r;
}
template <class D>
inline F<D> fpow(const F<D>& a, const uint64_t* e, int ne) {
  F<D> r = F<D>::one();
  for (int i = ne - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = r * r;
      if ((e[i] >> b) & 1) r = r * a;
    }
  return r;
}
template <class D>
inline F<D> finv(const F<D>& a) {
  uint64_t e[D::N];
  memcpy(e, D::P, sizeof(e));
  e[0] -= 2;
  return fpow(a, e, D::N);
}
template <class D>
inline F<D> to_mont(const F<D>& a) {
  F<D> r2;
  memcpy(r2.v, D::R2, sizeof(r2.v));
  return a * r2;
}
template <class D>
inline F<D> from_mont(const F<D>& a) {
  F<D> o = F<D>::zero();
  o.v[0] = 1;
  return a * o;
}
template <class D>
inline F<D> from_u64(uint64_t x) {
  F<D> a = F<D>::zero();
  a.v[0] = x;
  return to_mont(a);
}

// Fp2 ------------------------------------------------------------------------
template <class D, int BETA>
struct F2 {
  F<D> a0, a1;
  static F2 zero() { return {F<D>::zero(), F<D>::zero()}; }
  static F2 one() { return {F<D>::one(), F<D>::zero()}; }
  bool is_zero() const { return a0.is_zero() && a1.is_zero(); }
  bool operator==(const F2& o) const { return a0 == o.a0 && a1 == o.a1; }
};
template <class D, int B>
inline F<D> mul_beta(const F<D>& x) {
  if (B == -1) return -x;
  F<D> x2 = x + x, x4 = x2 + x2;
  return -(x4 + x);
}
template <class D, int B>
inline F2<D, B> operator+(const F2<D, B>& a, const F2<D, B>& b) { return {a.a0 + b.a0, a.a1 + b.a1}; }
template <class D, int B>
inline F2<D, B> operator-(const F2<D, B>& a, const F2<D, B>& b) { return {a.a0 - b.a0, a.a1 - b.a1}; }
template <class D, int B>
inline F2<D, B> operator-(const F2<D, B>& a) { return {-a.a0, -a.a1}; }
template <class D, int B>
inline F2<D, B> operator*(const F2<D, B>& a, const F2<D, B>& b) {
  F<D> v0 = a.a0 * b.a0, v1 = a.a1 * b.a1;
  F<D> s = (a.a0 + a.a1) * (b.a0 + b.a1);
  return {v0 + mul_beta<D, B>(v1), s - v0 - v1};
}
template <class D, int B>
inline F2<D, B> finv(const F2<D, B>& a) {
  F<D> n = a.a0 * a.a0 - mul_beta<D, B>(a.a1 * a.a1);
  F<D> ni = finv(n);
  return {a.a0 * ni, -(a.a1 * ni)};
}

// Jacobian group law (a = 0) ---------------------------------------------------
template <class FF>
struct Jac {
  FF x, y, z;
  static Jac inf() { return {FF::one(), FF::one(), FF::zero()}; }
  bool is_inf() const { return z.is_zero(); }
};
template <class FF>
struct Aff {
  FF x, y;
  bool is_inf() const { return x.is_zero() && y.is_zero(); }
};

template <class FF>
inline Jac<FF> jdbl(const Jac<FF>& p) {
  if (p.is_inf()) return p;
  FF A = p.x * p.x, B = p.y * p.y, C = B * B;
  FF t = p.x + B;
  FF D = t * t - A - C;
  D = D + D;
  FF E = A + A + A;
  FF X3 = E * E - (D + D);
  FF C2 = C + C, C4 = C2 + C2, C8 = C4 + C4;
  FF Y3 = E * (D - X3) - C8;
  FF yz = p.y * p.z;
  return {X3, Y3, yz + yz};
}
template <class FF>
inline Jac<FF> jadd(const Jac<FF>& p, const Jac<FF>& q) {
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  FF Z1Z1 = p.z * p.z, Z2Z2 = q.z * q.z;
  FF U1 = p.x * Z2Z2, U2 = q.x * Z1Z1;
  FF S1 = p.y * (q.z * Z2Z2), S2 = q.y * (p.z * Z1Z1);
  if (U1 == U2) {
    if (S1 == S2) return jdbl(p);
    return Jac<FF>::inf();
  }
  FF H = U2 - U1;
  FF I = (H + H) * (H + H);
  FF J = H * I;
  FF r = S2 - S1;
  r = r + r;
  FF V = U1 * I;
  FF X3 = r * r - J - (V + V);
  FF S1J = S1 * J;
  FF Y3 = r * (V - X3) - (S1J + S1J);
  FF zs = p.z + q.z;
  FF Z3 = (zs * zs - Z1Z1 - Z2Z2) * H;
  return {X3, Y3, Z3};
}
template <class FF>
inline Jac<FF> to_jac(const Aff<FF>& a) {
  if (a.is_inf()) return Jac<FF>::inf();
  return {a.x, a.y, FF::one()};
}
template <class FF>
inline Jac<FF> jadd_aff(const Jac<FF>& p, const Aff<FF>& q) {
  return jadd(p, to_jac(q));
}
template <class FF>
inline Aff<FF> to_aff(const Jac<FF>& p) {
  if (p.is_inf()) return {FF::zero(), FF::zero()};
  FF zi = finv(p.z);
  FF zi2 = zi * zi;
  return {p.x * zi2, p.y * (zi2 * zi)};
}
// [k]p, k canonical little-endian u64 words
template <class FF>
inline Jac<FF> jmul(const Jac<FF>& p, const uint64_t* k, int nk) {
  Jac<FF> r = Jac<FF>::inf();
  for (int i = nk - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = jdbl(r);
      if ((k[i] >> b) & 1) r = jadd(r, p);
    }
  return r;
}
// XYZZ (x = X/ZZ, y = Y/ZZZ) -> Jacobian: Z = ZZZ/ZZ... avoid inversion with
// Z_j = ZZ*ZZZ, X_j = X*ZZ*ZZZ^2, Y_j = Y*ZZZ^2*ZZ^3 = Y*ZZZ^4 (ZZ^3 = ZZZ^2).
template <class FF>
inline Jac<FF> xyzz_to_jac(const FF& X, const FF& Y, const FF& ZZ, const FF& ZZZ) {
  if (ZZ.is_zero()) return Jac<FF>::inf();
  FF zzz2 = ZZZ * ZZZ;
  return {X * ZZ * zzz2, Y * zzz2 * zzz2, ZZ * ZZZ};
}

}  // namespace host
}  // namespace gm
