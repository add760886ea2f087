// Device-side elliptic-curve arithmetic for the MSM bucket phase (gfx950).
//
// Curves: short Weierstrass y^2 = x^3 + b (a = 0) -- BN254 / BLS12-377, G1 over
// Fp and G2 over Fp2.  Points arrive in gnark-crypto's G1Affine / G2Affine memory
// layout ({X, Y}, Montgomery limbs, infinity encoded as (0,0)).
//
// Buckets are kept in XYZZ coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2):
//   mixed add  (madd-2008-s)   8M + 2S
//   add        (add-2008-s)   12M + 2S
//   double     (dbl-2008-s-1)  6M + 3S
// (hyperelliptic.org EFD, "g1p/auto-shortw-xyzz").  Infinity is ZZ = 0.
#pragma once
#include "field.hpp"

namespace gm {

// ---- field-op dispatch for Fe<P> and Fe2<P,B> -------------------------------
template <class F>
struct FOps;

template <class P>
struct FOps<Fe<P>> {
  using T = Fe<P>;
  GM_DEV static T zero() { return fe_zero<P>(); }
  GM_DEV static T one() { return fe_one<P>(); }
};
template <class P, int B>
struct FOps<Fe2<P, B>> {
  using T = Fe2<P, B>;
  GM_DEV static T zero() { return {fe_zero<P>(), fe_zero<P>()}; }
  GM_DEV static T one() { return {fe_one<P>(), fe_zero<P>()}; }
};

template <class F>
struct Affine {
  F x, y;
};
template <class F>
struct XYZZ {
  F x, y, zz, zzz;
};

template <class F>
GM_DEV bool aff_is_inf(const Affine<F>& p) {
  return fe_is_zero(p.x) && fe_is_zero(p.y);
}

template <class F>
GM_DEV XYZZ<F> xyzz_inf() {
  XYZZ<F> r;
  r.x = FOps<F>::one();
  r.y = FOps<F>::one();
  r.zz = FOps<F>::zero();
  r.zzz = FOps<F>::zero();
  return r;
}
template <class F>
GM_DEV bool xyzz_is_inf(const XYZZ<F>& p) {
  return fe_is_zero(p.zz);
}

// 2*P for affine P (mdbl-2008-s-1); P must not be infinity.
template <class F>
GM_DEV XYZZ<F> xyzz_dbl_aff(const Affine<F>& p) {
  F U = fe_dbl(p.y);
  F V = fe_sqr(U);
  F W = fe_mul(U, V);
  F S = fe_mul(p.x, V);
  F X2 = fe_sqr(p.x);
  F M = fe_add(fe_dbl(X2), X2);
  XYZZ<F> r;
  r.x = fe_sub(fe_sqr(M), fe_dbl(S));
  r.y = fe_sub(fe_mul(M, fe_sub(S, r.x)), fe_mul(W, p.y));
  r.zz = V;
  r.zzz = W;
  return r;
}

// a += p, p affine (infinity allowed: skipped).
template <class F>
GM_DEV void xyzz_add_aff(XYZZ<F>& a, const Affine<F>& p) {
  if (aff_is_inf(p)) return;
  if (xyzz_is_inf(a)) {
    a.x = p.x;
    a.y = p.y;
    a.zz = FOps<F>::one();
    a.zzz = FOps<F>::one();
    return;
  }
  // ordered so that each temporary dies as early as possible (register pressure
  // decides the occupancy of the accumulation kernel, esp. for Fp2 coordinates)
  F P = fe_sub(fe_mul(p.x, a.zz), a.x);   // U2 - X1
  F R = fe_sub(fe_mul(p.y, a.zzz), a.y);  // S2 - Y1
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) {
      a = xyzz_dbl_aff(p);
    } else {
      a = xyzz_inf<F>();
    }
    return;
  }
  F PP = fe_sqr(P);
  F PPP = fe_mul(P, PP);
  a.zz = fe_mul(a.zz, PP);
  F Q = fe_mul(a.x, PP);
  a.zzz = fe_mul(a.zzz, PPP);
  F X3 = fe_sub(fe_sub(fe_sqr(R), PPP), fe_dbl(Q));
  a.y = fe_sub(fe_mul(R, fe_sub(Q, X3)), fe_mul(a.y, PPP));
  a.x = X3;
}

// Lazily reduced a += (neg ? -p : p) for G1 buckets (see field.hpp "Lazily
// reduced arithmetic").  Invariants on a: x < 8p, y < 4p, zz < 2p, zzz < 2p
// (canonical values qualify); p canonical.  Every product below has inputs with
// ab <= 100 p^2 (largest: P^2 with P < 10p).  zz is never a non-zero multiple
// of p (zz * PP with PP != 0 mod p), so fe_is_zero(zz) still tests infinity.
// The digit sign is applied to S2 = y zzz (carry-free 2p - S2) rather than to y,
// and X3 = R^2 - PPP - 2Q takes one borrow chain (fe_sub2x_lz).
// CH: one dependent mad chain per product (fe_mul CHAIN) -- A/B variant of the
// accumulation kernel only (GM_MSM_ACC_CHAIN=1).
template <class P, int CH = 0>
GM_DEV void xyzz_add_aff_lz(XYZZ<Fe<P>>& a, const Affine<Fe<P>>& p, bool neg) {
  static_assert(P::BITS + 7 <= RADIX * P::N, "lazy reduction needs R' > 128 p");
  using F = Fe<P>;
  if (aff_is_inf(p)) return;
  if (xyzz_is_inf(a)) {
    a.x = p.x;
    a.y = neg ? fe_neg(p.y) : p.y;
    a.zz = fe_one<P>();
    a.zzz = fe_one<P>();
    return;
  }
  F Pd = fe_sub_lz<8>(fe_mul<P, false, CH>(p.x, a.zz), a.x);   // U2 - X1   < 10p
  // +-S2 - Y1 < 6p  (S2 = y zzz < 2p; 2p - S2 in (0, 2p])
  F R = fe_sub_lz<4>(fe_cneg2p_cf(fe_mul<P, false, CH>(p.y, a.zzz), neg), a.y);
  if (fe_is_zero_lz<10>(Pd)) {
    if (fe_is_zero_lz<6>(R)) {
      Affine<F> q = p;
      if (neg) q.y = fe_neg(p.y);
      a = xyzz_dbl_aff(q);
    } else {
      a = xyzz_inf<F>();
    }
    return;
  }
  F PP = fe_sqr<P, false, CH>(Pd);                              // < 2p
  F PPP = fe_mul<P, false, CH>(Pd, PP);                         // < 2p
  a.zz = fe_mul<P, false, CH>(a.zz, PP);
  F Q = fe_mul<P, false, CH>(a.x, PP);                          // < 2p
  a.zzz = fe_mul<P, false, CH>(a.zzz, PPP);
  F X3 = fe_sub2x_lz<6>(fe_sqr<P, false, CH>(R), PPP, Q);       // R^2 - PPP - 2Q + 6p < 8p
  // R (< 6p) * (Q - X3 + 9p < 11p) + (5p - Y1) (Y1 < 4p) * PPP (< 2p), ONE unsigned
  // reduction (fe_mul2_redc_u; Y1's negation folded into the carry-free operand
  // 5p - Y1, so no signed columns and no + p pass): < 76 p^2 / R' + p < 1.5p.
  // Q - X3 + 9p is carry-free too (fe_sub_cf, limbs < 3 2^29) where the columns
  // hold it: N (3 + 2 + 1) 2^58 < 2^64 for N <= 10 (BN254; BLS12-377's 13 limbs
  // take the normalised difference)
  if constexpr (P::N <= 10)
    a.y = fe_mul2_redc_u<P, CH>(R, fe_sub_cf<9>(Q, X3), fe_negk_cf<5>(a.y), PPP);
  else
    a.y = fe_mul2_redc_u<P, CH>(R, fe_sub_lz<8>(Q, X3), fe_negk_cf<5>(a.y), PPP);
  a.x = X3;
}
// Lazily reduced a += p for G2 buckets (Fp2 coordinates).  Invariants: every
// component of a.x, a.y, a.zz, a.zzz < 2p; p canonical.  Product inputs stay
// below 4p per component (see fe2_mul_lz / fe2_sqr_lz).
template <class P, int BETA>
GM_DEV void xyzz_add_aff_lz(XYZZ<Fe2<P, BETA>>& a, const Affine<Fe2<P, BETA>>& p) {
  static_assert(P::BITS + 7 <= RADIX * P::N, "lazy reduction needs R' > 128 p");
  using F = Fe2<P, BETA>;
  if (aff_is_inf(p)) return;
  if (xyzz_is_inf(a)) {
    a.x = p.x;
    a.y = p.y;
    a.zz = FOps<F>::one();
    a.zzz = FOps<F>::one();
    return;
  }
  F Pd = fe2_sub_lz<2>(fe2_mul_lz(p.x, a.zz), a.x);   // U2 - X1   < 4p
  F R = fe2_sub_lz<2>(fe2_mul_lz(p.y, a.zzz), a.y);   // S2 - Y1   < 4p
  if (fe_is_zero_lz<4>(Pd.a0) && fe_is_zero_lz<4>(Pd.a1)) {
    if (fe_is_zero_lz<4>(R.a0) && fe_is_zero_lz<4>(R.a1)) {
      a = xyzz_dbl_aff(p);
    } else {
      a = xyzz_inf<F>();
    }
    return;
  }
  F PP = fe2_sqr_lz<4>(Pd);                            // < 2p
  F PPP = fe2_mul_lz(Pd, PP);                          // < 2p
  a.zz = fe2_mul_lz(a.zz, PP);
  F Q = fe2_mul_lz(a.x, PP);                           // < 2p
  a.zzz = fe2_mul_lz(a.zzz, PPP);
  F X3 = fe2_sub_lz<4>(fe2_sub_lz<2>(fe2_sqr_lz<4>(R), PPP), fe2_add_lz(Q, Q));  // < 8p
  fe2_to2p<8>(X3);
  F Y3 = fe2_sub_lz<2>(fe2_mul_lz(R, fe2_sub_lz<2>(Q, X3)), fe2_mul_lz(a.y, PPP));  // < 4p
  fe2_to2p<4>(Y3);
  a.x = X3;
  a.y = Y3;
}
template <class P, int BETA>
GM_DEV XYZZ<Fe2<P, BETA>> xyzz_canon_lz(const XYZZ<Fe2<P, BETA>>& a) {
  auto c = [](const Fe2<P, BETA>& v) { return Fe2<P, BETA>{fe_canon<1>(v.a0), fe_canon<1>(v.a1)}; };
  return {c(a.x), c(a.y), c(a.zz), c(a.zzz)};
}

// canonical form of a lazily accumulated bucket
template <class P>
GM_DEV XYZZ<Fe<P>> xyzz_canon_lz(const XYZZ<Fe<P>>& a) {
  XYZZ<Fe<P>> r;
  r.x = fe_canon<3>(a.x);
  r.y = fe_canon<2>(a.y);
  r.zz = fe_canon<1>(a.zz);
  r.zzz = fe_canon<1>(a.zzz);
  return r;
}

// 2*a (dbl-2008-s-1, a = 0).  Infinity maps to infinity (ZZ3 = V*0).
template <class F>
GM_DEV XYZZ<F> xyzz_dbl(const XYZZ<F>& a) {
  F U = fe_dbl(a.y);
  F V = fe_sqr(U);
  F W = fe_mul(U, V);
  F S = fe_mul(a.x, V);
  F X2 = fe_sqr(a.x);
  F M = fe_add(fe_dbl(X2), X2);
  XYZZ<F> r;
  r.x = fe_sub(fe_sqr(M), fe_dbl(S));
  r.y = fe_sub(fe_mul(M, fe_sub(S, r.x)), fe_mul(W, a.y));
  r.zz = fe_mul(V, a.zz);
  r.zzz = fe_mul(W, a.zzz);
  return r;
}

// a + b (add-2008-s) with all special cases.
template <class F>
GM_DEV XYZZ<F> xyzz_add(const XYZZ<F>& a, const XYZZ<F>& b) {
  if (xyzz_is_inf(a)) return b;
  if (xyzz_is_inf(b)) return a;
  F U1 = fe_mul(a.x, b.zz);
  F U2 = fe_mul(b.x, a.zz);
  F S1 = fe_mul(a.y, b.zzz);
  F S2 = fe_mul(b.y, a.zzz);
  F P = fe_sub(U2, U1);
  F R = fe_sub(S2, S1);
  if (fe_is_zero(P)) {
    if (fe_is_zero(R)) return xyzz_dbl(a);
    return xyzz_inf<F>();
  }
  F PP = fe_sqr(P);
  F PPP = fe_mul(P, PP);
  F Q = fe_mul(U1, PP);
  XYZZ<F> r;
  r.x = fe_sub(fe_sub(fe_sqr(R), PPP), fe_dbl(Q));
  r.y = fe_sub(fe_mul(R, fe_sub(Q, r.x)), fe_mul(S1, PPP));
  r.zz = fe_mul(fe_mul(a.zz, b.zz), PP);
  r.zzz = fe_mul(fe_mul(a.zzz, b.zzz), PPP);
  return r;
}

// canonical form of a point whose coordinates are < 2p
template <class P>
GM_DEV XYZZ<Fe<P>> xyzz_canon2(const XYZZ<Fe<P>>& a) {
  return {fe_canon<1>(a.x), fe_canon<1>(a.y), fe_canon<1>(a.zz), fe_canon<1>(a.zzz)};
}

// Lazily reduced a + b (G1 bucket fixup and reduction): coordinates < 2p in and
// out (canonical values qualify).  Product inputs stay below 4p x 4p = 16 p^2.
// A lazily reduced zz is a non-zero residue unless the point is infinity (set
// canonically), so fe_is_zero(zz) still tests infinity.
template <class P>
GM_DEV XYZZ<Fe<P>> xyzz_add_lz(const XYZZ<Fe<P>>& a, const XYZZ<Fe<P>>& b) {
  using F = Fe<P>;
  if (xyzz_is_inf(a)) return b;
  if (xyzz_is_inf(b)) return a;
  const F U1 = fe_mul_lz(a.x, b.zz);  // < 2p
  const F U2 = fe_mul_lz(b.x, a.zz);
  const F S1 = fe_mul_lz(a.y, b.zzz);
  const F S2 = fe_mul_lz(b.y, a.zzz);
  const F Pd = fe_sub_lz<2>(U2, U1);  // < 4p
  const F R = fe_sub_lz<2>(S2, S1);   // < 4p
  if (fe_is_zero_lz<4>(Pd)) {
    if (fe_is_zero_lz<4>(R)) return xyzz_dbl(xyzz_canon2(a));
    return xyzz_inf<F>();
  }
  const F PP = fe_sqr_lz(Pd);  // < 2p
  const F PPP = fe_mul_lz(Pd, PP);
  const F Q = fe_mul_lz(U1, PP);
  F X3 = fe_sub_lz<4>(fe_sub_lz<2>(fe_sqr_lz(R), PPP), fe_add_lz(Q, Q));  // < 8p
  fe_to2p<8>(X3);
  // R (< 4p) (Q - X3 + 2p < 4p) + (3p - S1) PPP (S1 < 1.1p, PPP < 2p), one unsigned
  // reduction: < 22 p^2 / R' + p < 1.2p, below 2p without a subtraction
  const F Y3 = fe_mul2_redc_u(R, fe_sub_lz<2>(Q, X3), fe_negk_cf<3>(S1), PPP);
  XYZZ<F> r;
  r.x = X3;
  r.y = Y3;
  r.zz = fe_mul_lz(fe_mul_lz(a.zz, b.zz), PP);
  r.zzz = fe_mul_lz(fe_mul_lz(a.zzz, b.zzz), PPP);
  return r;
}

// Affine point in gnark layout (X then Y, each Coord<F>::WORDS u32) -> internal.
template <class F>
GM_DEV Affine<F> load_affine_gnark(const uint32_t* __restrict__ src) {
  Affine<F> r;
  r.x = Coord<F>::load_internal(src);
  r.y = Coord<F>::load_internal(src + Coord<F>::WORDS);
  return r;
}
// Affine point in "packed internal" layout (see Coord::load_packed): the MSM's
// resident point format -- gnark's size (64 B for BN254 G1, 128-B lines hold two
// points, no point straddles a 64-B sector) with no per-load conversion multiply.
template <class F>
GM_DEV Affine<F> load_affine_packed(const uint32_t* __restrict__ src) {
  Affine<F> r;
  r.x = Coord<F>::load_packed(src);
  r.y = Coord<F>::load_packed(src + Coord<F>::WORDS);
  return r;
}
template <class F>
GM_DEV void store_affine_packed(uint32_t* __restrict__ dst, const Affine<F>& a) {
  Coord<F>::store_packed(dst, a.x);
  Coord<F>::store_packed(dst + Coord<F>::WORDS, a.y);
}
template <class F>
GM_DEV void store_affine_gnark(uint32_t* __restrict__ dst, const Affine<F>& a) {
  Coord<F>::store_gnark(dst, a.x);
  Coord<F>::store_gnark(dst + Coord<F>::WORDS, a.y);
}

template <class F>
GM_DEV Affine<F> aff_neg(const Affine<F>& p) {
  Affine<F> r;
  r.x = p.x;
  r.y = fe_neg(p.y);
  return r;
}

// [k]a for a small non-negative integer k (< 2^32), double-and-add from the top.
template <class F>
GM_DEV XYZZ<F> xyzz_mul_small(const XYZZ<F>& a, uint32_t k) {
  XYZZ<F> r = xyzz_inf<F>();
  if (k == 0) return r;
  int top = 31 - __builtin_clz(k);
  r = a;
  for (int b = top - 1; b >= 0; b--) {
    r = xyzz_dbl(r);
    if ((k >> b) & 1) r = xyzz_add(r, a);
  }
  return r;
}

// Curve bundles ---------------------------------------------------------------
using Bn254Fp2 = Fe2<Bn254Fp, -1>;
using Bls377Fp2 = Fe2<Bls377Fp, -5>;

}  // namespace gm
