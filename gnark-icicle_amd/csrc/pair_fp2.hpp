// Fp2 arithmetic with the two components split across a lane pair (G2 bucket
// accumulation).  Lane 2k holds component a0 of an Fp2 element, lane 2k+1 its
// a1; the partner's component comes over DPP (quad_perm [1,0,3,2]).  Each lane
// then needs Fp-sized registers -- a G2 mixed add held whole in one lane needs
// more than the 256 VGPRs a wave can address and spills (BN254: 29 spills,
// BLS12-377: 415) -- and the Fp2 product is computed as ONE Montgomery
// reduction of two accumulated raw products per lane:
//   lane 0: c0 = a0 b0 + BETA a1 b1      lane 1: c1 = a0 b1 + a1 b0
// (2 x N^2 + N^2 mads per lane, 6 N^2 per pair -- the same as three reduced
// Karatsuba products in one lane, with both lanes busy).
// All control flow that depends on values is made pair-uniform (pair_all).
#pragma once
#include "curve.hpp"

namespace gm {

GM_DEV bool pair_odd() { return (threadIdx.x & 1) != 0; }

GM_DEV uint32_t pair_swap32(uint32_t x) {
  // quad_perm [1,0,3,2]: every lane reads its xor-1 neighbour
  return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0xB1, 0xF, 0xF, false);
}
template <class P>
GM_DEV Fe<P> fe_swap(const Fe<P>& a) {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = pair_swap32(a.v[i]);
  return r;
}
// x on both lanes of the pair.  The swap runs on both lanes unconditionally:
// a DPP read of a lane that is switched off returns the reader's own value.
GM_DEV bool pair_all(bool x) {
  const uint32_t mine = x ? 1u : 0u;
  const uint32_t other = pair_swap32(mine);
  return (mine & other) != 0;
}

template <class P>
GM_DEV Fe<P> fe_select(bool c, const Fe<P>& a, const Fe<P>& b) {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// Component of a * b (Fp2 = Fp[u]/(u^2 - BETA)), inputs < 4p per component
// with normalised limbs, result < 1.2p (BN254; ~p for BLS12-377).
//   lane 0: a0 b0 + BETA a1 b1 = a.b + (5p - ap).(|BETA| bp)
//   lane 1: a1 b0 + a0 b1      = a.bp + ap.b
// Lane 0's subtraction is folded into its operand (carry-free 5p - ap), so
// both lanes run ONE unsigned reduction of two products with the same
// instructions: no per-lane sign select in every column, no + p pass and no
// final conditional subtraction (the sum is < (16 + 20) p^2 / R' + p < 1.22p
// for BN254, R' / p ~ 169).
template <class P, int BETA, bool CH = false>
GM_DEV Fe<P> pf2_mul(const Fe<P>& a, const Fe<P>& b) {
  static_assert(BETA == -1 || BETA == -5, "unsupported non-residue");
  const bool odd = pair_odd();
  const Fe<P> ap = fe_swap(a), bp = fe_swap(b);
  Fe<P> y2 = odd ? b : bp;
  if constexpr (BETA == -5) {
    const Fe<P> b5 = fe_times5_lz(bp);  // < 20p, normalised limbs
    y2 = fe_select(odd, b, b5);
  }
  return fe_mul2_redc_u<P, CH>(a, fe_select(odd, bp, b), fe_select(odd, ap, fe_negk_cf<5>(ap)), y2);
}

// x1 y1 + x2 y2 - x3 y3 - x4 y4 + p in ONE Montgomery reduction (signed columns:
// the positive side of a column is <= 27 * 2^58 < 2^63 for N = 9, the negative
// <= 18 * 2^58).  Inputs with normalised limbs; for the BN254 G2 Y3 below the
// negative products are < 20 p^2 < p R', so the result is >= 0, and < 2.3p.
template <class P>
GM_DEV Fe<P> fe_mul4_redc(const Fe<P>& x1, const Fe<P>& y1, const Fe<P>& x2, const Fe<P>& y2, const Fe<P>& x3,
                          const Fe<P>& y3, const Fe<P>& x4, const Fe<P>& y4) {
  constexpr int N = P::N;
  static_assert(N <= 9, "signed column bound needs N <= 9");
  uint32_t m[N];
  Fe<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t cp = 0, cn = 0;
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++) {
      cp += (uint64_t)x1.v[i] * y1.v[k - i] + (uint64_t)x2.v[i] * y2.v[k - i];
      cn += (uint64_t)x3.v[i] * y3.v[k - i] + (uint64_t)x4.v[i] * y4.v[k - i];
    }
    acc += cp - cn;
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k - 1 < N - 1 ? k - 1 : N - 1); i++)
      acc += (uint64_t)m[i] * P::p(k - i);
    if (k < N) {
      m[k] = ((uint32_t)acc * P::INV) & LIMB_MASK;
      acc += (uint64_t)m[k] * P::p(0);
    } else {
      r.v[k - N] = (uint32_t)acc & LIMB_MASK;
    }
    acc = (uint64_t)((int64_t)acc >> RADIX);
  }
  r.v[N - 1] = (uint32_t)acc;  // two's complement top limb when negative
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {  // + p
    const uint32_t sm = r.v[i] + P::p(i) + c;
    r.v[i] = i == N - 1 ? sm : (sm & LIMB_MASK);
    c = sm >> RADIX;
  }
  return r;
}

// Component of R W - Y PP (Fp2, BETA = -1) as ONE reduction of four products
// per lane (fe_mul4_redc):
//   lane 0: R0 W0 + Y1 P1 - R1 W1 - Y0 P0     lane 1: R1 W0 + R0 W1 - Y1 P0 - Y0 P1
// Inputs normalised, R, W < 4p, Y, PP < 2p (negative side < 20 p^2 < p R');
// result < 2.3p.  Used for Y3 of the mixed add and of the full add / doubling.
template <class P>
GM_DEV Fe<P> pf2_mul_sub(const Fe<P>& R, const Fe<P>& W, const Fe<P>& Y, const Fe<P>& PP) {
  const bool odd = pair_odd();
  const Fe<P> Rp = fe_swap(R), Wp = fe_swap(W), Yp = fe_swap(Y), Pp = fe_swap(PP);
  return fe_mul4_redc(R, fe_select(odd, Wp, W), fe_select(odd, Rp, Yp), fe_select(odd, W, Pp),
                      fe_select(odd, Y, Rp), fe_select(odd, Pp, Wp), fe_select(odd, Yp, Y), PP);
}

// Component of a^2, inputs < IN p per component, result < 2p.
template <class P, int BETA, int IN, bool CH = false>
GM_DEV Fe<P> pf2_sqr(const Fe<P>& a) {
  if constexpr (BETA == -1) {
    static_assert(IN <= 4, "pf2_sqr output bound (< 2p) needs inputs < 4p");
    // lane 0: (a0 + a1)(a0 - a1);  lane 1: 2 a1 a0
    const bool odd = pair_odd();
    const Fe<P> ap = fe_swap(a);
    const Fe<P> u = fe_add_lz(a, odd ? a : ap);
    const Fe<P> v = odd ? ap : fe_sub_lz<IN>(a, ap);
    // u < 2 IN p, v < 2 IN p: (2 IN p)^2 / R' + p < 1.4p for IN <= 4 (BN254
    // R' / p ~ 169): already below 2p, no conditional subtraction
    return fe_mul<P, false, CH>(u, v);
  } else {
    return pf2_mul<P, BETA, CH>(a, a);
  }
}

// XYZZ point, this lane's components
template <class P>
struct PXYZZ {
  Fe<P> x, y, zz, zzz;
};

template <class P>
GM_DEV PXYZZ<P> pxyzz_inf() {
  // infinity: zz = zzz = 0 (x, y = 1 as in xyzz_inf: component a0 = 1, a1 = 0)
  PXYZZ<P> r;
  const Fe<P> one = pair_odd() ? fe_zero<P>() : fe_one<P>();
  r.x = one;
  r.y = one;
  r.zz = fe_zero<P>();
  r.zzz = fe_zero<P>();
  return r;
}
template <class P>
GM_DEV bool pxyzz_is_inf(const PXYZZ<P>& a) {
  return pair_all(fe_is_zero(a.zz));
}

// 2 P for affine P (canonical components, not infinity) -- the rare
// accumulation case "bucket == point"; results canonicalised.
template <class P, int BETA>
GM_DEV PXYZZ<P> pxyzz_dbl_aff(const Fe<P>& px, const Fe<P>& py) {
  const Fe<P> U = fe_add_lz(py, py);                               // < 2p
  const Fe<P> V = pf2_sqr<P, BETA, 2>(U);                          // < 2p
  const Fe<P> Wv = pf2_mul<P, BETA>(U, V);
  const Fe<P> S = pf2_mul<P, BETA>(px, V);
  const Fe<P> X2 = pf2_sqr<P, BETA, 1>(px);                        // < 2p
  Fe<P> M = fe_add_lz(fe_add_lz(X2, X2), X2);                      // < 6p
  fe_to2p<8>(M);                                                   // < 2p
  PXYZZ<P> r;
  Fe<P> X3 = fe_sub_lz<4>(pf2_sqr<P, BETA, 2>(M), fe_add_lz(S, S));  // < 6p
  fe_to2p<8>(X3);
  Fe<P> Y3 = fe_sub_lz<2>(pf2_mul<P, BETA>(M, fe_sub_lz<2>(S, X3)), pf2_mul<P, BETA>(Wv, py));  // < 4p
  r.x = fe_canon<3>(X3);
  r.y = fe_canon<2>(Y3);
  r.zz = fe_canon<1>(V);
  r.zzz = fe_canon<1>(Wv);
  return r;
}

// a += (neg ? -P : P) (P affine, canonical components; infinity (0,0)
// skipped).  Invariants on a: every component < 2p (as xyzz_add_aff_lz for
// Fe2).  BN254: as in the G1 add, the sign goes onto S2 (carry-free 2p - S2 per
// component) and X3 takes one borrow chain (G2 2^20 accumulation 5.18 -> 5.13
// ms).  BLS12-377 keeps y negated up front and three chains: its 14-limb add
// already spills at three waves per SIMD, and the trimmed form spilled more
// (171 -> 185 VGPRs, 2^22 accumulation 46.5 -> 47.4 ms; profiles/r03e_ab.txt).
// CH: one mad chain per product (fe_mul CHAIN) in the add's products
template <class P, int BETA, bool CH = false>
GM_DEV void pxyzz_add_aff(PXYZZ<P>& a, const Fe<P>& px, const Fe<P>& py_in, bool neg) {
  static_assert(P::BITS + 7 <= RADIX * P::N, "lazy reduction needs R' > 128 p");
  constexpr bool TRIM = P::N <= 9;
  if (pair_all(fe_is_zero(px) && fe_is_zero(py_in))) return;
  Fe<P> py = py_in;
  if constexpr (!TRIM) {
    if (neg) py = fe_neg(py_in);
  }
  if (pxyzz_is_inf(a)) {
    a.x = px;
    a.y = (TRIM && neg) ? fe_neg(py) : py;
    a.zz = pair_odd() ? fe_zero<P>() : fe_one<P>();
    a.zzz = a.zz;
    return;
  }
  const Fe<P> Pd = fe_sub_lz<2>(pf2_mul<P, BETA, CH>(px, a.zz), a.x);    // U2 - X1   < 4p
  Fe<P> R;                                                          // +-S2 - Y1 < 4p
  if constexpr (TRIM) {
    // S2 < 2p; 2p - S2 in (0, 2p]
    R = fe_sub_lz<2>(fe_cneg2p_cf(pf2_mul<P, BETA, CH>(py, a.zzz), neg), a.y);
  } else {
    R = fe_sub_lz<2>(pf2_mul<P, BETA, CH>(py, a.zzz), a.y);
  }
  if (pair_all(fe_is_zero_lz<4>(Pd))) {
    if (pair_all(fe_is_zero_lz<4>(R))) a = pxyzz_dbl_aff<P, BETA>(px, (TRIM && neg) ? fe_neg(py) : py);
    else a = pxyzz_inf<P>();
    return;
  }
  const Fe<P> PP = pf2_sqr<P, BETA, 4, CH>(Pd);                     // < 2p
  const Fe<P> PPP = pf2_mul<P, BETA, CH>(Pd, PP);                   // < 2p
  a.zz = pf2_mul<P, BETA, CH>(a.zz, PP);
  const Fe<P> Q = pf2_mul<P, BETA, CH>(a.x, PP);                    // < 2p
  a.zzz = pf2_mul<P, BETA, CH>(a.zzz, PPP);
  Fe<P> X3;                                                         // < 8p
  if constexpr (TRIM) {
    X3 = fe_sub2x_lz<6>(pf2_sqr<P, BETA, 4, CH>(R), PPP, Q);
  } else {
    X3 = fe_sub_lz<4>(fe_sub_lz<2>(pf2_sqr<P, BETA, 4, CH>(R), PPP), fe_add_lz(Q, Q));
  }
  fe_to2p<8>(X3);
  Fe<P> Y3;
  if constexpr (TRIM && BETA == -1) {
    // Y3 = R W - Y1 PPP (W = Q - X3) as ONE reduction of four products per lane:
    //   lane 0: R0 W0 + Y1 P1 - R1 W1 - Y0 P0     lane 1: R1 W0 + R0 W1 - Y1 P0 - Y0 P1
    Y3 = pf2_mul_sub(R, fe_sub_lz<2>(Q, X3), a.y, PPP);  // < 2.3p
  } else {
    Y3 = fe_sub_lz<2>(pf2_mul<P, BETA, CH>(R, fe_sub_lz<2>(Q, X3)), pf2_mul<P, BETA, CH>(a.y, PPP));  // < 4p
  }
  fe_to2p<4>(Y3);
  a.x = X3;
  a.y = Y3;
}

// ---------------------------------------------------------------------------
// G2 bucket accumulation on lane pairs: the k_msm_accum_seg contract (slices of
// K sorted entries, buckets cut by slice edges to part_first / part_last) with
// slice t owned by lanes 2t (component a0 of every coordinate) and 2t+1 (a1).
// Everything that steers control flow (keys, vals, slice bounds) is read by
// both lanes alike, so the pair stays converged; value tests go through
// pair_all.  Buckets are written in the XYZZ<Fe2> layout, canonical.
// ---------------------------------------------------------------------------
template <class P>
GM_DEV void pair_emit_coord(uint32_t* __restrict__ dst, const Fe<P>& a) {
#pragma unroll
  for (int i = 0; i < P::N; i++) dst[i] = a.v[i];
}
template <class P>
GM_DEV void pair_emit(uint32_t* __restrict__ xyzz, const PXYZZ<P>& a) {
  // XYZZ<Fe2<P>> = {x.a0, x.a1, y.a0, y.a1, zz.a0, zz.a1, zzz.a0, zzz.a1}
  uint32_t* d = xyzz + (pair_odd() ? P::N : 0);
  pair_emit_coord<P>(d, fe_canon<1>(a.x));
  pair_emit_coord<P>(d + 2 * P::N, fe_canon<1>(a.y));
  pair_emit_coord<P>(d + 4 * P::N, fe_canon<1>(a.zz));
  pair_emit_coord<P>(d + 6 * P::N, fe_canon<1>(a.zzz));
}

// this lane's components (x, y) of a packed Fe2 affine point, as gnark words
template <class P>
struct PairPt {
  FeG<P> x, y;
};
template <class P>
GM_DEV PairPt<P> pair_load_pt(const uint32_t* __restrict__ pt) {
  const int c = pair_odd() ? P::NG : 0;
  return {feg_load<P>(pt + c), feg_load<P>(pt + 2 * P::NG + c)};
}

#ifndef GM_PAIR_WPE
#define GM_PAIR_WPE 1  // no cap; per-TU override (msm_bls12377_g2.hip)
#endif
// PF: prefetch the next point's components (2 x NG registers) while the
// current add runs; without it the other waves hide the load (GM_MSM_PAIR_PF=0).
// WPE: waves-per-SIMD floor for the register allocator (1 = no cap).
template <class P, int BETA, bool PF = true, int WPE = GM_PAIR_WPE, bool V4 = false, bool CH = false>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(WPE)))
k_msm_accum_seg_pair(const uint32_t* __restrict__ points, uint32_t n,
                                                            const uint32_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ vals,
                                                            const uint32_t* __restrict__ offsets, uint32_t total,
                                                            uint32_t K, uint32_t* __restrict__ buckets,
                                                            uint32_t* __restrict__ part_first,
                                                            uint32_t* __restrict__ part_last,
                                                            uint32_t* __restrict__ err) {
  constexpr int XW = 8 * P::N;      // u32 words of one XYZZ<Fe2<P>>
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  const uint32_t Mv = offsets[total];
  const uint32_t start = t * K;
  if (start >= Mv) return;
  const uint32_t end = min(start + K, Mv);
  auto emit = [&](uint32_t b, const PXYZZ<P>& acc, bool is_first, bool is_last) {
    const uint32_t bs = offsets[b], be = offsets[b + 1];
    if (bs >= start && be <= end) {
      pair_emit<P>(buckets + (size_t)b * XW, acc);
    } else {
      if (is_first) pair_emit<P>(part_first + (size_t)t * XW, acc);
      if (is_last) pair_emit<P>(part_last + (size_t)t * XW, acc);
    }
  };
  // keys / values in 16-byte groups of four entries (as accum_seg_body_v4: one
  // load per four entries instead of a strided 4-byte load per entry; slices
  // start at multiples of K, K % 4 == 0 for V4, reads stay in the arena's
  // 256-byte-rounded allocation)
  uint4 kg, vg;
  if constexpr (V4) {
    kg = *reinterpret_cast<const uint4*>(keys + start);
    vg = *reinterpret_cast<const uint4*>(vals + start);
  } else {
    kg.x = keys[start];
    vg.x = vals[start];
  }
  uint32_t v = vg.x;
  uint32_t cur = kg.x;
  bool first = true;
  PXYZZ<P> acc = pxyzz_inf<P>();
  if ((v & 0x7fffffffu) >= n) {
    if (!pair_odd()) atomicOr(err, 2u);
    return;
  }
  PairPt<P> pt = pair_load_pt<P>(points + (size_t)(v & 0x7fffffffu) * 4 * P::NG);
  for (uint32_t q = start; q < end; q++) {
    uint32_t k;
    if constexpr (V4) {
      k = kg.x;
      if (((q - start) & 3) == 3) {
        if (q + 1 < end) {
          kg = *reinterpret_cast<const uint4*>(keys + q + 1);
          vg = *reinterpret_cast<const uint4*>(vals + q + 1);
        }
      } else {
        kg = make_uint4(kg.y, kg.z, kg.w, kg.w);
        vg = make_uint4(vg.y, vg.z, vg.w, vg.w);
      }
    } else {
      k = keys[q];
    }
    // prefetch the next point's components while this add runs
    uint32_t vn = 0;
    PairPt<P> ptn;
    if (q + 1 < end) {
      vn = V4 ? vg.x : vals[q + 1];
      if ((vn & 0x7fffffffu) >= n) {
        if (!pair_odd()) atomicOr(err, 2u);
        return;
      }
      if (PF) ptn = pair_load_pt<P>(points + (size_t)(vn & 0x7fffffffu) * 4 * P::NG);
    }
    if (!PF) pt = pair_load_pt<P>(points + (size_t)(v & 0x7fffffffu) * 4 * P::NG);
    if (k != cur) {
      emit(cur, acc, first, false);
      first = false;
      acc = pxyzz_inf<P>();
      cur = k;
    }
    const Fe<P> px = fe_unpack<P>(pt.x);
    const Fe<P> py = fe_unpack<P>(pt.y);
    pxyzz_add_aff<P, BETA, CH>(acc, px, py, (v >> 31) != 0);
    v = vn;
    if (PF) pt = ptn;
  }
  emit(cur, acc, first, true);
}


// ---------------------------------------------------------------------------
// Full XYZZ arithmetic on lane pairs (bucket fixup and reduction), canonical
// components in and out -- the pair form of xyzz_dbl / xyzz_add (curve.hpp):
// the one-lane G2 versions keep two whole Fp2 points live and spill (BLS12-377
// k_msm_seg: 375 VGPRs spilled).
// ---------------------------------------------------------------------------
template <class P>
GM_DEV PXYZZ<P> pxyzz_load(const uint32_t* __restrict__ xyzz) {
  const uint32_t* s = xyzz + (pair_odd() ? P::N : 0);
  PXYZZ<P> r;
#pragma unroll
  for (int i = 0; i < P::N; i++) {
    r.x.v[i] = s[i];
    r.y.v[i] = s[2 * P::N + i];
    r.zz.v[i] = s[4 * P::N + i];
    r.zzz.v[i] = s[6 * P::N + i];
  }
  return r;
}
// canonical a stored as is
template <class P>
GM_DEV void pxyzz_store(uint32_t* __restrict__ xyzz, const PXYZZ<P>& a) {
  uint32_t* d = xyzz + (pair_odd() ? P::N : 0);
  pair_emit_coord<P>(d, a.x);
  pair_emit_coord<P>(d + 2 * P::N, a.y);
  pair_emit_coord<P>(d + 4 * P::N, a.zz);
  pair_emit_coord<P>(d + 6 * P::N, a.zzz);
}

// 2 a (dbl-2008-s-1), canonical in / out; infinity -> infinity.
template <class P, int BETA>
GM_DEV PXYZZ<P> pxyzz_dbl(const PXYZZ<P>& a) {
  const Fe<P> U = fe_add_lz(a.y, a.y);                               // < 2p
  const Fe<P> V = pf2_sqr<P, BETA, 2>(U);                            // < 2p
  const Fe<P> Wv = pf2_mul<P, BETA>(U, V);
  const Fe<P> S = pf2_mul<P, BETA>(a.x, V);
  const Fe<P> X2 = pf2_sqr<P, BETA, 1>(a.x);
  Fe<P> M = fe_add_lz(fe_add_lz(X2, X2), X2);                        // < 6p
  fe_to2p<8>(M);
  Fe<P> X3 = fe_sub_lz<4>(pf2_sqr<P, BETA, 2>(M), fe_add_lz(S, S));  // < 6p
  fe_to2p<8>(X3);
  Fe<P> Y3;  // M (S - X3) - Wv Y1
  if constexpr (BETA == -1 && P::N <= 9) {
    Y3 = pf2_mul_sub(M, fe_sub_lz<2>(S, X3), Wv, a.y);  // < 2.3p: one reduction of four products
  } else {
    Y3 = fe_sub_lz<2>(pf2_mul<P, BETA>(M, fe_sub_lz<2>(S, X3)), pf2_mul<P, BETA>(Wv, a.y));  // < 4p
  }
  PXYZZ<P> r;
  r.x = fe_canon<1>(X3);
  r.y = fe_canon<2>(Y3);
  r.zz = fe_canon<1>(pf2_mul<P, BETA>(V, a.zz));
  r.zzz = fe_canon<1>(pf2_mul<P, BETA>(Wv, a.zzz));
  return r;
}

// a + b (add-2008-s) with all special cases, canonical in / out.
template <class P, int BETA>
GM_DEV PXYZZ<P> pxyzz_add(const PXYZZ<P>& a, const PXYZZ<P>& b) {
  if (pxyzz_is_inf(a)) return b;
  if (pxyzz_is_inf(b)) return a;
  const Fe<P> U1 = pf2_mul<P, BETA>(a.x, b.zz);                      // < 2p
  const Fe<P> U2 = pf2_mul<P, BETA>(b.x, a.zz);
  const Fe<P> S1 = pf2_mul<P, BETA>(a.y, b.zzz);
  const Fe<P> S2 = pf2_mul<P, BETA>(b.y, a.zzz);
  const Fe<P> Pd = fe_sub_lz<2>(U2, U1);                             // < 4p
  const Fe<P> R = fe_sub_lz<2>(S2, S1);                              // < 4p
  if (pair_all(fe_is_zero_lz<4>(Pd))) {
    if (pair_all(fe_is_zero_lz<4>(R))) return pxyzz_dbl<P, BETA>(a);
    return pxyzz_inf<P>();
  }
  const Fe<P> PP = pf2_sqr<P, BETA, 4>(Pd);                          // < 2p
  const Fe<P> PPP = pf2_mul<P, BETA>(Pd, PP);
  const Fe<P> Q = pf2_mul<P, BETA>(U1, PP);
  Fe<P> X3 = fe_sub_lz<4>(fe_sub_lz<2>(pf2_sqr<P, BETA, 4>(R), PPP), fe_add_lz(Q, Q));  // < 8p
  fe_to2p<8>(X3);
  Fe<P> Y3;  // R (Q - X3) - S1 PPP
  if constexpr (BETA == -1 && P::N <= 9) {
    Y3 = pf2_mul_sub(R, fe_sub_lz<2>(Q, X3), S1, PPP);  // < 2.3p: one reduction of four products
  } else {
    Y3 = fe_sub_lz<2>(pf2_mul<P, BETA>(R, fe_sub_lz<2>(Q, X3)), pf2_mul<P, BETA>(S1, PPP));  // < 4p
  }
  PXYZZ<P> r;
  r.x = fe_canon<1>(X3);
  r.y = fe_canon<2>(Y3);
  r.zz = fe_canon<1>(pf2_mul<P, BETA>(pf2_mul<P, BETA>(a.zz, b.zz), PP));
  r.zzz = fe_canon<1>(pf2_mul<P, BETA>(pf2_mul<P, BETA>(a.zzz, b.zzz), PPP));
  return r;
}

// Pair forms of k_msm_fixup / k_msm_fix_tree / k_msm_fixup_long / k_msm_seg
// (msm_impl.hpp; same contracts, buffers as XYZZ<Fe2<P>> words, pair per task).
template <class P, int BETA>
__global__ void __launch_bounds__(128) k_msm_fixup_pair(const uint32_t* __restrict__ offsets, uint32_t total,
                                                        uint32_t K, uint32_t* __restrict__ buckets,
                                                        const uint32_t* __restrict__ part_first,
                                                        const uint32_t* __restrict__ part_last,
                                                        uint32_t* __restrict__ maxspan, uint32_t fix_serial) {
  constexpr int XW = 8 * P::N;
  const uint32_t b = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (b >= total) return;
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t0 == t1) return;
  if (t1 - t0 > fix_serial) {
    if (!pair_odd()) atomicMax(maxspan, t1 - t0);
    return;
  }
  PXYZZ<P> acc = pxyzz_load<P>(part_last + (size_t)t0 * XW);
  for (uint32_t t = t0 + 1; t <= t1; t++) acc = pxyzz_add<P, BETA>(acc, pxyzz_load<P>(part_first + (size_t)t * XW));
  pxyzz_store<P>(buckets + (size_t)b * XW, acc);
}

// k_msm_fixup_edge (msm_impl.hpp) on lane pairs: one pair per slice edge t >= 1
template <class P, int BETA>
__global__ void __launch_bounds__(128) k_msm_fixup_edge_pair(const uint32_t* __restrict__ keys,
                                                             const uint32_t* __restrict__ offsets, uint32_t total,
                                                             uint32_t K, uint32_t nslices,
                                                             uint32_t* __restrict__ buckets,
                                                             const uint32_t* __restrict__ part_first,
                                                             const uint32_t* __restrict__ part_last,
                                                             uint32_t* __restrict__ maxspan, uint32_t fix_serial) {
  constexpr int XW = 8 * P::N;
  const uint32_t t = ((blockIdx.x * blockDim.x + threadIdx.x) >> 1) + 1;
  if (t >= nslices) return;
  const size_t q = (size_t)t * K;
  if (q >= offsets[total]) return;
  const uint32_t b = keys[q];
  const uint32_t bs = offsets[b];
  if (bs >= q || bs / K != t - 1) return;
  const uint32_t t0 = t - 1, t1 = (offsets[b + 1] - 1) / K;
  if (t1 - t0 > fix_serial) {
    if (!pair_odd()) atomicMax(maxspan, t1 - t0);
    return;
  }
  PXYZZ<P> acc = pxyzz_load<P>(part_last + (size_t)t0 * XW);
  for (uint32_t u = t; u <= t1; u++) acc = pxyzz_add<P, BETA>(acc, pxyzz_load<P>(part_first + (size_t)u * XW));
  pxyzz_store<P>(buckets + (size_t)b * XW, acc);
}

template <class P, int BETA>
__global__ void __launch_bounds__(128) k_msm_fix_tree_pair(const uint32_t* __restrict__ keys,
                                                           const uint32_t* __restrict__ offsets, uint32_t total,
                                                           uint32_t K, uint32_t nslices, uint32_t d,
                                                           uint32_t* __restrict__ part_first, uint32_t fix_serial) {
  constexpr int XW = 8 * P::N;
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (t >= nslices || (size_t)t * K >= offsets[total]) return;
  const uint32_t b = keys[(size_t)t * K];
  const uint32_t t0 = offsets[b] / K, t1 = (offsets[b + 1] - 1) / K;
  if (t1 - t0 <= fix_serial || t <= t0) return;
  const uint32_t rel = t - (t0 + 1), len = t1 - t0, step = 1u << d;
  if ((rel & ((step << 1) - 1)) == 0 && rel + step < len) {
    const PXYZZ<P> r = pxyzz_add<P, BETA>(pxyzz_load<P>(part_first + (size_t)t * XW),
                                          pxyzz_load<P>(part_first + (size_t)(t + step) * XW));
    pxyzz_store<P>(part_first + (size_t)t * XW, r);
  }
}

template <class P, int BETA>
__global__ void __launch_bounds__(128) k_msm_fixup_long_pair(const uint32_t* __restrict__ offsets, uint32_t total,
                                                             uint32_t K, uint32_t* __restrict__ buckets,
                                                             const uint32_t* __restrict__ part_first,
                                                             const uint32_t* __restrict__ part_last,
                                                             uint32_t fix_serial) {
  constexpr int XW = 8 * P::N;
  const uint32_t b = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (b >= total) return;
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t1 - t0 <= fix_serial) return;
  const PXYZZ<P> r = pxyzz_add<P, BETA>(pxyzz_load<P>(part_last + (size_t)t0 * XW),
                                        pxyzz_load<P>(part_first + (size_t)(t0 + 1) * XW));
  pxyzz_store<P>(buckets + (size_t)b * XW, r);
}

// (empty buckets read as infinity, as in k_msm_seg)
template <class P, int BETA>
__global__ void __launch_bounds__(128) k_msm_seg_pair(const uint32_t* __restrict__ buckets,
                                                      const uint32_t* __restrict__ offsets, uint32_t nb, uint32_t L,
                                                      uint32_t nseg, uint32_t W, uint32_t* __restrict__ nodes) {
  constexpr int XW = 8 * P::N;
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (t >= W * nseg) return;
  const uint32_t w = t / nseg, s = t % nseg;
  const size_t b0 = (size_t)w * nb + (size_t)s * L;
  const uint32_t* B = buckets + b0 * XW;
  const uint32_t* O = offsets + b0;
  uint32_t o_hi = O[L];
  uint32_t o_lo = O[L - 1];
  PXYZZ<P> S = o_lo == o_hi ? pxyzz_inf<P>() : pxyzz_load<P>(B + (size_t)(L - 1) * XW), T = S;
  for (int j = (int)L - 2; j >= 0; j--) {
    o_hi = o_lo;
    o_lo = O[j];
    S = pxyzz_add<P, BETA>(S, o_lo == o_hi ? pxyzz_inf<P>() : pxyzz_load<P>(B + (size_t)j * XW));
    T = pxyzz_add<P, BETA>(T, S);
  }
  pxyzz_store<P>(nodes + 2 * (size_t)t * XW, S);
  pxyzz_store<P>(nodes + (2 * (size_t)t + 1) * XW, T);
}

// k_msm_bitsum on lane pairs: 512 threads = 256 pairs, two tasks per pair.
constexpr uint32_t BS_PAIR_THREADS = 512;
template <class P, int BETA>
__global__ void __launch_bounds__(BS_PAIR_THREADS) k_msm_bitsum_pair(const uint32_t* __restrict__ in, uint32_t m,
                                                                  uint32_t Qin, uint32_t NT, uint32_t lgNT,
                                                                  uint32_t* __restrict__ out) {
  constexpr int XW = 8 * P::N;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem_words[];
  uint32_t* X = smem_words;
  const uint32_t groups = m / NT;
  const uint32_t w = blockIdx.x / groups, j = blockIdx.x % groups;
  const uint32_t* src = in + ((size_t)w * m + (size_t)j * NT) * Qin * XW;
  for (uint32_t q = threadIdx.x; q < NT * Qin * XW; q += blockDim.x) X[q] = src[q];
  __syncthreads();
  const uint32_t pt = threadIdx.x >> 1, npairs = blockDim.x >> 1;
  for (uint32_t d = 0; d < lgNT; d++) {
    const uint32_t qc = Qin + d + 1;
    const uint32_t tasks = (NT >> (d + 1)) * qc;
    const uint32_t child = (Qin << d);
    // the pair's two tasks one after the other, one result live at a time.  A
    // task's only read slot that another task writes is base + child at d = 0
    // (written by task (p, Qin), read by the earlier-numbered task (p, 0)), so
    // the second round never reads what the first one changed.
    for (uint32_t t = pt; t < 2 * npairs; t += npairs) {
      PXYZZ<P> r;
      uint32_t slot = 0xffffffffu;
      if (t < tasks) {
        const uint32_t p = t / qc, q = t % qc, base = p * 2 * child;
        r = (q + 1 < qc) ? pxyzz_add<P, BETA>(pxyzz_load<P>(X + (base + q) * XW), pxyzz_load<P>(X + (base + child + q) * XW))
                         : pxyzz_load<P>(X + (base + child) * XW);
        slot = base + q;
      }
      __syncthreads();
      if (slot != 0xffffffffu) pxyzz_store<P>(X + slot * XW, r);
      __syncthreads();
    }
  }
  const uint32_t Qout = Qin + lgNT;
  uint32_t* dst = out + ((size_t)w * groups + j) * Qout * XW;
  for (uint32_t q = threadIdx.x; q < Qout * XW; q += blockDim.x) dst[q] = X[q];
}

}  // namespace gm
