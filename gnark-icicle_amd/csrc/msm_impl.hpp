#pragma once
// Pippenger bucket MSM on gfx950 -- replaces iciclegnark MsmOnDevice /
// MsmG2OnDevice (backend/groth16/bn254/icicle/icicle.go:302,315,332,355,382).
//
// Pipeline (one HIP stream, all state in HBM; msm_plan + msm_run below):
//   1. k_msm_digits / k_msm_s1_scatter   Montgomery -> canonical scalar, signed
//                       c-bit digits of all W windows; non-zero digits are
//                       partitioned into coarse bins (bucket >> F) -- pass 1 of a
//                       hand-written two-level counting sort (no library sort).
//   2. k_msm_s2_*       (msm_sort.hip) each coarse bin -> its buckets: sorted
//                       (bucket, point index | sign << 31) entries and the bucket
//                       start offsets, written directly.
//   3. k_msm_accum_seg  load-balanced slices of K sorted entries per thread:
//                       lazily reduced XYZZ mixed adds of the gathered points
//                       (sign applied on load); buckets cut by slice edges go to
//                       part_first / part_last and are merged by k_msm_fixup
//                       (k_msm_fix_tree + k_msm_fixup_long for spans > FIX_SERIAL).
//   4. k_msm_seg        bucket reduction level 1: running sums over segments of
//                       L buckets;  k_msm_bitsum: LDS bit-sum trees up to one node
//                       per window;  k_msm_export: nodes -> gnark words.
//   5. host: Horner over the window / bit-position nodes, XYZZ -> Jacobian.
// With a precomputed point set (MsmPrecomp) every window shares one bucket set
// and steps 4-5 run once.
//
// Exact group arithmetic: the result is independent of summation order.
#include "curves.hpp"
#include "msm.hpp"
#include "pair_fp2.hpp"
#include "runtime.hpp"

#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace gm {

// ---------------------------------------------------------------------------
// scalar digits
// ---------------------------------------------------------------------------
template <class Fr>
GM_DEV uint32_t window_bits(const FeG<Fr>& k, uint32_t bit, uint32_t mask) {
  const uint32_t idx = bit >> 5, sh = bit & 31;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < Fr::NG; i++) {
    lo = (idx == (uint32_t)i) ? k.w[i] : lo;
    hi = (idx + 1 == (uint32_t)i) ? k.w[i] : hi;
  }
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  return (uint32_t)(v >> sh) & mask;
}

// gnark Montgomery fr.Element -> canonical integer as packed u32 words
template <class Fr>
GM_DEV FeG<Fr> load_scalar_canonical(const uint32_t* __restrict__ s, uint32_t i) {
  return fe_pack(fe_gnark_to_canonical(fe_load_g<Fr>(s, i)));
}

// Plain layout: bucket b = w*nb + |d|-1 (window-major), entry value = point
// index | sign << 31.  Precomputed (shared-bucket) layout: b = |d|-1 for every
// window, value = w*stride + i (the shifted copy) | sign << 31.
// Windows 0..wn-1 are c bits wide, windows wn..W-1 (the `narrow` windows) c - 1
// bits, with c W - narrow = bits + 1: no window is left with only the few top
// bits of the scalar (precomputed layouts, msm.hpp MsmPrecomp, and plain
// non-GLV layouts; a plain 2^24 BN254 MSM at c = 20 has 8 windows of 20 bits
// and 5 of 19 instead of a 15-bit top window whose 2^14 buckets hold ~1024
// points each -- spans of 16 slices that need the tree fixup).
struct DigitGeom {
  uint32_t n, c, W, nb, shared_stride, F;  // F: pass-1 bin = b >> F
  uint32_t wn;
};
// bit offset and width of window w
GM_HD void window_geom(uint32_t c, uint32_t wn, uint32_t w, uint32_t& off, uint32_t& cw) {
  off = w * c - (w > wn ? w - wn : 0u);
  cw = w >= wn ? c - 1 : c;
}

// ---------------------------------------------------------------------------
// Bucket sort of the digits: a two-level counting sort written for this job.
// Order inside a bucket is irrelevant (group addition is exact), so no pass has
// to be stable, and zero digits are dropped at the source.
//   k_msm_digits     (here, per scalar field) one thread per point: the W
//                    signed digits, stored window-major (coalesced) as
//                    dig[w*n + i] = (|d|-1) | sign << 31 (~0: zero digit), and
//                    the coarse histogram (bin H = bucket >> F; LDS, then one
//                    global atomic per bin per block)
//   msm_sort.hip     k_msm_s1_scan: coarse bases; k_msm_s1_scatter: one block
//                    per (window, 8K points) partitions those digits into the
//                    coarse bins (a plain-layout block only touches its own
//                    window's bins, so its write runs are long); pass 2 sorts
//                    every coarse bin into its 2^F buckets and writes the
//                    sorted keys / values and the bucket offsets directly.
// ---------------------------------------------------------------------------
constexpr uint32_t DG_THREADS = 1024, DG_PPT = 4;

template <class Fr>
__global__ void __launch_bounds__(1024) k_msm_digits(const uint32_t* __restrict__ scalars, DigitGeom g,
                                                     uint32_t NC, uint32_t* __restrict__ dig,
                                                     uint32_t* __restrict__ ccount) {
  extern __shared__ uint32_t dg_lds[];
  const uint32_t t = threadIdx.x;
  for (uint32_t q = t; q < NC; q += DG_THREADS) dg_lds[q] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * DG_THREADS * DG_PPT;
  for (uint32_t r = 0; r < DG_PPT; r++) {
    const uint32_t i = base + r * DG_THREADS + t;
    if (i >= g.n) break;
    const FeG<Fr> k = load_scalar_canonical<Fr>(scalars, i);
    uint32_t carry = 0;
    for (uint32_t w = 0; w < g.W; w++) {
      uint32_t off, cw;
      window_geom(g.c, g.wn, w, off, cw);
      const uint32_t raw = window_bits(k, off, (1u << cw) - 1) + carry;
      uint32_t d, neg;
      if (raw > (1u << (cw - 1))) {
        d = (1u << cw) - raw;
        carry = 1;
        neg = 1;
      } else {
        d = raw;
        carry = 0;
        neg = 0;
      }
      dig[(size_t)w * g.n + i] = d ? (d - 1) | (neg << 31) : 0xffffffffu;
      if (d) atomicAdd(&dg_lds[(g.shared_stride ? d - 1 : w * g.nb + d - 1) >> g.F], 1u);
    }
  }
  __syncthreads();
  for (uint32_t q = t; q < NC; q += DG_THREADS)
    if (dg_lds[q]) atomicAdd(&ccount[q], dg_lds[q]);
}

// ---------------------------------------------------------------------------
// GLV split for BN254 G1: phi(x, y) = (beta x, y) = [lambda] P with beta, lambda
// primitive cube roots of unity (p resp. r).  Short lattice basis of
// {(a, b) : a + b lambda = 0 mod r}: v1 = (a1, b1), v2 = (a2, b2) with
// a1 = b2 - |b1| ~ 2^126.8, b1 = -a2, a2 ~ 2^63.1.  c1 = floor(k g1 / 2^384),
// c2 = floor(k g2 / 2^384) with g1 = floor(2^384 b2 / r), g2 = floor(2^384 |b1| / r)
// undershoot b2 k / r and |b1| k / r by e1, e2 in [0, 1 + 2^-130), so
// k1 = k - c1 a1 - c2 a2 = e1 a1 + e2 a2 lies in [0, 2^127) and
// k2 = c1 |b1| - c2 b2 = -(e1 |b1|) + e2 b2 in (-2^127, 2^127): both are exact
// in 128-bit wrap-around arithmetic.  Constants derived by
// tools/glv_constants.py (checked there against the oracle's group law).
// ---------------------------------------------------------------------------
struct GlvBn254 {
  GM_HD static constexpr uint64_t g1(int i) {
    constexpr uint64_t a[5] = {0x163b4843cb4b9a5eull, 0x149d540fd5e495ccull, 0x5398fd0300ff6565ull,
                               0x4ccef014a773d2d2ull, 0x0000000000000002ull};
    return a[i];
  }
  GM_HD static constexpr uint64_t g2(int i) {
    constexpr uint64_t a[4] = {0x8fa7d32d2fafba64ull, 0x6eb9c714773a6ef2ull, 0xd91d232ec7e0b3d7ull,
                               0x0000000000000002ull};
    return a[i];
  }
  static constexpr uint64_t A1_LO = 0x8211bbeb7d4f1128ull, A1_HI = 0x6f4d8248eeb859fcull;
  static constexpr uint64_t A2 = 0x89d3256894d213e3ull;  // = |b1|
  static constexpr uint64_t B2_LO = 0x0be4e1541221250bull, B2_HI = 0x6f4d8248eeb859fdull;
  // beta in the internal radix-2^29 Montgomery form (beta * 2^261 mod p)
  GM_HD static constexpr uint32_t beta29(int i) {
    constexpr uint32_t a[9] = {0x18ccb791u, 0x175b1c3au, 0x0b83d6e2u, 0x0e8ed071u, 0x1282bee2u,
                               0x04220e84u, 0x1fe4017fu, 0x15084d4au, 0x00169119u};
    return a[i];
  }
  // G2 (the twist y^2 = x^3 + b' over Fp2): (x, y) -> (beta^2 x, y) is [lambda] on
  // the r-torsion (the other cube root of unity of Fp; tools/glv_constants.py)
  GM_HD static constexpr uint32_t beta29_g2(int i) {
    constexpr uint32_t a[9] = {0x0a337995u, 0x158d1d23u, 0x189c9b98u, 0x12fa4e45u, 0x185faadcu,
                               0x0176f16du, 0x0eed93bau, 0x14291140u, 0x000c0afeu};
    return a[i];
  }
};

// ---------------------------------------------------------------------------
// GLV split for BLS12-377: lambda = x^2 - 1 (x = 0x8508c00000000001, the curve
// seed) is a cube root of unity mod r with lambda^2 < r < (lambda + 1)^2, so
// k = k1 + k2 lambda with k2 = floor(k / lambda), k1 = k mod lambda -- both in
// [0, 2^127), no signs.  q = floor(k g / 2^384), g = floor(2^384 / lambda),
// undershoots k / lambda by less than one: one conditional correction.
// phi(x, y) = (beta x, y) on G1, (beta^2 x, y) on the G2 twist (tools/glv_constants.py
// checks both against the oracle's group law).
// ---------------------------------------------------------------------------
struct GlvBls377 {
  GM_HD static constexpr uint64_t g(int i) {
    constexpr uint64_t a[5] = {0x5cc5a03b7b820d29ull, 0x3366fc876f25c6b5ull, 0x7f72ed32af90182cull,
                               0xb3f7aa969fd37160ull, 0x0000000000000003ull};
    return a[i];
  }
  static constexpr uint64_t LAM_LO = 0x0a11800000000000ull, LAM_HI = 0x452217cc90000001ull;
  GM_HD static constexpr uint32_t beta29(int i) {
    constexpr uint32_t a[14] = {0x1c8a7893u, 0x0b7d08f2u, 0x06b88506u, 0x162aa2edu, 0x1c5fdf80u,
                                0x11b95a22u, 0x03b86dd7u, 0x1191f770u, 0x10701220u, 0x1501c11fu,
                                0x1cee88bbu, 0x118d05ecu, 0x06f2fa26u, 0x00000000u};
    return a[i];
  }
  GM_HD static constexpr uint32_t beta29_g2(int i) {
    constexpr uint32_t a[14] = {0x098a903fu, 0x0deef70eu, 0x0bd62e43u, 0x12fc3bfau, 0x0de940feu,
                                0x047b8e82u, 0x17ec1b27u, 0x1a776815u, 0x120a67b5u, 0x0a70d0c4u,
                                0x0271dc9au, 0x182f7308u, 0x19602487u, 0x00000000u};
    return a[i];
  }
};

// beta of phi per base field: g1 for G1 points, g2 (= beta^2) for the G2 twist
template <class P>
struct GlvBeta;
template <>
struct GlvBeta<Bn254Fp> {
  GM_HD static constexpr uint32_t g1(int i) { return GlvBn254::beta29(i); }
  GM_HD static constexpr uint32_t g2(int i) { return GlvBn254::beta29_g2(i); }
};
template <>
struct GlvBeta<Bls377Fp> {
  GM_HD static constexpr uint32_t g1(int i) { return GlvBls377::beta29(i); }
  GM_HD static constexpr uint32_t g2(int i) { return GlvBls377::beta29_g2(i); }
};

// x -> beta x of the GLV endomorphism, G1 (Fp) and G2 (Fp2, beta in Fp)
template <class P>
GM_DEV Fe<P> glv_phi_x(const Fe<P>& x) {
  Fe<P> b;
#pragma unroll
  for (int j = 0; j < P::N; j++) b.v[j] = GlvBeta<P>::g1(j);
  return fe_mul(x, b);
}
template <class P, int B>
GM_DEV Fe2<P, B> glv_phi_x(const Fe2<P, B>& x) {
  Fe<P> b;
#pragma unroll
  for (int j = 0; j < P::N; j++) b.v[j] = GlvBeta<P>::g2(j);
  return {fe_mul(x.a0, b), fe_mul(x.a1, b)};
}

// floor(k * G / 2^384) for a 256-bit k and a G of NG 64-bit limbs (< 2^128 here)
template <int NG, class GF>
GM_DEV unsigned __int128 glv_mulshift(const uint64_t (&k)[4], GF g) {
  uint64_t t[4 + NG] = {};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NG; j++) {
      const unsigned __int128 v = (unsigned __int128)k[i] * g(j) + t[i + j] + carry;
      t[i + j] = (uint64_t)v;
      carry = (uint64_t)(v >> 64);
    }
    t[i + NG] = carry;
  }
  return ((unsigned __int128)t[7] << 64) | t[6];
}

// one scalar's signed digits, written at dig[w * g.n + i]; flip: negate them
template <class Fr>
GM_DEV void emit_digits(const FeG<Fr>& k, uint32_t flip, uint32_t i, const DigitGeom& g, uint32_t* __restrict__ dig,
                        uint32_t* lds) {
  const uint32_t mask = (1u << g.c) - 1;
  uint32_t carry = 0;
  for (uint32_t w = 0; w < g.W; w++) {
    const uint32_t raw = window_bits(k, w * g.c, mask) + carry;
    uint32_t d, neg;
    if (raw > g.nb) {
      d = (1u << g.c) - raw;
      carry = 1;
      neg = 1;
    } else {
      d = raw;
      carry = 0;
      neg = 0;
    }
    dig[(size_t)w * g.n + i] = d ? (d - 1) | ((neg ^ flip) << 31) : 0xffffffffu;
    if (d) atomicAdd(&lds[(w * g.nb + d - 1) >> g.F], 1u);
  }
}

// Scalar split k = k1 + k2 lambda per curve: k1 in [0, 2^127), |k2| < 2^127,
// neg2 = sign of k2 (BLS12-377: always 0).
template <class C>
struct Glv {
  static constexpr bool ok = false;
};
template <>
struct Glv<CurveBN254> {
  static constexpr bool ok = true;
  using U = unsigned __int128;
  GM_DEV static void split(const uint64_t (&k64)[4], U& k1, U& k2, uint32_t& neg2) {
    const U c1 = glv_mulshift<5>(k64, GlvBn254::g1);
    const U c2 = glv_mulshift<4>(k64, GlvBn254::g2);
    const U a1 = ((U)GlvBn254::A1_HI << 64) | GlvBn254::A1_LO;
    const U b2 = ((U)GlvBn254::B2_HI << 64) | GlvBn254::B2_LO;
    const U klo = ((U)k64[1] << 64) | k64[0];
    k1 = klo - c1 * a1 - c2 * (U)GlvBn254::A2;  // in [0, 2^127)
    k2 = c1 * (U)GlvBn254::A2 - c2 * b2;        // signed, |k2| < 2^127
    neg2 = (uint32_t)(k2 >> 127);
    if (neg2) k2 = (U)0 - k2;
  }
};
template <>
struct Glv<CurveBLS12377> {
  static constexpr bool ok = true;
  using U = unsigned __int128;
  GM_DEV static void split(const uint64_t (&k64)[4], U& k1, U& k2, uint32_t& neg2) {
    U q = glv_mulshift<5>(k64, GlvBls377::g);  // floor(k / lambda) or one less
    const U lam = ((U)GlvBls377::LAM_HI << 64) | GlvBls377::LAM_LO;
    const U klo = ((U)k64[1] << 64) | k64[0];
    U r = klo - q * lam;  // true value in [0, 2 lambda): exact mod 2^128
    if (r >= lam) {
      r -= lam;
      q += 1;
    }
    k1 = r;
    k2 = q;
    neg2 = 0;
  }
};

// k_msm_digits for the GLV split (plain layout): thread i writes the digits of
// k1 at virtual point i and of k2 at virtual point n0 + i (g.n = 2 n0).
template <class C>
__global__ void __launch_bounds__(1024) k_msm_digits_glv(const uint32_t* __restrict__ scalars, DigitGeom g,
                                                         uint32_t n0, uint32_t NC, uint32_t* __restrict__ dig,
                                                         uint32_t* __restrict__ ccount) {
  using Fr = typename C::Fr;
  extern __shared__ uint32_t dg_lds[];
  const uint32_t t = threadIdx.x;
  for (uint32_t q = t; q < NC; q += DG_THREADS) dg_lds[q] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * DG_THREADS * DG_PPT;
  for (uint32_t r = 0; r < DG_PPT; r++) {
    const uint32_t i = base + r * DG_THREADS + t;
    if (i >= n0) break;
    const FeG<Fr> k = load_scalar_canonical<Fr>(scalars, i);
    uint64_t k64[4];
#pragma unroll
    for (int j = 0; j < 4; j++) k64[j] = (uint64_t)k.w[2 * j] | ((uint64_t)k.w[2 * j + 1] << 32);
    unsigned __int128 k1, k2;
    uint32_t neg2;
    Glv<C>::split(k64, k1, k2, neg2);
    FeG<Fr> m1, m2;
#pragma unroll
    for (int j = 0; j < Fr::NG; j++) {
      m1.w[j] = j < 4 ? (uint32_t)(k1 >> (32 * j)) : 0u;
      m2.w[j] = j < 4 ? (uint32_t)(k2 >> (32 * j)) : 0u;
    }
    emit_digits<Fr>(m1, 0u, i, g, dig, dg_lds);
    emit_digits<Fr>(m2, neg2, n0 + i, g, dig, dg_lds);
  }
  __syncthreads();
  for (uint32_t q = t; q < NC; q += DG_THREADS)
    if (dg_lds[q]) atomicAdd(&ccount[q], dg_lds[q]);
}

// gnark-layout points -> internal layout (GLV: plus phi(P_i) = (beta x, y) at
// n + i; G2: beta^2 on the twist), with coalesced HBM traffic: a block stages its 256 points
// through LDS (16-B lane loads / stores over contiguous bytes) and converts
// from there, instead of each lane reading and writing 64 B at a 64-B lane
// stride.  GLV: the phi copy goes out through the same LDS tile.  LDS rows are
// padded by 16 B (point stride Q + 1 uint4) against bank conflicts.
template <class F, bool GLV>
__global__ void __launch_bounds__(256) k_msm_convert_points_lds(const uint32_t* __restrict__ src, size_t n,
                                                                uint32_t* __restrict__ dst) {
  constexpr int PW = 2 * Coord<F>::WORDS;
  constexpr uint32_t Q = PW / 4;  // uint4 per point
  static_assert(PW % 4 == 0, "points are whole uint4s");
  __shared__ uint4 tile[256 * (Q + 1)];
  const size_t b0 = (size_t)blockIdx.x * 256;
  const uint32_t np = (uint32_t)min((size_t)256, n - b0);
  const uint32_t t = threadIdx.x;
  const uint4* s = reinterpret_cast<const uint4*>(src) + b0 * Q;
  for (uint32_t q = t; q < np * Q; q += 256) tile[(q / Q) * (Q + 1) + q % Q] = s[q];
  __syncthreads();
  uint32_t* mine = reinterpret_cast<uint32_t*>(tile + t * (Q + 1));
  Affine<F> a;
  if (t < np) {
    a = load_affine_gnark<F>(mine);
    store_affine_packed<F>(mine, a);
  }
  __syncthreads();
  uint4* d = reinterpret_cast<uint4*>(dst) + b0 * Q;
  for (uint32_t q = t; q < np * Q; q += 256) d[q] = tile[(q / Q) * (Q + 1) + q % Q];
  if constexpr (GLV) {
    __syncthreads();
    if (t < np) {
      a.x = glv_phi_x(a.x);
      store_affine_packed<F>(mine, a);
    }
    __syncthreads();
    uint4* d2 = reinterpret_cast<uint4*>(dst) + (n + b0) * Q;
    for (uint32_t q = t; q < np * Q; q += 256) d2[q] = tile[(q / Q) * (Q + 1) + q % Q];
  }
}

// ---------------------------------------------------------------------------
// points: gnark layout -> internal layout (once per MSM, into workspace)
// ---------------------------------------------------------------------------
template <class F>
__global__ void __launch_bounds__(256) k_msm_convert_points(const uint32_t* __restrict__ src, size_t n,
                                                            uint32_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int PW = 2 * Coord<F>::WORDS;
  store_affine_packed<F>(dst + i * PW, load_affine_gnark<F>(src + i * PW));
}

// Fixed-base copies: pts[w*stride + i] = [2^off(w)] pts[i] for w = 1..W-1
// (copy 0 already converted; off(w) = window_geom's offset, windows >= wn one
// bit narrower).  width(w-1) doublings per copy in XYZZ, then one Fermat
// inversion back to affine; one-time setup cost, like the pk upload itself.
template <class F>
__global__ void __launch_bounds__(128) k_msm_precompute(uint32_t* __restrict__ pts, size_t n, size_t stride,
                                                        uint32_t c, uint32_t W, uint32_t wn) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int PW = 2 * Coord<F>::WORDS;
  const Affine<F> P = load_affine_packed<F>(pts + i * PW);
  Affine<F> zero;
  zero.x = FOps<F>::zero();
  zero.y = FOps<F>::zero();
  if (aff_is_inf(P)) {
    for (uint32_t w = 1; w < W; w++) store_affine_packed<F>(pts + (w * stride + i) * PW, zero);
    return;
  }
  XYZZ<F> acc;
  acc.x = P.x;
  acc.y = P.y;
  acc.zz = FOps<F>::one();
  acc.zzz = FOps<F>::one();
  for (uint32_t w = 1; w < W; w++) {
    const uint32_t cw = (w - 1 >= wn) ? c - 1 : c;
    for (uint32_t k = 0; k < cw; k++) acc = xyzz_dbl(acc);
    Affine<F> r = zero;
    if (!xyzz_is_inf(acc)) {
      const F t = fe_inv(fe_mul(acc.zz, acc.zzz));
      r.x = fe_mul(acc.x, fe_mul(t, acc.zzz));  // X / ZZ
      r.y = fe_mul(acc.y, fe_mul(t, acc.zz));   // Y / ZZZ
    }
    store_affine_packed<F>(pts + (w * stride + i) * PW, r);
  }
}

// raw words of one packed point (vector loads; unpacked just before use)
template <int PW>
struct PackedPt {
  uint32_t w[PW];
};
template <int PW>
GM_DEV PackedPt<PW> load_packed_pt(const uint32_t* __restrict__ src) {
  static_assert(PW % 4 == 0, "packed points are whole 16-byte chunks");
  PackedPt<PW> r;
#pragma unroll
  for (int q = 0; q < PW / 4; q++) {
    const uint4 v = reinterpret_cast<const uint4*>(src)[q];
    r.w[4 * q] = v.x;
    r.w[4 * q + 1] = v.y;
    r.w[4 * q + 2] = v.z;
    r.w[4 * q + 3] = v.w;
  }
  return r;
}

// Load-balanced accumulation over the sorted entry list: thread t owns entries
// [t*K, t*K+K).  A bucket whose whole range lies in the thread's slice is
// written straight to `buckets`; the (at most two) buckets cut by the slice
// edges go to part_first[t] / part_last[t] and are merged by k_msm_fixup.
// Skewed scalar distributions (one huge bucket) therefore cost the same as
// uniform ones in this phase.
// Buckets accumulate lazily reduced (xyzz_add_aff_lz), canonical on emit.
template <class F>
struct LazyAcc {
  static constexpr bool on = false;
  template <bool CH = false>
  GM_DEV static void add(XYZZ<F>& a, Affine<F> p, bool neg) {
    if (neg) p.y = fe_neg(p.y);
    xyzz_add_aff(a, p);
  }
  GM_DEV static XYZZ<F> canon(const XYZZ<F>& a) { return a; }
};
template <class P>
struct LazyAcc<Fe<P>> {
  static constexpr bool on = true;
  template <bool CH = false>
  GM_DEV static void add(XYZZ<Fe<P>>& a, const Affine<Fe<P>>& p, bool neg) {
    // CH: strict mad chains (level 2) -- isolated 2^20 accumulation ~1 % faster than
    // per-column chains, bench line +1.7 % (profiles/r05an_strict_chain_ab.txt)
    xyzz_add_aff_lz<P, CH ? 2 : 0>(a, p, neg);
  }
  GM_DEV static XYZZ<Fe<P>> canon(const XYZZ<Fe<P>>& a) { return xyzz_canon_lz(a); }
};
template <class P, int B>
struct LazyAcc<Fe2<P, B>> {
  static constexpr bool on = true;
  template <bool CH = false>
  GM_DEV static void add(XYZZ<Fe2<P, B>>& a, Affine<Fe2<P, B>> p, bool neg) {
    if (neg) p.y = fe_neg(p.y);
    xyzz_add_aff_lz(a, p);
  }
  GM_DEV static XYZZ<Fe2<P, B>> canon(const XYZZ<Fe2<P, B>>& a) { return xyzz_canon_lz(a); }
};

template <class F>
GM_DEV void accum_emit(uint32_t b, const XYZZ<F>& acc_raw, bool is_first, bool is_last, uint32_t start,
                       uint32_t end, uint32_t t, const uint32_t* __restrict__ offsets,
                       XYZZ<F>* __restrict__ buckets, XYZZ<F>* __restrict__ part_first,
                       XYZZ<F>* __restrict__ part_last) {
  const XYZZ<F> acc = LazyAcc<F>::canon(acc_raw);
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (bs >= start && be <= end) {
    buckets[b] = acc;
  } else {
    if (is_first) part_first[t] = acc;
    if (is_last) part_last[t] = acc;
  }
}

// Profiled launches (ProfScope::wave_stamp): lane 0 of a wave stamps the wall
// clock on entry (atomicMin) and after the body, where the wave's lanes have
// reconverged (atomicMax): first wave start .. last wave end of the launch.  Blocks
// are dispatched in index order, so the entry stamps of the first 64 blocks hold the
// first wave; every wave stamps its end.  The pair is the block's (index mod 64,
// 256 B apart): one shared pair took every wave's atomics on one L2 channel, and
// the entry stamps of all waves arrive as one burst (bench -2 %, r06ae).
GM_DEV void wave_stamp_begin(unsigned long long* stamp) {
  if (stamp && blockIdx.x < 64 && (threadIdx.x & 63) == 0)
    atomicMin(stamp + blockIdx.x * 32, (unsigned long long)wall_clock64());
}
GM_DEV void wave_stamp_end(unsigned long long* stamp) {
  if (stamp && (threadIdx.x & 63) == 0)
    atomicMax(stamp + (blockIdx.x & 63) * 32 + 1, (unsigned long long)wall_clock64());
}

// G1 accumulation body: keys and values arrive four entries per 16-byte load
// instead of one 4-byte load per entry (r05).  A thread's slice is K
// consecutive entries and consecutive lanes are K entries apart, so each 4-byte
// load touched one cache line per lane and the line rarely survived in L1 until
// the lane's next entry (rocprofv3 FETCH_SIZE of the accumulation: 2.8 GB per
// 2^20 MSM against 1.1 GB of 64-byte point gathers, profiles/r05f_*).  The next
// group's keys / values are loaded at the last entry of the current group.  (Pinning
// the point's four 16-byte loads with an empty asm, against the vectoriser's
// unaligned x2 / x3 / x4 split, costs 32 B of scratch per lane.)  Reads past
// the thread's last entry stay inside the allocation: slices start at multiples
// of K (K % 4 == 0) and the workspace arena rounds every allocation to 256 bytes.
template <class F, bool CH, bool PREFETCH = false>
GM_DEV void accum_seg_body_v4(const uint32_t* __restrict__ points, uint32_t n, const uint32_t* __restrict__ keys,
                              const uint32_t* __restrict__ vals, const uint32_t* __restrict__ offsets,
                              uint32_t total, uint32_t K, XYZZ<F>* __restrict__ buckets,
                              XYZZ<F>* __restrict__ part_first, XYZZ<F>* __restrict__ part_last,
                              uint32_t* __restrict__ err) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t Mv = offsets[total];  // valid (non-zero-digit) entries
  const uint32_t start = t * K;
  if (start >= Mv) return;
  const uint32_t end = min(start + K, Mv);
  uint4 kg = *reinterpret_cast<const uint4*>(keys + start);
  uint4 vg = *reinterpret_cast<const uint4*>(vals + start);
  bool first = true;
  XYZZ<F> acc = xyzz_inf<F>();
  uint32_t cur = kg.x;
  uint32_t v = vg.x;
  if ((v & 0x7fffffffu) >= n) {
    atomicOr(err, 2u);
    return;
  }
  constexpr int PW = 2 * Coord<F>::WORDS;  // u32 words per packed point
  PackedPt<PW> P;
  if (PREFETCH) P = load_packed_pt<PW>(points + (size_t)(v & 0x7fffffffu) * PW);
  for (uint32_t q = start; q < end; q++) {
    const uint32_t k = kg.x;
    // next entry: shift the group; at a group boundary load the next group (its
    // latency overlaps this entry's add)
    if (((q - start) & 3) == 3) {
      if (q + 1 < end) {
        kg = *reinterpret_cast<const uint4*>(keys + q + 1);
        vg = *reinterpret_cast<const uint4*>(vals + q + 1);
      }
    } else {
      kg = make_uint4(kg.y, kg.z, kg.w, kg.w);
      vg = make_uint4(vg.y, vg.z, vg.w, vg.w);
    }
    const uint32_t vn = vg.x;  // entry q + 1 (when q + 1 < end)
    PackedPt<PW> Pn;
    if (q + 1 < end) {
      if ((vn & 0x7fffffffu) >= n) {
        atomicOr(err, 2u);
        return;
      }
      if (PREFETCH) Pn = load_packed_pt<PW>(points + (size_t)(vn & 0x7fffffffu) * PW);
    }
    if (!PREFETCH) P = load_packed_pt<PW>(points + (size_t)(v & 0x7fffffffu) * PW);
    if (k != cur) {
      accum_emit(cur, acc, first, false, start, end, t, offsets, buckets, part_first, part_last);
      first = false;
      acc = xyzz_inf<F>();
      cur = k;
    }
    const Affine<F> A = load_affine_packed<F>(P.w);
    LazyAcc<F>::template add<CH>(acc, A, (v >> 31) != 0);
    v = vn;
    if (PREFETCH) P = Pn;
  }
  accum_emit(cur, acc, first, true, start, end, t, offsets, buckets, part_first, part_last);
}

// BN254 G1: one strict mad chain per product inside the add (r05; the split-
// column schedule measured slower, profiles/r05e_acc_chain_ab.txt,
// r05an_strict_chain_ab.txt), four waves per SIMD, no prefetch: the other waves
// hide the point loads (profiles/r03e_ab.txt).  Applied to every MSM kernel the
// chains slowed the one-to-two-wave reduction kernels (r04h, r05ax).
template <class F>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4)))
k_msm_accum_seg_ch(const uint32_t* __restrict__ points, uint32_t n, const uint32_t* __restrict__ keys,
                   const uint32_t* __restrict__ vals, const uint32_t* __restrict__ offsets, uint32_t total,
                   uint32_t K, XYZZ<F>* __restrict__ buckets, XYZZ<F>* __restrict__ part_first,
                   XYZZ<F>* __restrict__ part_last, uint32_t* __restrict__ err,
                   unsigned long long* __restrict__ stamp) {
  wave_stamp_begin(stamp);
  accum_seg_body_v4<F, true>(points, n, keys, vals, offsets, total, K, buckets, part_first, part_last, err);
  wave_stamp_end(stamp);
}
// Four waves fit the 9-limb fields only: BLS12-377's 14-limb add spills 216
// VGPRs under the cap and takes the prefetching kernel (two waves, no spill).
template <class F>
struct AccumW4 {
  static constexpr bool ok = false;
};
template <class P>
struct AccumW4<Fe<P>> {
  static constexpr bool ok = P::N <= 9;
};
// The next point prefetched into registers while the current add runs
// (BLS12-377 G1: two waves per SIMD).
template <class F>
__global__ void __launch_bounds__(128) k_msm_accum_seg_pf4(const uint32_t* __restrict__ points, uint32_t n,
                                                           const uint32_t* __restrict__ keys,
                                                           const uint32_t* __restrict__ vals,
                                                           const uint32_t* __restrict__ offsets, uint32_t total,
                                                           uint32_t K, XYZZ<F>* __restrict__ buckets,
                                                           XYZZ<F>* __restrict__ part_first,
                                                           XYZZ<F>* __restrict__ part_last,
                                                           uint32_t* __restrict__ err,
                                                           unsigned long long* __restrict__ stamp) {
  wave_stamp_begin(stamp);
  accum_seg_body_v4<F, false, true>(points, n, keys, vals, offsets, total, K, buckets, part_first, part_last, err);
  wave_stamp_end(stamp);
}
// G1 accumulation kernel of a field
template <class F>
constexpr auto g1_accum_kernel() {
  if constexpr (AccumW4<F>::ok) return k_msm_accum_seg_ch<F>;
  else return k_msm_accum_seg_pf4<F>;
}

// G2: Fp2 components split across lane pairs (pair_fp2.hpp), keys / values in
// groups of four as in the G1 accumulation.
template <class F>
struct PairSel {
  static constexpr bool ok = false;
};
template <class P, int B>
struct PairSel<Fe2<P, B>> {
  static constexpr bool ok = true;
  // BN254: one mad chain per product in the pair add, no prefetch, three waves
  // per SIMD (168 VGPRs, no spill; the prefetching kernel needs 200 and runs
  // two): G2 2^20 accumulation 3.91-3.92 -> 3.86-3.89 ms, Groth16 2^24
  // 148.0-149.3 -> 146.8-147.8 ms (profiles/r05aj_pair_chain_ab.txt).
  // BLS12-377: no prefetch (its pair kernel spills at three waves with the
  // prefetch registers: 2^22 accumulation 46.1 -> 44.2 ms, profiles/r03i_ab.txt),
  // two waves (r04e_g2_ab.txt).
  static constexpr auto kernel() {
    if constexpr (P::N <= 9) return k_msm_accum_seg_pair<P, B, false, 3, true, true>;
    else return k_msm_accum_seg_pair<P, B, false, GM_PAIR_WPE, true>;
  }
  static constexpr auto fixup() { return k_msm_fixup_pair<P, B>; }
  static constexpr auto fixup_edge() { return k_msm_fixup_edge_pair<P, B>; }
  static constexpr auto fix_tree() { return k_msm_fix_tree_pair<P, B>; }
  static constexpr auto fixup_long() { return k_msm_fixup_long_pair<P, B>; }
  static constexpr auto seg() { return k_msm_seg_pair<P, B>; }
  static constexpr auto bitsum() { return k_msm_bitsum_pair<P, B>; }
};
// one-lane kernels are instantiated for G1 fields; G2 runs on lane pairs
template <class F>
constexpr bool kOneLane = !PairSel<F>::ok;

// Full adds of the fixup / reduction kernels: lazily reduced for G1
// (xyzz_add_lz, canonical on store), canonical xyzz_add otherwise.
template <class F>
struct FullAdd {
  GM_DEV static XYZZ<F> add(const XYZZ<F>& a, const XYZZ<F>& b) { return xyzz_add(a, b); }
  GM_DEV static XYZZ<F> canon(const XYZZ<F>& a) { return a; }
};
template <class P>
struct FullAdd<Fe<P>> {
  GM_DEV static XYZZ<Fe<P>> add(const XYZZ<Fe<P>>& a, const XYZZ<Fe<P>>& b) { return xyzz_add_lz(a, b); }
  GM_DEV static XYZZ<Fe<P>> canon(const XYZZ<Fe<P>>& a) { return xyzz_canon2(a); }
};

// Merge the partial sums of buckets cut by slice edges.  Bucket b spans slices
// t0..t1 and its sum is part_last[t0] + part_first[t0+1] + ... + part_first[t1].
// Spans up to FIX_SERIAL slices are summed by one thread; longer spans (a huge
// bucket: skewed witness values, or the nearly empty top window of a scalar
// field much narrower than W*c bits) are tree-reduced in place over part_first
// by k_msm_fix_tree levels -- depth log2(span) adds instead of span serial adds.
constexpr uint32_t FIX_SERIAL = 8;

template <class F>
__global__ void __launch_bounds__(128) k_msm_fixup(const uint32_t* __restrict__ offsets, uint32_t total,
                                                   uint32_t K, XYZZ<F>* __restrict__ buckets,
                                                   const XYZZ<F>* __restrict__ part_first,
                                                   const XYZZ<F>* __restrict__ part_last,
                                                   uint32_t* __restrict__ maxspan) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= total) return;
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t0 == t1) return;
  if (t1 - t0 > FIX_SERIAL) {
    atomicMax(maxspan, t1 - t0);
    return;
  }
  XYZZ<F> acc = part_last[t0];
  for (uint32_t t = t0 + 1; t <= t1; t++) acc = FullAdd<F>::add(acc, part_first[t]);
  buckets[b] = FullAdd<F>::canon(acc);
}

// The same merge, one thread per slice edge t >= 1: the bucket holding entry t K
// is cut by the edge when it starts before it, and the thread of its first edge
// (t = t0 + 1) merges its parts -- the same adds in the same order.  Used when
// buckets are shorter than a slice (M < K * buckets: the plain-key Groth16 2^24
// MSMs, ~32 entries per bucket at K = 64): per bucket, a wave then mixes cut and
// whole buckets and half its lanes idle through the add, while nearly every
// edge cuts a bucket once.  Buckets longer than a slice are cut by one to three
// edges each, so per edge the lanes idle instead: 2^24 plain 148.2 -> 147.3 ms,
// precomputed (~96 entries per bucket) 137.5 -> 140.8 ms, 2^20 G1 (64 per bucket
// at K = 32) fixup 0.11 -> 0.175 ms (profiles/r06g_fixup_edge_ab.txt).
template <class F>
__global__ void __launch_bounds__(128) k_msm_fixup_edge(const uint32_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ offsets, uint32_t total,
                                                        uint32_t K, uint32_t nslices,
                                                        XYZZ<F>* __restrict__ buckets,
                                                        const XYZZ<F>* __restrict__ part_first,
                                                        const XYZZ<F>* __restrict__ part_last,
                                                        uint32_t* __restrict__ maxspan) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (t >= nslices) return;
  const size_t q = (size_t)t * K;  // first entry of slice t
  if (q >= offsets[total]) return;
  const uint32_t b = keys[q];
  const uint32_t bs = offsets[b];
  if (bs >= q || bs / K != t - 1) return;  // not cut by this edge, or not its first edge
  const uint32_t t0 = t - 1, t1 = (offsets[b + 1] - 1) / K;
  if (t1 - t0 > FIX_SERIAL) {
    atomicMax(maxspan, t1 - t0);
    return;
  }
  XYZZ<F> acc = part_last[t0];
  for (uint32_t u = t; u <= t1; u++) acc = FullAdd<F>::add(acc, part_first[u]);
  buckets[b] = FullAdd<F>::canon(acc);
}
// One level d of the pairwise tree over part_first[t0+1 .. t1] of every long span.
template <class F>
__global__ void __launch_bounds__(128) k_msm_fix_tree(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ offsets, uint32_t total,
                                                      uint32_t K, uint32_t nslices, uint32_t d,
                                                      XYZZ<F>* __restrict__ part_first) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nslices || (size_t)t * K >= offsets[total]) return;
  const uint32_t b = keys[(size_t)t * K];
  const uint32_t t0 = offsets[b] / K, t1 = (offsets[b + 1] - 1) / K;
  if (t1 - t0 <= FIX_SERIAL || t <= t0) return;
  const uint32_t rel = t - (t0 + 1), len = t1 - t0, step = 1u << d;
  if ((rel & ((step << 1) - 1)) == 0 && rel + step < len)
    part_first[t] = FullAdd<F>::canon(FullAdd<F>::add(part_first[t], part_first[t + step]));
}

template <class F>
__global__ void __launch_bounds__(128) k_msm_fixup_long(const uint32_t* __restrict__ offsets, uint32_t total,
                                                        uint32_t K, XYZZ<F>* __restrict__ buckets,
                                                        const XYZZ<F>* __restrict__ part_first,
                                                        const XYZZ<F>* __restrict__ part_last) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= total) return;
  const uint32_t bs = offsets[b], be = offsets[b + 1];
  if (be == bs) return;
  const uint32_t t0 = bs / K, t1 = (be - 1) / K;
  if (t1 - t0 <= FIX_SERIAL) return;
  buckets[b] = FullAdd<F>::canon(FullAdd<F>::add(part_last[t0], part_first[t0 + 1]));
}

// ---------------------------------------------------------------------------
// Bucket reduction: window sum P_w = sum_j (j+1) B_j over the nb buckets of a
// window.  A single EC add costs ~15-20 us of latency in one wave, so the
// reduction is organised to keep every serial chain short and all 1024 SIMDs
// busy, and to leave the inherently serial Horner tail (~W*c doublings) to the
// host, where one group op is ~50x cheaper in latency:
//
//   level 1 (k_msm_seg): segments of L buckets, running sums
//        S_s = sum_l B_{sL+l},  T_s = sum_l (l+1) B_{sL+l}
//     so P_w = sum_s T_s + L * sum_s s*S_s.
//   levels 2.. (k_msm_bitsum): LDS trees over the segments that never multiply
//     by the index: a node carries [G, U, Y_0..Y_{K-1}] with G = sum S, U = sum T
//     and Y_b = sum of S over the node's segments whose local index has bit b
//     set.  Merging two sibling nodes of 2^d segments is (K+3) independent adds
//     (Y_d of the parent is G of the right child), one per thread, so a tree
//     over NT segments has depth log2(NT) adds and ~3 adds of work per segment.
//   host: P_w = U + sum_b 2^(b + log2 L) Y_b, merged into the window Horner.
// ---------------------------------------------------------------------------
// node layout: per window, m nodes of Q = 2 + K XYZZ points [G, U, Y_0..Y_{K-1}]
// At most 512 tree tasks (adds) per level: two per thread.  (A 512-thread
// block with one task per thread measured no faster at 2^20: the tree's tail
// is short of blocks, not of threads.)
constexpr uint32_t BS_THREADS = 256;
// A bucket with no entries (offsets[b] == offsets[b + 1]) was never written by
// the accumulation or the fixup: it reads as infinity here, so the buckets need no
// clearing before the accumulation (a 1 GB memset per plain 2^24 MSM).
template <class F>
__global__ void __launch_bounds__(128) k_msm_seg(const XYZZ<F>* __restrict__ buckets,
                                                 const uint32_t* __restrict__ offsets, uint32_t nb, uint32_t L,
                                                 uint32_t nseg, uint32_t W, XYZZ<F>* __restrict__ nodes) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= W * nseg) return;
  const uint32_t w = t / nseg, s = t % nseg;
  const size_t b0 = (size_t)w * nb + (size_t)s * L;
  const XYZZ<F>* B = buckets + b0;
  const uint32_t* O = offsets + b0;
  uint32_t o_hi = O[L];
  uint32_t o_lo = O[L - 1];
  XYZZ<F> S = o_lo == o_hi ? xyzz_inf<F>() : B[L - 1], T = S;
  for (int j = (int)L - 2; j >= 0; j--) {
    o_hi = o_lo;
    o_lo = O[j];
    S = FullAdd<F>::add(S, o_lo == o_hi ? xyzz_inf<F>() : B[j]);
    T = FullAdd<F>::add(T, S);
  }
  nodes[2 * (size_t)t] = FullAdd<F>::canon(S);
  nodes[2 * (size_t)t + 1] = FullAdd<F>::canon(T);
}

// One tree level group: block (w, j) merges nodes [j*NT, (j+1)*NT) of window w
// (Qin points each) into one node of Qin + log2(NT) points.
template <class F>
__global__ void __launch_bounds__(BS_THREADS) k_msm_bitsum(const XYZZ<F>* __restrict__ in, uint32_t m,
                                                    uint32_t Qin, uint32_t NT, uint32_t lgNT,
                                                    XYZZ<F>* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  XYZZ<F>* X = reinterpret_cast<XYZZ<F>*>(smem_raw);
  const uint32_t groups = m / NT;
  const uint32_t w = blockIdx.x / groups, j = blockIdx.x % groups;
  const XYZZ<F>* src = in + ((size_t)w * m + (size_t)j * NT) * Qin;
  for (uint32_t q = threadIdx.x; q < NT * Qin; q += blockDim.x) X[q] = src[q];
  __syncthreads();
  for (uint32_t d = 0; d < lgNT; d++) {
    const uint32_t qc = Qin + d + 1;           // quantities of a parent node
    const uint32_t tasks = (NT >> (d + 1)) * qc;
    const uint32_t child = (Qin << d);          // slots spanned by one child
    XYZZ<F> r0, r1;
    uint32_t s0 = 0xffffffffu, s1 = 0xffffffffu;
    {
      const uint32_t t = threadIdx.x;
      if (t < tasks) {
        const uint32_t p = t / qc, q = t % qc, base = p * 2 * child;
        r0 = (q + 1 < qc) ? FullAdd<F>::canon(FullAdd<F>::add(X[base + q], X[base + child + q])) : X[base + child];
        s0 = base + q;
      }
    }
    {
      const uint32_t t = threadIdx.x + blockDim.x;
      if (t < tasks) {
        const uint32_t p = t / qc, q = t % qc, base = p * 2 * child;
        r1 = (q + 1 < qc) ? FullAdd<F>::canon(FullAdd<F>::add(X[base + q], X[base + child + q])) : X[base + child];
        s1 = base + q;
      }
    }
    __syncthreads();
    if (s0 != 0xffffffffu) X[s0] = r0;
    if (s1 != 0xffffffffu) X[s1] = r1;
    __syncthreads();
  }
  const uint32_t Qout = Qin + lgNT;
  XYZZ<F>* dst = out + ((size_t)w * groups + j) * Qout;
  for (uint32_t q = threadIdx.x; q < Qout; q += blockDim.x) dst[q] = X[q];
}

// internal XYZZ -> gnark-layout (X, Y, ZZ, ZZZ) words for the host finish
template <class F>
__global__ void __launch_bounds__(128) k_msm_export(const XYZZ<F>* __restrict__ nodes, uint32_t count,
                                                    uint32_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  uint32_t* o = out + (size_t)t * 4 * Coord<F>::WORDS;
  const XYZZ<F> r = nodes[t];
  Coord<F>::store_gnark(o, r.x);
  Coord<F>::store_gnark(o + Coord<F>::WORDS, r.y);
  Coord<F>::store_gnark(o + 2 * Coord<F>::WORDS, r.zz);
  Coord<F>::store_gnark(o + 3 * Coord<F>::WORDS, r.zzz);
}

// ---------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------
// Window size minimising a cost model in EC adds: n*W accumulation adds plus
// ~3 adds per bucket in the reduction (W*2^(c-1) buckets), W = ceil((bits+1)/c).
// Picks c = 16 for 2^20 BN254 points, 20 for 2^24, and c = 17 (W = 15, a full top
// window) instead of 18 for 2^22 BLS12-377 points.
static int choose_window(size_t n, int bits) {
  int best = 8;
  double best_cost = 1e300;
  for (int c = 8; c <= 20; c++) {
    const double W = (double)((bits + 1 + c - 1) / c);
    const double cost = (double)n * W + 3.0 * W * (double)(1u << (c - 1));
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

// Keys, sort and bucket offsets for one scalar vector (see MsmPlan).
template <class C>
int msm_plan(gm_ctx* ctx, Arena& arena, const void* scalars_dev, size_t n, const MsmPrecomp* pre,
             MsmPlan& plan, bool glv) {
  hipStream_t st = ctx->stream;
  plan = MsmPlan();
  plan.n = n;
  plan.bits = C::FR_BITS;
  if (n == 0) return GM_OK;
  if (glv && (!Glv<C>::ok || (pre && pre->c))) {
    set_error("msm: the GLV split needs a plain (not precomputed) layout");
    return GM_ERR_INVALID;
  }
  const size_t n0 = n;  // scalars
  if (glv) {            // virtual points: P_i and phi(P_i)
    n = 2 * n0;
    plan.n = n;
    plan.bits = 127;
  }
  if (n >= (size_t(1) << 31)) {
    set_error("msm: n must be < 2^31");
    return GM_ERR_INVALID;
  }
  const bool shared = pre && pre->c;
  if (shared && (pre->stride < n || (size_t)pre->W * pre->stride >= (size_t(1) << 31) || pre->narrow >= pre->W ||
                 (size_t)pre->c * pre->W - pre->narrow < (size_t)C::FR_BITS + 1)) {
    set_error("msm: precomputed point set does not cover this MSM");
    return GM_ERR_INVALID;
  }
  const uint32_t c = shared ? pre->c
                            : (ctx->msm_c_override ? (uint32_t)ctx->msm_c_override
                                                   : (uint32_t)choose_window(n, plan.bits));
  // ceil((bits+1)/c): the top signed digit never carries
  const uint32_t W = shared ? pre->W : (uint32_t)(plan.bits + 1 + c - 1) / c;
  plan.c = c;
  plan.W = W;
  plan.nb = 1u << (c - 1);
  plan.Wred = shared ? 1 : W;
  plan.total = plan.Wred * plan.nb;
  plan.npts = shared ? (size_t)W * pre->stride : n;
  const size_t M = (size_t)W * n;  // upper bound on the entries: zero digits are dropped
  plan.M = M;
  if (M >= (size_t(1) << 31)) {
    set_error("msm: n * windows must be < 2^31");
    return GM_ERR_INVALID;
  }
  // Sort geometry: ~2K entries per coarse bin for uniform digits (the final pass
  // sorts a bin of up to S2_STAGE entries in LDS; the narrow top window's bins
  // are ~2x fuller).  Pass-1 bins (b >> (F + G)) are coarsened by G until one
  // pass-1 block (one window of S1 points in the plain layout) touches at most
  // 512 of them (long write runs) and there are at most 8192; G > 0 adds the
  // middle pass (msm_sort.hip).
  SortGeom sg;
  sg.T = plan.total;
  sg.M = M;
  sg.F = 4;
  // A GLV plan's windows are full width (|k1|, |k2| < 0.87 * 2^127: no narrow top
  // window) with twice the entries per bucket: ~4K-entry bins keep one pass-1
  // block within 512 bins (no middle pass) and still fit S2_STAGE.
  // The shared-bucket (precomputed) layout takes ~1.5K-entry bins: its 2^24 sort 3.78 -> 3.34 ms, 2^20 0.28 ->
  // 0.19 ms against ~0.75K, while ~3K are slower again (profiles/r06v_shared_sort_bins_ab.txt); the plain
  // layout's 2^24 sort is slower with ~2K bins than ~1K (3.29 -> 3.51 ms, r06u_sort_bins_ab.txt) and with ~0.5K
  // (3.35 -> 3.83 ms, r06w_plain_sort_bins_ab.txt).
  const double bin_entries = glv || shared ? 4096.0 : 2048.0;
  while (sg.F < 13 && (double)M * std::ldexp(1.0, (int)sg.F + 1) <= bin_entries * sg.T) sg.F++;
  auto bins = [&](uint32_t sh) { return (uint32_t)(((uint64_t)sg.T + (1ull << sh) - 1) >> sh); };
  auto touched = [&](uint32_t sh) { return shared ? bins(sh) : std::max(1u, plan.nb >> sh); };
  // GM_MSM_SORT_MING: minimum G (tests exercise the middle pass at small sizes)
  const char* ming = getenv("GM_MSM_SORT_MING");
  sg.G = ming ? (uint32_t)std::min(10, std::max(0, atoi(ming))) : 0u;
  // (shared layout at 2^20: 8192 pass-1 bins with G = 0 measured 0.285 ms vs
  // 0.315 with the middle pass -- its 109 MB of entries stay in the caches, which
  // merge the short write runs; at 2^24, 1.6 GB, they do not: 2.4 ms per sort)
  const uint32_t max_touched = (shared && M < (size_t(1) << 24)) ? 8192u : 512u;
  while (sg.G < 10 && (touched(sg.F + sg.G) > max_touched || bins(sg.F + sg.G) > 8192)) sg.G++;
  while (sg.G && sg.F + sg.G > 31) sg.G--;
  sg.NC = bins(sg.F);
  sg.NS = bins(sg.F + sg.G);
  if (sg.NS > 8192) {
    set_error("msm: too many buckets for the sort");
    return GM_ERR_INVALID;
  }
  int rc;
  DevBuf dig, keys_out, vals_out, offsets, scount;
  if ((rc = dig.alloc(arena, sizeof(uint32_t) * M)) || (rc = keys_out.alloc(arena, sizeof(uint32_t) * M)) ||
      (rc = vals_out.alloc(arena, sizeof(uint32_t) * M)) ||
      (rc = offsets.alloc(arena, sizeof(uint32_t) * ((size_t)plan.total + 1))) ||
      (rc = scount.alloc(arena, sizeof(uint32_t) * sg.NS)))
    return rc;
  DigitGeom g;
  g.n = (uint32_t)n;
  g.c = c;
  g.W = W;
  g.nb = plan.nb;
  g.shared_stride = shared ? (uint32_t)pre->stride : 0u;
  g.wn = shared ? W - pre->narrow : W;
  if (!shared && !glv) {
    // plain layout: balance the windows (see DigitGeom)
    const uint32_t narrow = c * W - (uint32_t)(plan.bits + 1);
    if (narrow < W) g.wn = W - narrow;
  }
  plan.wn = g.wn;
  g.F = sg.F + sg.G;  // the digits kernel counts pass-1 bins
  {
    ProfScope ps(ctx, "msm_digits");
    GM_HIP(hipMemsetAsync(scount.p, 0, sizeof(uint32_t) * sg.NS, st));
    if constexpr (Glv<C>::ok) {
      if (glv)
        hipLaunchKernelGGL(k_msm_digits_glv<C>, dim3(blocks_for(n0, DG_THREADS * DG_PPT)), dim3(DG_THREADS),
                         sizeof(uint32_t) * sg.NS, st, reinterpret_cast<const uint32_t*>(scalars_dev), g,
                           (uint32_t)n0, sg.NS, dig.as<uint32_t>(), scount.as<uint32_t>());
    }
    if (!glv)
      hipLaunchKernelGGL(k_msm_digits<typename C::Fr>, dim3(blocks_for(n, DG_THREADS * DG_PPT)), dim3(DG_THREADS),
                         sizeof(uint32_t) * sg.NS, st, reinterpret_cast<const uint32_t*>(scalars_dev), g, sg.NS,
                         dig.as<uint32_t>(), scount.as<uint32_t>());
    GM_HIP(hipGetLastError());
  }
  {
    ProfScope ps(ctx, "msm_sort");
    if ((rc = msm_sort_digits(ctx, arena, sg, n, W, plan.nb, g.shared_stride, dig.as<uint32_t>(),
                              scount.as<uint32_t>(), keys_out.as<uint32_t>(), vals_out.as<uint32_t>(),
                              offsets.as<uint32_t>())))
      return rc;
  }
  plan.keys = keys_out.as<uint32_t>();
  plan.vals = vals_out.as<uint32_t>();
  plan.offsets = offsets.as<uint32_t>();
  return GM_OK;
}

// Bucket reduction of a launched MSM (k_msm_seg, LDS bit-sum levels, export
// into t.wsum); sets t.Q, the points per exported node.
template <class C, bool G2>
int msm_reduce(gm_ctx* ctx, MsmTail& t) {
  using DF = typename GroupSel<C, G2>::DF;
  hipStream_t st = ctx->stream;
  ProfScope ps(ctx, "msm_bucket_reduce");
  uint32_t Q = 2;  // points per node: [G, U, Y_0..Y_{Q-3}]
  constexpr bool pairs = PairSel<DF>::ok;
  if constexpr (PairSel<DF>::ok) {
    if (pairs)
      hipLaunchKernelGGL(PairSel<DF>::seg(), dim3(blocks_for(2 * (size_t)t.Wr * t.nseg, 128)), dim3(128), 0, st,
                         (const uint32_t*)t.buckets, (const uint32_t*)t.offsets, t.nb, t.L, t.nseg, t.Wr,
                         (uint32_t*)t.nodes_a);
  }
  if constexpr (kOneLane<DF>) {
    if (!pairs)
      hipLaunchKernelGGL(k_msm_seg<DF>, dim3(blocks_for((size_t)t.Wr * t.nseg, 128)), dim3(128), 0, st,
                         (const XYZZ<DF>*)t.buckets, (const uint32_t*)t.offsets, t.nb, t.L, t.nseg, t.Wr,
                         (XYZZ<DF>*)t.nodes_a);
  }
  // LDS tree levels until one node per window
  constexpr size_t SLOT_BUDGET = (96u << 10) / sizeof(XYZZ<DF>);
  uint32_t m = t.nseg;
  XYZZ<DF>* cur = (XYZZ<DF>*)t.nodes_a;
  XYZZ<DF>* nxt = (XYZZ<DF>*)t.nodes_b;
  while (m > 1) {
    uint32_t lg = 0;
    // largest power-of-two group with NT*Q slots in budget and <= 2 tasks per thread
    while ((2u << lg) <= m && (size_t)(2u << lg) * Q <= SLOT_BUDGET && (1u << lg) * (Q + 1) <= 2 * BS_THREADS) lg++;
    if (lg == 0) {
      set_error("msm: bucket reduction does not fit LDS");
      return GM_ERR_INVALID;
    }
    const uint32_t NT = 1u << lg;
    const uint32_t groups = m / NT;
    if constexpr (PairSel<DF>::ok) {
      if (pairs)
        hipLaunchKernelGGL(PairSel<DF>::bitsum(), dim3(t.Wr * groups), dim3(BS_PAIR_THREADS), sizeof(XYZZ<DF>) * NT * Q,
                           st, (const uint32_t*)cur, m, Q, NT, lg, (uint32_t*)nxt);
    }
    if constexpr (kOneLane<DF>) {
      if (!pairs)
        hipLaunchKernelGGL(k_msm_bitsum<DF>, dim3(t.Wr * groups), dim3(BS_THREADS), sizeof(XYZZ<DF>) * NT * Q, st,
                           cur, m, Q, NT, lg, nxt);
    }
    Q += lg;
    m = groups;
    std::swap(cur, nxt);
  }
  hipLaunchKernelGGL(k_msm_export<DF>, dim3(blocks_for((size_t)t.Wr * Q, 128)), dim3(128), 0, st, cur, t.Wr * Q,
                     (uint32_t*)t.wsum);
  GM_HIP(hipGetLastError());
  t.Q = Q;
  return GM_OK;
}

// Buckets spanning more than FIX_SERIAL slices: tree fixup over part_first.
template <class C, bool G2>
int msm_fix_long(gm_ctx* ctx, MsmTail& t, uint32_t maxspan) {
  using DF = typename GroupSel<C, G2>::DF;
  hipStream_t st = ctx->stream;
  const size_t nslices = (t.M + t.K - 1) / t.K;
  if constexpr (PairSel<DF>::ok) {
    {
      for (uint32_t d = 0; (1u << d) < maxspan; d++)
        hipLaunchKernelGGL(PairSel<DF>::fix_tree(), dim3(blocks_for(2 * nslices, 128)), dim3(128), 0, st, t.keys,
                           t.offsets, t.total, t.K, (uint32_t)nslices, d, (uint32_t*)t.pfirst, FIX_SERIAL);
      hipLaunchKernelGGL(PairSel<DF>::fixup_long(), dim3(blocks_for(2 * (size_t)t.total, 128)), dim3(128), 0, st,
                         t.offsets, t.total, t.K, (uint32_t*)t.buckets, (const uint32_t*)t.pfirst,
                         (const uint32_t*)t.plast, FIX_SERIAL);
      GM_HIP(hipGetLastError());
      return GM_OK;
    }
  }
  if constexpr (kOneLane<DF>) {
    for (uint32_t d = 0; (1u << d) < maxspan; d++)
      hipLaunchKernelGGL(k_msm_fix_tree<DF>, dim3(blocks_for(nslices, 128)), dim3(128), 0, st, t.keys, t.offsets,
                         t.total, t.K, (uint32_t)nslices, d, (XYZZ<DF>*)t.pfirst);
    hipLaunchKernelGGL(k_msm_fixup_long<DF>, dim3(blocks_for(t.total, 128)), dim3(128), 0, st, t.offsets, t.total,
                       t.K, (XYZZ<DF>*)t.buckets, (const XYZZ<DF>*)t.pfirst, (const XYZZ<DF>*)t.plast);
  }
  GM_HIP(hipGetLastError());
  return GM_OK;
}

// readback of (error, max span) and the exported nodes into t.stage, event after it
template <class C, bool G2>
int msm_readback(gm_ctx* ctx, MsmTail& t) {
  using DF = typename GroupSel<C, G2>::DF;
  constexpr int WORDS = Coord<DF>::WORDS;
  hipStream_t st = ctx->stream;
  const size_t wbytes = sizeof(uint32_t) * 4 * WORDS * t.Wr * t.Q;
  if (!t.stage) {  // a re-readback (after a long-span fixup) reuses the tail's buffer
    if (int r = tail_pinned_acquire(ctx, 16 + wbytes, &t.stage, &t.stage_idx)) return r;
    t.stage_ctx = ctx;
  }
  GM_HIP(hipMemcpyAsync(t.stage, t.errw, 16, hipMemcpyDeviceToHost, st));
  GM_HIP(hipMemcpyAsync(t.stage + 16, t.wsum, wbytes, hipMemcpyDeviceToHost, st));
  if (!t.done) GM_HIP(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
  GM_HIP(hipEventRecord(t.done, st));
  return GM_OK;
}

// Bucket accumulation and (speculative) reduction over a plan, queued on the
// context's stream; msm_finish completes it.
template <class C, bool G2>
int msm_launch(gm_ctx* ctx, Arena& arena, const MsmPlan& plan, const void* points_internal, MsmTail& t) {
  using DF = typename GroupSel<C, G2>::DF;
  using HF = typename GroupSel<C, G2>::HF;
  hipStream_t st = ctx->stream;
  t.n = plan.n;
  if (plan.n == 0) return GM_OK;
  t.c = plan.c;
  t.W = plan.W;
  t.wn = plan.wn;
  t.nb = plan.nb;
  t.total = plan.total;
  t.Wr = plan.Wred;
  t.M = plan.M;
  t.keys = plan.keys;
  t.offsets = plan.offsets;
  // level-1 segment length (buckets).  Measured at 2^20 (BN254 G1 / G2 /
  // BLS12-377 G2 reduction ms): L = 1: 0.83 / 4.2 / 16.9, L = 2: 0.51 / 2.6 / 9.6,
  // L = 4: 0.36 / 1.74 / 6.05 -- the LDS bit-sum trees cost more per add than the
  // running sums.  So L grows (to 32) as long as k_msm_seg keeps >= 128K threads
  // (two waves per SIMD): 4 for 2^20 plain, 16 for the one-window 2^21 buckets
  // of a precomputed 2^24 key (segment lengths 4 / 8 re-measured in the pipelined
  // loop, profiles/r05ai_segl_ab.txt).
  uint32_t Lwant = 4;
  while (Lwant < 32 && (size_t)t.Wr * t.nb / (2 * Lwant) >= (size_t(1) << 17)) Lwant *= 2;
  t.L = t.nb >= Lwant ? Lwant : t.nb;
  t.nseg = t.nb / t.L;
  // Entries per accumulation thread.  64 by default; 24 for G1 MSMs of at most
  // 2^25 entries (the 2^20 GLV bench MSM: 2^24 entries = 4,096 waves at 64, one
  // round of four waves per SIMD, so the slowest waves set the time; at 32 the
  // accumulation alone drops 1.38-1.43 -> 1.34 ms and the pipelined MSM loop gains
  // 4-7 %, profiles/r04ae_slice_sweep.txt; with the ordered accumulations, 24
  // gives shorter block rounds, so the next MSM's sort kernels find wave slots
  // sooner: 641 -> 649 Mpoints/s same box, r06ai_slice_ab.txt).  Larger MSMs keep 64 (Groth16 2^24:
  // 156.9 vs 159.3 ms at 32).  The long-span bound FIX_SERIAL * K stays above the
  // fullest uniform bucket (64 entries at 2^20).  K % 4 == 0: the accumulation
  // loads keys / values four entries at a time.  (K = 128 for the Groth16 2^24
  // MSMs: within noise, profiles/r06d_g16_k128_ab.txt.)
  t.K = !G2 && plan.M <= (size_t(1) << 25) ? 24u : 64u;
  int rc;
  constexpr int WORDS = Coord<DF>::WORDS;  // u32 words of one gnark-layout coordinate
  static_assert(sizeof(HF) == 4 * WORDS, "host/device layout mismatch");
  const size_t nslices = (t.M + t.K - 1) / t.K;
  DevBuf buckets, nodes_a, nodes_b, wsum, errw, pfirst, plast;
  if ((rc = errw.alloc(arena, 16)) || (rc = buckets.alloc(arena, sizeof(XYZZ<DF>) * (size_t)t.total)) ||
      (rc = nodes_a.alloc(arena, sizeof(XYZZ<DF>) * 2 * (size_t)t.Wr * t.nseg)) ||
      (rc = nodes_b.alloc(arena, sizeof(XYZZ<DF>) * 2 * (size_t)t.Wr * t.nseg)) ||
      (rc = wsum.alloc(arena, sizeof(uint32_t) * 4 * WORDS * t.Wr * (2 + t.c))) ||
      (rc = pfirst.alloc(arena, sizeof(XYZZ<DF>) * nslices)) || (rc = plast.alloc(arena, sizeof(XYZZ<DF>) * nslices)))
    return rc;
  t.buckets = buckets.p;
  t.nodes_a = nodes_a.p;
  t.nodes_b = nodes_b.p;
  t.wsum = wsum.p;
  t.errw = errw.p;
  t.pfirst = pfirst.p;
  t.plast = plast.p;
  GM_HIP(hipMemsetAsync(errw.p, 0, 16, st));
  {
    // async MSMs: this accumulation starts after the previous one (gm_ctx::acc_tail)
    if (ctx->acc_chain) {
      if (!ctx->acc_tail) GM_HIP(hipEventCreateWithFlags(&ctx->acc_tail, hipEventDisableTiming));
      else GM_HIP(hipStreamWaitEvent(st, ctx->acc_tail, 0));
    }
    struct TailMark {  // recorded once the accumulation is queued
      gm_ctx* c;
      hipStream_t s;
      ~TailMark() {
        if (c->acc_chain) hipEventRecord(c->acc_tail, s);
      }
    } tail_mark{ctx, st};
    ProfScope ps(ctx, G2 ? "msm_accum_g2" : "msm_accum_g1", true);  // stamped by the launch
    if constexpr (PairSel<DF>::ok) {
      hipExtLaunchKernelGGL(PairSel<DF>::kernel(), dim3(blocks_for(2 * nslices, 128)), dim3(128), 0, st, ps.a, ps.b,
                            0, reinterpret_cast<const uint32_t*>(points_internal), (uint32_t)plan.npts, plan.keys,
                            plan.vals, plan.offsets, t.total, t.K, buckets.as<uint32_t>(), pfirst.as<uint32_t>(),
                            plast.as<uint32_t>(), errw.as<uint32_t>());
    } else {
      hipExtLaunchKernelGGL(g1_accum_kernel<DF>(), dim3(blocks_for(nslices, 128)), dim3(128), 0, st, ps.a, ps.b, 0,
                            reinterpret_cast<const uint32_t*>(points_internal), (uint32_t)plan.npts, plan.keys,
                            plan.vals, plan.offsets, t.total, t.K, buckets.as<XYZZ<DF>>(), pfirst.as<XYZZ<DF>>(),
                            plast.as<XYZZ<DF>>(), errw.as<uint32_t>(), ps.wave_stamp("msm_accum_g1_exec"));
    }
  }
  {
    ProfScope ps(ctx, "msm_fixup");
    if (plan.M < (size_t)t.K * t.total) {  // buckets shorter than a slice: per edge
      if (nslices > 1) {
        if constexpr (PairSel<DF>::ok)
          hipLaunchKernelGGL(PairSel<DF>::fixup_edge(), dim3(blocks_for(2 * (nslices - 1), 128)), dim3(128), 0, st,
                             plan.keys, plan.offsets, t.total, t.K, (uint32_t)nslices, buckets.as<uint32_t>(),
                             pfirst.as<uint32_t>(), plast.as<uint32_t>(), errw.as<uint32_t>() + 1, FIX_SERIAL);
        else
          hipLaunchKernelGGL(k_msm_fixup_edge<DF>, dim3(blocks_for(nslices - 1, 128)), dim3(128), 0, st, plan.keys,
                             plan.offsets, t.total, t.K, (uint32_t)nslices, buckets.as<XYZZ<DF>>(),
                             pfirst.as<XYZZ<DF>>(), plast.as<XYZZ<DF>>(), errw.as<uint32_t>() + 1);
      }
    } else if constexpr (PairSel<DF>::ok) {
      hipLaunchKernelGGL(PairSel<DF>::fixup(), dim3(blocks_for(2 * (size_t)t.total, 128)), dim3(128), 0, st,
                         plan.offsets, t.total, t.K, buckets.as<uint32_t>(), pfirst.as<uint32_t>(),
                         plast.as<uint32_t>(), errw.as<uint32_t>() + 1, FIX_SERIAL);
    } else {
      hipLaunchKernelGGL(k_msm_fixup<DF>, dim3(blocks_for(t.total, 128)), dim3(128), 0, st, plan.offsets, t.total,
                         t.K, buckets.as<XYZZ<DF>>(), pfirst.as<XYZZ<DF>>(), plast.as<XYZZ<DF>>(),
                         errw.as<uint32_t>() + 1);
    }
  }
  // Bucket reduction, launched speculatively: buckets spanning more than
  // FIX_SERIAL slices (skewed scalars) are only known once errw[1] (max span)
  // reaches the host, so the reduction is queued right away and redone after the
  // long-span fixup in that (rare) case.  Speculate only when uniform scalars
  // would give no long span: the fullest bucket is then a top-window digit
  // (n / 2^top_bits entries; plus the other windows' share when buckets are
  // shared).  Large MSMs whose top window is narrow (2^24: 1024-4096 entries per
  // top digit) sync on the max span first.
  {
    // expected entries of the fullest bucket: bucket 0 gets n / h_w from window
    // w, h_w = the largest digit of w (its width, or the bits left above it)
    double fullest = 0;
    for (uint32_t w = 0; w < t.W; w++) {
      uint32_t off, cw;
      window_geom(t.c, plan.wn, w, off, cw);
      const int left = plan.bits - (int)off;
      const double h = std::ldexp(1.0, std::max(0, std::min((int)cw - 1, left)));
      const double load = (double)plan.n / h;
      fullest = t.Wr == 1 ? fullest + load : std::max(fullest, load);
    }
    if (fullest > 0.5 * FIX_SERIAL * t.K) {
      uint8_t* pb;
      int pbi;
      if ((rc = tail_pinned_acquire(ctx, 16, &pb, &pbi))) return rc;
      const hipError_t e1 = hipMemcpyAsync(pb, errw.p, 16, hipMemcpyDeviceToHost, st);
      const hipError_t e2 = e1 == hipSuccess ? hipStreamSynchronize(st) : e1;
      uint32_t ms;
      memcpy(&ms, pb + 4, 4);
      tail_pinned_release(ctx, pbi);
      GM_HIP(e2);
      if (ms > FIX_SERIAL) {
        if ((rc = msm_fix_long<C, G2>(ctx, t, ms))) return rc;
        GM_HIP(hipMemsetAsync(errw.as<uint32_t>() + 1, 0, 4, st));  // long spans resolved
      }
    }
  }
  if ((rc = msm_reduce<C, G2>(ctx, t))) return rc;
  return msm_readback<C, G2>(ctx, t);
}

// Host tail of a launched MSM: waits for its readback (not for the stream),
// redoes the reduction after a tree fixup if a long span showed up, then the
// host Horner over the window / bit-position nodes.
template <class C, bool G2>
int msm_finish(gm_ctx* ctx, MsmTail& t, typename GroupSel<C, G2>::HF (&jac_out)[3]) {
  using HF = typename GroupSel<C, G2>::HF;
  using HJ = host::Jac<HF>;
  if (t.n == 0) {
    HJ inf = HJ::inf();
    jac_out[0] = inf.x;
    jac_out[1] = inf.y;
    jac_out[2] = inf.z;
    return GM_OK;
  }
  int rc;
  GM_HIP(hipEventSynchronize(t.done));
  uint32_t herr, maxspan;
  memcpy(&herr, t.stage, 4);
  memcpy(&maxspan, t.stage + 4, 4);
  if (maxspan > FIX_SERIAL) {
    if ((rc = msm_fix_long<C, G2>(ctx, t, maxspan)) || (rc = msm_reduce<C, G2>(ctx, t)) ||
        (rc = msm_readback<C, G2>(ctx, t)))
      return rc;
    GM_HIP(hipEventSynchronize(t.done));
    memcpy(&herr, t.stage, 4);
  }
  if (herr) {
    set_error("msm: internal consistency check failed (code " + std::to_string(herr) + ")");
    return GM_ERR_DEVICE;
  }
  const uint32_t Wr = t.Wr, Q = t.Q, c = t.c;
  std::vector<HF> hw(4 * (size_t)Wr * Q);
  memcpy(hw.data(), t.stage + 16, sizeof(HF) * hw.size());
  t.release_stage();  // the buffer may serve the next readback
  // Host Horner over bit positions: window w (bit offset off_w, window_geom)
  // contributes U_w at 2^off_w and Y_{w,b} at 2^(off_w + log2 L + b)
  // (b < Q - 2 = log2(nseg), log2 L + log2 nseg = c - 1, so every exponent
  // stays below the next window's offset).  Shared buckets: one window, w = 0.
  uint32_t lgL = 0;
  while ((1u << lgL) < t.L) lgL++;
  const int top = (int)(c * Wr);
  std::vector<std::vector<uint32_t>> at(top + 1);  // point ids per exponent
  for (uint32_t w = 0; w < Wr; w++) {
    uint32_t off, cw;
    window_geom(c, Wr == 1 ? 1u : t.wn, w, off, cw);
    at[off].push_back(w * Q + 1);
    for (uint32_t b = 0; b + 2 < Q; b++) at[off + lgL + b].push_back(w * Q + 2 + b);
  }
  HJ acc = HJ::inf();
  for (int e = top; e >= 0; e--) {
    if (!acc.is_inf()) acc = host::jdbl(acc);
    for (uint32_t id : at[e]) {
      const HF* p = &hw[4 * (size_t)id];
      if (p[2].is_zero()) continue;
      acc = host::jadd(acc, host::xyzz_to_jac(p[0], p[1], p[2], p[3]));
    }
  }
  jac_out[0] = acc.x;
  jac_out[1] = acc.y;
  jac_out[2] = acc.z;
  return GM_OK;
}

template <class C, bool G2>
int msm_run(gm_ctx* ctx, const MsmPlan& plan, const void* points_internal,
            typename GroupSel<C, G2>::HF (&jac_out)[3]) {
  Arena arena(ctx);
  MsmTail t;
  int rc = msm_launch<C, G2>(ctx, arena, plan, points_internal, t);
  return rc ? rc : msm_finish<C, G2>(ctx, t, jac_out);
}

template <class C, bool G2>
int msm_device_launch(gm_ctx* ctx, Arena& arena, const void* scalars_dev, const void* points_dev, size_t n,
                      bool points_internal, const MsmPrecomp* pre, MsmTail& t, hipEvent_t inputs_read) {
  using DF = typename GroupSel<C, G2>::DF;
  int rc;
  const void* pts = points_dev;
  DevBuf ipts;
  bool glv = false;
  if (!points_internal && n) {
    if (pre && pre->c) {
      set_error("msm: a precomputed point set must be device-internal");
      return GM_ERR_INVALID;
    }
    glv = Glv<C>::ok && msm_glv_on(ctx, G2, n);
    if ((rc = ipts.alloc(arena, 2 * Coord<DF>::WORDS * sizeof(uint32_t) * n * (glv ? 2 : 1)))) return rc;
    ProfScope ps(ctx, "msm_convert_points");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(points_dev);
    if (glv)
      hipLaunchKernelGGL((k_msm_convert_points_lds<DF, true>), dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                         src, n, ipts.as<uint32_t>());
    else
      hipLaunchKernelGGL((k_msm_convert_points_lds<DF, false>), dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                         src, n, ipts.as<uint32_t>());
    pts = ipts.p;
  }
  MsmPlan plan;
  if ((rc = msm_plan<C>(ctx, arena, scalars_dev, n, pre, plan, glv))) return rc;
  // the caller's scalars (digits) and gnark-layout points (conversion) are not
  // read past this point
  if (inputs_read) GM_HIP(hipEventRecord(inputs_read, ctx->stream));
  return msm_launch<C, G2>(ctx, arena, plan, pts, t);
}

template <class C, bool G2>
int msm_device(gm_ctx* ctx, const void* scalars_dev, const void* points_dev, size_t n,
               typename GroupSel<C, G2>::HF (&jac_out)[3], bool points_internal, const MsmPrecomp* pre) {
  Arena arena(ctx);
  MsmTail t;
  int rc = msm_device_launch<C, G2>(ctx, arena, scalars_dev, points_dev, n, points_internal, pre, t);
  return rc ? rc : msm_finish<C, G2>(ctx, t, jac_out);
}

template <class C, bool G2>
size_t msm_internal_point_bytes() {
  return 2 * Coord<typename GroupSel<C, G2>::DF>::WORDS * sizeof(uint32_t);
}

template <class C, bool G2>
int msm_prepare_points(gm_ctx* ctx, const void* gnark_points, size_t n, void* dst) {
  using DF = typename GroupSel<C, G2>::DF;
  if (n == 0) return GM_OK;
  hipLaunchKernelGGL(k_msm_convert_points<DF>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                     reinterpret_cast<const uint32_t*>(gnark_points), n, reinterpret_cast<uint32_t*>(dst));
  GM_HIP(hipGetLastError());
  return GM_OK;
}

template <class C, bool G2>
int msm_precompute_points(gm_ctx* ctx, const void* gnark_points, size_t n, const MsmPrecomp& pre, void* dst) {
  using DF = typename GroupSel<C, G2>::DF;
  if (n == 0) return GM_OK;
  if (pre.stride < n || pre.W == 0 || pre.c == 0) {
    set_error("msm precompute: bad layout");
    return GM_ERR_INVALID;
  }
  hipLaunchKernelGGL(k_msm_convert_points<DF>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                     reinterpret_cast<const uint32_t*>(gnark_points), n, reinterpret_cast<uint32_t*>(dst));
  if (pre.W > 1)
    hipLaunchKernelGGL(k_msm_precompute<DF>, dim3(blocks_for(n, 128)), dim3(128), 0, ctx->stream,
                       reinterpret_cast<uint32_t*>(dst), n, pre.stride, pre.c, pre.W, pre.W - pre.narrow);
  GM_HIP(hipGetLastError());
  return GM_OK;
}

// Explicit instantiation for one (curve, group); each lives in its own
// translation unit (msm_<curve>_<group>.hip) so the four compile in parallel.
// The scalar-only plan is instantiated with the G1 unit.
#define GM_MSM_INSTANTIATE(C, G2)                                                              \
  template size_t msm_internal_point_bytes<C, G2>();                                          \
  template int msm_prepare_points<C, G2>(gm_ctx*, const void*, size_t, void*);                \
  template int msm_precompute_points<C, G2>(gm_ctx*, const void*, size_t, const MsmPrecomp&, void*); \
  template int msm_run<C, G2>(gm_ctx*, const MsmPlan&, const void*, typename GroupSel<C, G2>::HF (&)[3]); \
  template int msm_launch<C, G2>(gm_ctx*, Arena&, const MsmPlan&, const void*, MsmTail&);      \
  template int msm_finish<C, G2>(gm_ctx*, MsmTail&, typename GroupSel<C, G2>::HF (&)[3]);     \
  template int msm_device_launch<C, G2>(gm_ctx*, Arena&, const void*, const void*, size_t, bool, \
                                        const MsmPrecomp*, MsmTail&, hipEvent_t);              \
  template int msm_device<C, G2>(gm_ctx*, const void*, const void*, size_t,                    \
                                 typename GroupSel<C, G2>::HF (&)[3], bool, const MsmPrecomp*);
#define GM_MSM_INSTANTIATE_PLAN(C) \
  template int msm_plan<C>(gm_ctx*, Arena&, const void*, size_t, const MsmPrecomp*, MsmPlan&, bool);

}  // namespace gm
