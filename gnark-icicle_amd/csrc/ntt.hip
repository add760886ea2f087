// Radix-2 NTT over Fr on gfx950 -- replaces iciclegnark GenerateTwiddleFactors /
// NttOnDevice / INttOnDevice / PolyOps / ReverseScalars
// (backend/groth16/bn254/icicle/icicle.go:68-76,489-510) with gnark-crypto
// fft.Domain semantics (prove.go:372-378,396):
//   DIF: natural-order input -> bit-reversed output (Gentleman-Sande)
//   DIT: bit-reversed input  -> natural-order output (Cooley-Tukey)
//
// Decomposition (four-step, applied recursively): n = 2^logn is split into
// passes over index-bit ranges [lo, lo+t), t <= 8.  A pass runs, for every
// "other index" o = (hi, L), a 2^t-point sub-transform along j (element address
// hi*2^(lo+t) + j*2^lo + L) inside an LDS tile, and multiplies position (j, L)
// by w_{N'}^(L * bitrev_t(j)), N' = 2^(lo+t).  DIF runs passes high bits ->
// low bits with the twiddle after the sub-transform; DIT is the transpose:
// low -> high with the twiddle before.  Three passes cover 2^24 (8+8+8), i.e.
// three HBM round trips instead of 24.
#include <cstdlib>
#include <type_traits>

#include "curves.hpp"
#include "ntt.hpp"
#include "runtime.hpp"

namespace gm {

constexpr int NTT_TILE_LOG = 10;  // elements per LDS tile (32 KiB of Fr)
constexpr int NTT_TILE = 1 << NTT_TILE_LOG;
constexpr int NTT_TPB = 256;
constexpr int NTT_TMAX = 8;

// data vectors: gnark-layout words in HBM, unpacked limbs in registers / LDS
template <class P>
GM_DEV Fe<P> ld_fe(const Fe<P>* __restrict__ p, size_t i) {
  return fe_load_g<P>(p, i);
}
template <class P>
GM_DEV void st_fe(Fe<P>* __restrict__ p, size_t i, const Fe<P>& v) {
  fe_store_g<P>(p, i, v);
}
// device tables (twiddles, coset powers): internal limbs, stored as-is
template <class P>
GM_DEV Fe<P> ld_tab(const Fe<P>* __restrict__ t, size_t i) {
  return t[i];
}

GM_DEV uint32_t brev_bits(uint32_t x, int bits) { return bits ? (__brev(x) >> (32 - bits)) : 0; }

// One pass over index bits [lo, lo+t).  sub: w_T^x for x < T/2 (T = 2^t);
// tw: inter-pass twiddles (null if lo == 0).  Fused element-wise factors, all
// indexed by the element's global address:
//   pb, pc  first pass only: the loaded value a becomes a*b - c (computeH PolyOps)
//   pre     first pass only: multiply on load (coset powers)
//   post    last pass only: multiply on store (1/n, coset^-1, 1/(g^n - 1))
//
// Butterflies are Harvey-style lazy: tile values live in [0, 2p) (DIF) or
// [0, 4p) (DIT) between stages (no final subtraction in the twiddle product, 2p
// offsets instead of sign tests; field.hpp "Lazily reduced arithmetic"): one
// conditional subtraction per butterfly, canonical again on store.
//
// Butterfly enumeration of a stage with half-size m = 2^lm (NBF = 512 per tile):
//  * m <= 2: twiddle-index-major, so each wave shares one twiddle index jj and the
//    jj == 0 butterflies (twiddle 1: all of stage m = 1, half of m = 2) skip their
//    multiplication wave-uniformly (~19% of the stage multiplications);
//  * m >= 4: column-minor / jj-next, so consecutive lanes touch consecutive LDS
//    elements (9-dword stride, coprime with the 64 banks: conflict-free); the
//    jj-major order would put lanes 72m dwords apart (8- to 16-way conflicts).
GM_DEV void bfly_index(int q, int lm, int lgB, int& jj, int& ol, int& grp) {
  if (lm <= 1) {
    jj = q >> (NTT_TILE_LOG - 1 - lm);
    const int rem = q & ((NTT_TILE / 2 >> lm) - 1);
    ol = rem & ((1 << lgB) - 1);
    grp = rem >> lgB;
  } else {
    ol = q & ((1 << lgB) - 1);
    const int k = q >> lgB;
    jj = k & ((1 << lm) - 1);
    grp = k >> lm;
  }
}

// Radix-2 pass: the stages of one odd-t pass below t = 2 (k_ntt_pass4 runs the
// others).  Sub-transform twiddles are read through the cache, not staged in LDS
// (36 KiB of LDS per block: four blocks per CU; 1.5-2 % at 2^24 in r03,
// profiles/r03m_ntt_swg_ab.txt).
template <class P, bool DIT>
__global__ void __launch_bounds__(NTT_TPB) k_ntt_pass(Fe<P>* __restrict__ data, int logn, int lo,
                                                      int t, const Fe<P>* __restrict__ tw,
                                                      const Fe<P>* __restrict__ sub,
                                                      const Fe<P>* __restrict__ pre,
                                                      const Fe<P>* __restrict__ post,
                                                      const Fe<P>* __restrict__ pb,
                                                      const Fe<P>* __restrict__ pc) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Fe<P>* X = reinterpret_cast<Fe<P>*>(smem_raw);   // [T][B]
  constexpr int TPB = NTT_TPB;
  const int T = 1 << t;
  const int lgB = NTT_TILE_LOG - t;
  const int B = 1 << lgB;
  const size_t nother = (size_t)1 << (logn - t);
  const size_t o0 = (size_t)blockIdx.x * B;
  const size_t lomask = ((size_t)1 << lo) - 1;

  const Fe<P>* __restrict__ SW = sub;

  // load (j, o) -> X[j*B + o]
  for (int q = threadIdx.x; q < NTT_TILE; q += TPB) {
    int j, ol;
    if (lo == 0) {
      j = q & (T - 1);
      ol = q >> t;
    } else {
      ol = q & (B - 1);
      j = q >> lgB;
    }
    const size_t o = o0 + ol;
    if (o >= nother) continue;
    const size_t hi = o >> lo, L = o & lomask;
    const size_t addr = (hi << (lo + t)) + ((size_t)j << lo) + L;
    Fe<P> v = ld_fe(data, addr);
    if (pb) v = fe_sub(fe_mul(v, fe_to_internal(ld_fe(pb, addr))), ld_fe(pc, addr));
    if (pre) v = fe_mul(v, ld_tab(pre, addr));
    // inter-pass twiddle, lazily reduced (< 2p; the DIT tile takes < 4p)
    if (DIT && lo > 0) v = fe_mul_lz(v, ld_tab(tw, ((size_t)j << lo) + L));
    X[j * B + ol] = v;
  }
  __syncthreads();

  // Stages with lm >= 2 mix twiddle indices inside a wave (jj = 0 next to jj != 0
  // lanes), so a jj == 0 branch would cost those waves the multiplication AND the
  // reduction: there every lane multiplies (SW[0] = 1).  Stages lm <= 1 are
  // twiddle-index-major, i.e. wave-uniform, and keep the skip.
  constexpr int NBF = NTT_TILE / 2;  // butterflies per stage
  if (!DIT) {
    // inputs < 2p: s < 4p -> one conditional subtraction; d = (u - v + 2p) w < 2p
    for (int lm = t - 1; lm >= 0; lm--) {
      const int m = 1 << lm, step = T >> (lm + 1);
      if (lm >= 2 && NBF == 2 * TPB) {
        // two butterflies per thread, loads first: two independent product chains
        int jj[2], ol[2], grp[2], i0[2], i1[2];
        Fe<P> u[2], v[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          bfly_index(threadIdx.x + h * TPB, lm, lgB, jj[h], ol[h], grp[h]);
          const int j0 = (grp[h] << (lm + 1)) + jj[h];
          i0[h] = j0 * B + ol[h];
          i1[h] = (j0 + m) * B + ol[h];
          u[h] = X[i0[h]];
          v[h] = X[i1[h]];
        }
        Fe<P> s[2], d[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          s[h] = fe_add_lz(u[h], v[h]);               // < 4p
          fe_reduce_k<2>(s[h]);
          d[h] = fe_mul_lz(fe_sub_lz<2>(u[h], v[h]), SW[jj[h] * step]);  // < 2p
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
          X[i0[h]] = s[h];
          X[i1[h]] = d[h];
        }
        __syncthreads();
        continue;
      }
      for (int q = threadIdx.x; q < NBF; q += TPB) {
        int jj, ol, grp;
        bfly_index(q, lm, lgB, jj, ol, grp);
        const int j0 = (grp << (lm + 1)) + jj, j1 = j0 + m;
        const Fe<P> u = X[j0 * B + ol], v = X[j1 * B + ol];
        Fe<P> s = fe_add_lz(u, v);                    // < 4p
        fe_reduce_k<2>(s);
        X[j0 * B + ol] = s;
        Fe<P> d = fe_sub_lz<2>(u, v);                 // < 4p
        if (lm >= 2) {                                // block-uniform branch
          d = fe_mul_lz(d, SW[jj * step]);            // 4p * p < R' p: < 2p
        } else if (jj) {
          d = fe_mul_lz(d, SW[jj * step]);
        } else {
          fe_reduce_k<2>(d);
        }
        X[j1 * B + ol] = d;
      }
      __syncthreads();
    }
  } else {
    // Harvey: tile values < 4p; u -> < 2p (one conditional subtraction),
    // v w < 2p, then s = u + v w and d = u - v w + 2p are both < 4p unreduced.
    for (int lm = 0; lm < t; lm++) {
      const int m = 1 << lm, step = T >> (lm + 1);
      if (lm >= 2 && NBF == 2 * TPB) {
        // two butterflies per thread, loads first: two independent product chains
        int jj[2], ol[2], grp[2], i0[2], i1[2];
        Fe<P> u[2], v[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          bfly_index(threadIdx.x + h * TPB, lm, lgB, jj[h], ol[h], grp[h]);
          const int j0 = (grp[h] << (lm + 1)) + jj[h];
          i0[h] = j0 * B + ol[h];
          i1[h] = (j0 + m) * B + ol[h];
          u[h] = X[i0[h]];
          v[h] = X[i1[h]];
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
          fe_reduce_k<2>(u[h]);                       // < 2p
          v[h] = fe_mul_lz(v[h], SW[jj[h] * step]);   // < 2p
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
          X[i0[h]] = fe_add_lz(u[h], v[h]);           // < 4p
          X[i1[h]] = fe_sub_lz<2>(u[h], v[h]);        // < 4p
        }
        __syncthreads();
        continue;
      }
      for (int q = threadIdx.x; q < NBF; q += TPB) {
        int jj, ol, grp;
        bfly_index(q, lm, lgB, jj, ol, grp);
        const int j0 = (grp << (lm + 1)) + jj, j1 = j0 + m;
        Fe<P> u = X[j0 * B + ol];
        Fe<P> v = X[j1 * B + ol];
        fe_reduce_k<2>(u);                            // < 2p
        if (lm >= 2) {                                // block-uniform branch
          v = fe_mul_lz(v, SW[jj * step]);            // 4p * p < R' p: < 2p
        } else if (jj) {
          v = fe_mul_lz(v, SW[jj * step]);
        } else {
          fe_reduce_k<2>(v);
        }
        X[j0 * B + ol] = fe_add_lz(u, v);             // < 4p
        X[j1 * B + ol] = fe_sub_lz<2>(u, v);          // < 4p
      }
      __syncthreads();
    }
  }

  for (int q = threadIdx.x; q < NTT_TILE; q += TPB) {
    int j, ol;
    if (lo == 0) {
      j = q & (T - 1);
      ol = q >> t;
    } else {
      ol = q & (B - 1);
      j = q >> lgB;
    }
    const size_t o = o0 + ol;
    if (o >= nother) continue;
    const size_t hi = o >> lo, L = o & lomask;
    const size_t addr = (hi << (lo + t)) + ((size_t)j << lo) + L;
    Fe<P> v = X[j * B + ol];  // < 2p (DIF) / < 4p (DIT); canonical before the store
    // inter-pass twiddle of a DIF pass with lo > 0: never the last pass (that one
    // has lo = 0), so the value is stored lazily reduced (< 2p) for the next
    // pass, whose tile takes < 2p
    if (!DIT && lo > 0) v = fe_mul_lz(v, ld_tab(tw, ((size_t)j << lo) + L));
    if (post) v = fe_mul(v, ld_tab(post, addr));
    if (!(!DIT && lo > 0) && !post) {
      if (DIT) fe_reduce_k<2>(v);
      fe_reduce_once(v);
    }
    st_fe(data, addr, v);
  }
}

// ---------------------------------------------------------------------------
// Radix-4 pass (default for t >= 2): the same pass as k_ntt_pass, but every
// thread keeps four tile elements in registers and runs TWO radix-2 stages on
// them between LDS exchanges.  A tile of 1024 elements is 256 groups of four:
// round r takes elements j0 + {0, s, 2s, 3s} of column ol (quarter spacing
// s = 2^ls, j0 = grp * 4s + jj, jj < s), so
//   * the first round loads straight from HBM (fused pb/pc, pre and DIT twiddle)
//     and the last round stores straight to HBM: the tile crosses LDS t/2 - 1
//     times instead of t + 1 (t = 8: 3 exchanges instead of 9, 6 barriers
//     instead of 9);
//   * each round is four butterflies = four independent-ish product chains per
//     thread (two per stage) and only three twiddle loads (w_2m^jj, w_2m^(jj+s),
//     w_m^jj for DIF);
//   * rounds whose twiddles are 1 and w_4 (s = 1: the last DIF round, the first
//     DIT round) do one product instead of four, block-uniformly.
// An odd t leaves one radix-2 stage, run on the LDS tile at the end (DIF lm = 0,
// DIT lm = t - 1) exactly as in k_ntt_pass.
// Bounds: DIF round inputs < 2p, outputs < 2p (two of the four sums reduced),
// except the s = 1 round, whose outputs (< 8p) go straight to the store; DIT
// (Harvey) round inputs < 4p, outputs < 4p.  Intermediate DIT passes store
// lazily reduced (< 4p < 2^256; the next pass multiplies on load).
// ---------------------------------------------------------------------------
// waves per SIMD the radix-4 pass is compiled for (1: the compiler's choice);
// A/B builds override it with -DNTT_R4_WPE=4
#ifndef NTT_R4_WPE
#define NTT_R4_WPE 1
#endif
// round twiddles of the DIF pass fetched one round ahead (k_ntt_pass4)
#ifndef NTT_TW_PF
#define NTT_TW_PF 1
#endif
// the BN254 DIT kernel: four waves per SIMD (the growing-bound rounds take it from
// 123 to 132 VGPRs uncapped; capped at 128 it does not spill)
#ifndef NTT_DIT_WPE_BN254
#define NTT_DIT_WPE_BN254 4
#endif
// the DIF kernel (inter-pass twiddles on the store) separately: -DNTT_DIF_WPE=3
#ifndef NTT_DIF_WPE
#define NTT_DIF_WPE NTT_R4_WPE
#endif

// f(0), f(1), f(2), f(3) with compile-time indices (register-resident arrays)
template <class F>
GM_DEV void unroll4(F&& f) {
  f(std::integral_constant<int, 0>());
  f(std::integral_constant<int, 1>());
  f(std::integral_constant<int, 2>());
  f(std::integral_constant<int, 3>());
}

template <class P>
GM_DEV Fe<P> ntt_tw(const Fe<P>* __restrict__ sub, int i) {
  return sub[i];
}

// products of a round: one mad chain each (CH) or the compiler's split columns.
// A difference that only feeds a product is formed carry-free (fe_sub_cf: value
// below a + K p with K one above fe_sub_lz's, every product input < 33 p^2 < R' p).
// NTT_BFLY_CHAIN: the butterflies' chain level.  Strict (2, as the load / store
// products): 2^24 transform 2.072-2.091 -> 2.047-2.061 ms, coset within noise
// (profiles/r06d_ntt_bfly_chain_ab.txt); 1 = one chain per column (r05).
#ifndef NTT_BFLY_CHAIN
#define NTT_BFLY_CHAIN 2
#endif
#define MUL(x, y) (CH ? fe_mul<P, false, NTT_BFLY_CHAIN>(x, y) : fe_mul_lz(x, y))
// DIF radix-2 butterfly pair of one round: (u, v) -> (u + v, (u - v + Kp) w)
template <class P, int CH>
GM_DEV void r4_dif(Fe<P> (&e)[4], const Fe<P>& t1, const Fe<P>& t2, const Fe<P>& t3) {
  // stage lm: (e0, e2) by w_2m^jj, (e1, e3) by w_2m^(jj+s); inputs < 2p
  const Fe<P> s0 = fe_add_lz(e[0], e[2]);                        // < 4p
  const Fe<P> d0 = MUL(fe_sub_cf<3>(e[0], e[2]), t1);      // < 2p
  const Fe<P> s1 = fe_add_lz(e[1], e[3]);                        // < 4p
  const Fe<P> d1 = MUL(fe_sub_cf<3>(e[1], e[3]), t2);      // < 2p
  // stage lm - 1: (s0, s1), (d0, d1) by w_m^jj
  e[0] = fe_add_lz(s0, s1);                                      // < 8p
  fe_reduce_k<4>(e[0]);
  fe_reduce_k<2>(e[0]);                                          // < 2p
  e[1] = MUL(fe_sub_cf<5>(s0, s1), t3);                    // < 2p
  e[2] = fe_add_lz(d0, d1);                                      // < 4p
  fe_reduce_k<2>(e[2]);                                          // < 2p
  e[3] = MUL(fe_sub_cf<3>(d0, d1), t3);                    // < 2p
}
// the s = 1 DIF round (twiddles 1, w_4, 1): inputs < 2p, outputs < 8p
template <class P, int CH>
GM_DEV void r4_dif_w4(Fe<P> (&e)[4], const Fe<P>& w4) {
  const Fe<P> s0 = fe_add_lz(e[0], e[2]);                        // < 4p
  const Fe<P> d0 = fe_sub_lz<2>(e[0], e[2]);                     // < 4p
  const Fe<P> s1 = fe_add_lz(e[1], e[3]);                        // < 4p
  const Fe<P> d1 = MUL(fe_sub_cf<3>(e[1], e[3]), w4);      // < 2p
  e[0] = fe_add_lz(s0, s1);                                      // < 8p
  e[1] = fe_sub_lz<4>(s0, s1);                                   // < 8p
  e[2] = fe_add_lz(d0, d1);                                      // < 6p
  e[3] = fe_sub_lz<2>(d0, d1);                                   // < 6p
}
// DIF rounds of a pass that is not the last one (lo > 0, even t): bounds grow
// instead of every sum being reduced -- round R takes inputs < B p (B = 2^(R+1))
// and reduces only e0 (one conditional subtraction per round instead of three);
// the products (< 2p) reset the other lanes.  The last (w_4) round's outputs,
// < 64p at t = 8, go straight into the inter-pass twiddle product of the store
// (64 p^2 < R' p).
template <class P, int CH, int B>
GM_DEV void r4_dif_grow(Fe<P> (&e)[4], const Fe<P>& t1, const Fe<P>& t2, const Fe<P>& t3) {
  const Fe<P> s0 = fe_add_lz(e[0], e[2]);                        // < 2B p
  const Fe<P> d0 = MUL(fe_sub_cf<B + 1>(e[0], e[2]), t1);        // < 2p
  const Fe<P> s1 = fe_add_lz(e[1], e[3]);                        // < 2B p
  const Fe<P> d1 = MUL(fe_sub_cf<B + 1>(e[1], e[3]), t2);        // < 2p
  e[0] = fe_add_lz(s0, s1);                                      // < 4B p
  fe_reduce_k<2 * B>(e[0]);                                      // < 2B p
  e[1] = MUL(fe_sub_cf<2 * B + 1>(s0, s1), t3);                  // < 2p (value < (4B + 1) p)
  e[2] = fe_add_lz(d0, d1);                                      // < 4p
  e[3] = MUL(fe_sub_cf<3>(d0, d1), t3);                          // < 2p
}
template <class P, int CH, int B>
GM_DEV void r4_dif_w4_grow(Fe<P> (&e)[4], const Fe<P>& w4) {
  const Fe<P> s0 = fe_add_lz(e[0], e[2]);                        // < 2B p
  const Fe<P> d0 = fe_sub_lz<B>(e[0], e[2]);                     // < 2B p
  const Fe<P> s1 = fe_add_lz(e[1], e[3]);                        // < 2B p
  const Fe<P> d1 = MUL(fe_sub_cf<B + 1>(e[1], e[3]), w4);        // < 2p
  e[0] = fe_add_lz(s0, s1);                                      // < 4B p
  e[1] = fe_sub_lz<2 * B>(s0, s1);                               // < 4B p
  e[2] = fe_add_lz(d0, d1);                                      // < (2B + 2) p
  e[3] = fe_sub_lz<2>(d0, d1);                                   // < (2B + 2) p
}
// DIT (Harvey) round: (u, v) -> (u + v w, u - v w + 2p); inputs < 4p, outputs < 4p
template <class P, int CH>
GM_DEV void r4_dit(Fe<P> (&e)[4], const Fe<P>& a, const Fe<P>& b, const Fe<P>& c) {
  // stage lm: (e0, e1), (e2, e3) by w_2m^jj
  fe_reduce_k<2>(e[0]);
  fe_reduce_k<2>(e[2]);
  const Fe<P> v1 = MUL(e[1], a);                           // < 2p
  const Fe<P> v3 = MUL(e[3], a);
  Fe<P> s0 = fe_add_lz(e[0], v1);                                // < 4p
  Fe<P> s1 = fe_sub_lz<2>(e[0], v1);
  const Fe<P> s2 = fe_add_lz(e[2], v3);
  const Fe<P> s3 = fe_sub_cf<3>(e[2], v3);                       // product operand only
  // stage lm + 1: (s0, s2) by w_4m^jj, (s1, s3) by w_4m^(jj+s)
  fe_reduce_k<2>(s0);
  fe_reduce_k<2>(s1);
  const Fe<P> x = MUL(s2, b);
  const Fe<P> y = MUL(s3, c);
  e[0] = fe_add_lz(s0, x);
  e[2] = fe_sub_lz<2>(s0, x);
  e[1] = fe_add_lz(s1, y);
  e[3] = fe_sub_lz<2>(s1, y);
}
// the s = 1 DIT round (twiddles 1, 1, w_4): inputs < 2p, outputs < 4p
template <class P, int CH>
GM_DEV void r4_dit_w4(Fe<P> (&e)[4], const Fe<P>& w4) {
  const Fe<P> s0 = fe_add_lz(e[0], e[1]);                        // < 4p
  const Fe<P> s1 = fe_sub_lz<2>(e[0], e[1]);                     // < 4p
  const Fe<P> s2 = fe_add_lz(e[2], e[3]);                        // < 4p
  const Fe<P> y = MUL(fe_sub_cf<3>(e[2], e[3]), w4);       // < 2p
  e[0] = fe_add_lz(s0, s2);                                      // < 8p
  e[2] = fe_sub_lz<4>(s0, s2);                                   // < 8p
  e[1] = fe_add_lz(s1, y);                                       // < 6p
  e[3] = fe_sub_lz<2>(s1, y);                                    // < 6p
  unroll4([&](auto I) { fe_reduce_k<4>(e[I]); });               // < 4p
}
// DIT rounds with growing bounds (even t, GM_NTT_GROW bit 1): no conditional
// subtraction inside the pass.  The w_4 round takes inputs < 2p and leaves
// < 8p; a generic round takes < B p and leaves < (B + 4) p (products < 2p, every
// product input below 19p); the store brings the < 20p (t = 8) outputs below 4p
// with three subtractions per element instead of four per round.
template <class P, int CH>
GM_DEV void r4_dit_grow(Fe<P> (&e)[4], const Fe<P>& a, const Fe<P>& b, const Fe<P>& c) {
  const Fe<P> v1 = MUL(e[1], a);                                 // < 2p
  const Fe<P> v3 = MUL(e[3], a);
  const Fe<P> s0 = fe_add_lz(e[0], v1);                          // < (B + 2) p
  const Fe<P> s1 = fe_sub_lz<2>(e[0], v1);
  const Fe<P> s2 = fe_add_lz(e[2], v3);
  const Fe<P> y = MUL(fe_sub_cf<3>(e[2], v3), c);                // < 2p
  const Fe<P> x = MUL(s2, b);
  e[0] = fe_add_lz(s0, x);                                       // < (B + 4) p
  e[2] = fe_sub_lz<2>(s0, x);
  e[1] = fe_add_lz(s1, y);
  e[3] = fe_sub_lz<2>(s1, y);
}
template <class P, int CH>
GM_DEV void r4_dit_w4_grow(Fe<P> (&e)[4], const Fe<P>& w4) {
  const Fe<P> s0 = fe_add_lz(e[0], e[1]);                        // < 4p
  const Fe<P> s1 = fe_sub_lz<2>(e[0], e[1]);                     // < 4p
  const Fe<P> s2 = fe_add_lz(e[2], e[3]);                        // < 4p
  const Fe<P> y = MUL(fe_sub_cf<3>(e[2], e[3]), w4);             // < 2p
  e[0] = fe_add_lz(s0, s2);                                      // < 8p
  e[2] = fe_sub_lz<4>(s0, s2);                                   // < 8p
  e[1] = fe_add_lz(s1, y);                                       // < 6p
  e[3] = fe_sub_lz<2>(s1, y);                                    // < 6p
}

#undef MUL

// twiddles of a round whose lower stage is ls: w_4 for ls = 0, else DIF
// (t1, t2, t3) / DIT (a, b, c) of the thread's group k
template <class P, bool DIT>
GM_DEV void r4_fetch_tw(const Fe<P>* __restrict__ sub, int t, int ls, int k, Fe<P>& tw0, Fe<P>& tw1, Fe<P>& tw2) {
  const int sr = 1 << ls, jj = k & (sr - 1);
  if (sr == 1) {
    tw0 = tw1 = tw2 = ntt_tw(sub, 1 << (t - 2));  // all three written: nothing stays live across rounds
  } else if (!DIT) {
    tw0 = ntt_tw(sub, jj << (t - ls - 2));
    tw1 = ntt_tw(sub, (jj + sr) << (t - ls - 2));
    tw2 = ntt_tw(sub, jj << (t - ls - 1));
  } else {
    tw0 = ntt_tw(sub, jj << (t - ls - 1));
    tw1 = ntt_tw(sub, jj << (t - ls - 2));
    tw2 = ntt_tw(sub, (jj + sr) << (t - ls - 2));
  }
}

template <class P, bool DIT, int CH = 0>
__global__ void __launch_bounds__(NTT_TPB) __attribute__((amdgpu_waves_per_eu(DIT ? (std::is_same<P, Bn254Fr>::value ? NTT_DIT_WPE_BN254 : NTT_R4_WPE) : NTT_DIF_WPE))) k_ntt_pass4(Fe<P>* __restrict__ data, int logn, int lo, int t, int grow_mask,
                                                       const Fe<P>* __restrict__ tw,
                                                       const Fe<P>* __restrict__ sub,
                                                       const Fe<P>* __restrict__ pre,
                                                       const Fe<P>* __restrict__ post,
                                                       const Fe<P>* __restrict__ pb,
                                                       const Fe<P>* __restrict__ pc) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Fe<P>* X = reinterpret_cast<Fe<P>*>(smem_raw);  // [T][B]
  const int T = 1 << t;
  const int lgB = NTT_TILE_LOG - t;
  const int B = 1 << lgB;
  const size_t nother = (size_t)1 << (logn - t);
  const int ol = threadIdx.x & (B - 1);
  const int k = threadIdx.x >> lgB;  // group of the column: [0, T/4)
  const size_t o = (size_t)blockIdx.x * B + ol;
  const bool live = o < nother;
  const size_t lomask = ((size_t)1 << lo) - 1;
  const size_t base = ((o >> lo) << (lo + t)) + (o & lomask);  // (j, ol) lives at base + (j << lo)
  const bool last_pass = DIT ? (lo + t == logn) : (lo == 0);
  // growing DIF bounds (r4_dif_grow): passes whose store multiplies every element
  // by an inter-pass twiddle, with no lone radix-2 stage (it takes inputs < 2p);
  // GM_NTT_GROW=0 keeps every round's outputs < 2p (A/B)
  const bool grow = !DIT && lo > 0 && !(t & 1) && (grow_mask & 1);
  const bool dgrow = DIT && !(t & 1) && (grow_mask & 2);  // r4_dit_grow
  // rounds: DIF stages (t-1, t-2), (t-3, t-4), ...; DIT (0, 1), (2, 3), ...
  const int nr = t >> 1;
  auto quarter = [&](int r) { return DIT ? 2 * r : t - 2 - 2 * r; };  // ls of round r
  Fe<P> e[4];
  int j0 = 0, s = 0;
  auto place = [&](int r) {
    const int ls = quarter(r);
    s = 1 << ls;
    j0 = ((k >> ls) << (ls + 2)) + (k & (s - 1));
  };
  place(0);
  if (live) {
    unroll4([&](auto I) {
      const size_t addr = base + ((size_t)(j0 + I * s) << lo);
      Fe<P> v = ld_fe(data, addr);
      if (pb) v = fe_sub(fe_mul<P, true, CH>(v, fe_to_internal(ld_fe(pb, addr))), ld_fe(pc, addr));
      if (pre) v = fe_mul<P, true, CH>(v, ld_tab(pre, addr));
      if (DIT && lo > 0) v = fe_mul<P, false, CH>(v, ld_tab(tw, ((size_t)(j0 + I * s) << lo) + (o & lomask)));  // < 2p
      e[I] = v;
    });
  }
  // twiddles of round r: tw0 = w_4 for the s = 1 round, else DIF (t1, t2, t3) /
  // DIT (a, b, c).  The DIF pass (two waves per SIMD) fetches them one round
  // ahead, before the tile exchange, so their L2 latency overlaps the barriers
  // (NTT_TW_PF=0: fetched after the exchange, A/B); the DIT pass runs at four
  // waves and keeps the registers.
  Fe<P> tw0, tw1, tw2;
  constexpr bool tw_ahead = !DIT && NTT_TW_PF;
  if (tw_ahead && nr > 0) r4_fetch_tw<P, DIT>(sub, t, quarter(0), k, tw0, tw1, tw2);
  for (int r = 0; r < nr; r++) {
    if (r > 0) {
      // exchange through the tile: this round's elements of every thread
      __syncthreads();  // the previous round's reads are done
      unroll4([&](auto I) { X[(j0 + I * s) * B + ol] = e[I]; });
      __syncthreads();
      place(r);
      unroll4([&](auto I) { e[I] = X[(j0 + I * s) * B + ol]; });
    }
    if constexpr (tw_ahead) {
      if (grow) {  // lo > 0, even t (block-uniform): round r takes inputs < 2^(r+1) p
        if (s == 1) {
          switch (r) {
            case 0: r4_dif_w4_grow<P, CH, 2>(e, tw0); break;
            case 1: r4_dif_w4_grow<P, CH, 4>(e, tw0); break;
            case 2: r4_dif_w4_grow<P, CH, 8>(e, tw0); break;
            default: r4_dif_w4_grow<P, CH, 16>(e, tw0); break;
          }
        } else {
          switch (r) {
            case 0: r4_dif_grow<P, CH, 2>(e, tw0, tw1, tw2); break;
            case 1: r4_dif_grow<P, CH, 4>(e, tw0, tw1, tw2); break;
            default: r4_dif_grow<P, CH, 8>(e, tw0, tw1, tw2); break;
          }
        }
      } else if (s == 1) {
        r4_dif_w4<P, CH>(e, tw0);
      } else {
        r4_dif<P, CH>(e, tw0, tw1, tw2);
      }
    } else {
      // twiddles loaded where they are used (the DIT pass keeps four waves)
      const int ls = quarter(r);
      const int jj = k & (s - 1);
      if (grow) {
        if (s == 1) {
          const Fe<P> w4 = ntt_tw(sub, 1 << (t - 2));
          switch (r) {
            case 0: r4_dif_w4_grow<P, CH, 2>(e, w4); break;
            case 1: r4_dif_w4_grow<P, CH, 4>(e, w4); break;
            case 2: r4_dif_w4_grow<P, CH, 8>(e, w4); break;
            default: r4_dif_w4_grow<P, CH, 16>(e, w4); break;
          }
        } else {
          const Fe<P> t1 = ntt_tw(sub, jj << (t - ls - 2)), t2 = ntt_tw(sub, (jj + s) << (t - ls - 2)),
                      t3 = ntt_tw(sub, jj << (t - ls - 1));
          switch (r) {
            case 0: r4_dif_grow<P, CH, 2>(e, t1, t2, t3); break;
            case 1: r4_dif_grow<P, CH, 4>(e, t1, t2, t3); break;
            default: r4_dif_grow<P, CH, 8>(e, t1, t2, t3); break;
          }
        }
      } else if (s == 1) {  // block-uniform
        const Fe<P> w4 = ntt_tw(sub, 1 << (t - 2));
        if (DIT) {
          if (dgrow) r4_dit_w4_grow<P, CH>(e, w4);
          else r4_dit_w4<P, CH>(e, w4);
        } else {
          r4_dif_w4<P, CH>(e, w4);
        }
      } else if (!DIT) {
        r4_dif<P, CH>(e, ntt_tw(sub, jj << (t - ls - 2)), ntt_tw(sub, (jj + s) << (t - ls - 2)),
                      ntt_tw(sub, jj << (t - ls - 1)));
      } else if (dgrow) {
        r4_dit_grow<P, CH>(e, ntt_tw(sub, jj << (t - ls - 1)), ntt_tw(sub, jj << (t - ls - 2)),
                           ntt_tw(sub, (jj + s) << (t - ls - 2)));
      } else {
        r4_dit<P, CH>(e, ntt_tw(sub, jj << (t - ls - 1)), ntt_tw(sub, jj << (t - ls - 2)),
                      ntt_tw(sub, (jj + s) << (t - ls - 2)));
      }
    }
    if (tw_ahead && r + 1 < nr) r4_fetch_tw<P, DIT>(sub, t, quarter(r + 1), k, tw0, tw1, tw2);
  }
  if (t & 1) {
    // the lone radix-2 stage on the tile (DIF lm = 0 after the rounds: inputs
    // < 2p; DIT lm = t - 1: inputs < 4p), then the store from LDS
    __syncthreads();
    unroll4([&](auto I) { X[(j0 + I * s) * B + ol] = e[I]; });
    __syncthreads();
    const int lm = DIT ? t - 1 : 0;
    const int m = 1 << lm, step = T >> (lm + 1);
    for (int q = threadIdx.x; q < NTT_TILE / 2; q += NTT_TPB) {
      int jj, bol, grp;
      bfly_index(q, lm, lgB, jj, bol, grp);
      const int a0 = ((grp << (lm + 1)) + jj) * B + bol, a1 = a0 + m * B;
      Fe<P> u = X[a0], v = X[a1];
      if (!DIT) {
        Fe<P> sm = fe_add_lz(u, v);
        fe_reduce_k<2>(sm);
        Fe<P> d = fe_sub_lz<2>(u, v);
        if (lm >= 1) d = fe_mul_lz(d, ntt_tw(sub, jj * step));
        else fe_reduce_k<2>(d);
        X[a0] = sm;
        X[a1] = d;
      } else {
        fe_reduce_k<2>(u);
        if (jj || lm >= 2) v = fe_mul_lz(v, ntt_tw(sub, jj * step));
        else fe_reduce_k<2>(v);
        X[a0] = fe_add_lz(u, v);
        X[a1] = fe_sub_lz<2>(u, v);
      }
    }
    __syncthreads();
    unroll4([&](auto I) { e[I] = X[(j0 + I * s) * B + ol]; });  // < 2p (DIF) / < 4p (DIT)
  }
  if (!live) return;
  // store: the last round's (or the re-read lone-stage) elements.  Bounds here:
  // DIF < 8p (s = 1 round) or < 2p; DIT < 4p.
  const bool wide = !DIT && s == 1 && !(t & 1);
  unroll4([&](auto I) {
    const int j = j0 + I * s;
    const size_t addr = base + ((size_t)j << lo);
    Fe<P> v = e[I];
    if (dgrow && !post) {  // < 20p -> < 4p, the bound the branches below take
      fe_reduce_k<16>(v);
      fe_reduce_k<8>(v);
      fe_reduce_k<4>(v);
    }
    if (!DIT && lo > 0) {
      // inter-pass twiddle of a DIF pass (never the last pass): stored < 2p
      v = fe_mul<P, false, CH>(v, ld_tab(tw, ((size_t)j << lo) + (o & lomask)));
    } else if (post) {
      v = fe_mul<P, true, CH>(v, ld_tab(post, addr));  // inputs < 20p: (20p) p < R' p, output canonical
    } else if (DIT && !last_pass) {
      // lazily reduced (< 4p < 2^256): the next DIT pass multiplies it on load
    } else {
      if (wide) fe_reduce_k<4>(v);
      fe_reduce_k<2>(v);
      fe_reduce_once(v);
    }
    st_fe(data, addr, v);
  });
}

// ---------------------------------------------------------------------------
// table generation
// ---------------------------------------------------------------------------
template <class P>
GM_DEV Fe<P> fe_pow_u32(const Fe<P>& base, uint32_t e) {
  Fe<P> r = fe_one<P>();
  Fe<P> b = base;
  while (e) {
    if (e & 1) r = fe_mul(r, b);
    e >>= 1;
    if (e) b = fe_sqr(b);
  }
  return r;
}

// tw[j*2^lo + L] = w^(L * bitrev_t(j)), w = w_{2^(lo+t)} (canonical exponent < 2^(lo+t));
// w arrives in gnark form, tables are written in internal form.
template <class P>
__global__ void k_gen_pass_tw(Fe<P>* __restrict__ tw, int lo, int t, FeG<P> wg, FeG<P> mult_g) {
  const Fe<P> w = fe_to_internal(fe_unpack<P>(wg));
  const Fe<P> mult = fe_to_internal(fe_unpack<P>(mult_g));
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t size = (size_t)1 << (lo + t);
  if (i >= size) return;
  const uint32_t j = (uint32_t)(i >> lo), L = (uint32_t)(i & (((size_t)1 << lo) - 1));
  const uint64_t e = (uint64_t)L * brev_bits(j, t);
  // e < 2^(lo+t) <= 2^32 for supported sizes
  tw[i] = fe_mul(fe_pow_u32(w, (uint32_t)e), mult);
}

// out[x] = base^x * mult, x < count (gnark-form inputs, internal-form table)
template <class P>
__global__ void k_gen_powers(Fe<P>* __restrict__ out, size_t count, FeG<P> base_g, FeG<P> mult_g) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const Fe<P> base = fe_to_internal(fe_unpack<P>(base_g));
  const Fe<P> mult = fe_to_internal(fe_unpack<P>(mult_g));
  out[i] = fe_mul(fe_pow_u32(base, (uint32_t)i), mult);
}

// out[i] = mult * base^e, e = i or bitrev_logn(i) (full-size coset tables;
// gnark-form inputs, internal-form table)
template <class P, bool BREV>
__global__ void k_gen_coset(Fe<P>* __restrict__ out, size_t n, int logn, FeG<P> base_g, FeG<P> mult_g) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<P> base = fe_to_internal(fe_unpack<P>(base_g));
  const Fe<P> mult = fe_to_internal(fe_unpack<P>(mult_g));
  const uint32_t e = BREV ? brev_bits((uint32_t)i, logn) : (uint32_t)i;
  out[i] = fe_mul(fe_pow_u32(base, e), mult);
}

template <class P>
__global__ void __launch_bounds__(256) k_scale_const(Fe<P>* __restrict__ a, size_t n, FeG<P> kg) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<P> k = fe_to_internal(fe_unpack<P>(kg));
  st_fe(a, i, fe_mul(ld_fe(a, i), k));
}

// a <- (a*b - c) * den, all gnark form: mul(a_g, to_internal(b_g)) = (a*b)_g
template <class P>
__global__ void __launch_bounds__(256) k_poly_ops(Fe<P>* __restrict__ a, const Fe<P>* __restrict__ b,
                                                  const Fe<P>* __restrict__ c, size_t n, FeG<P> den_g) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<P> den = fe_to_internal(fe_unpack<P>(den_g));
  Fe<P> v = fe_sub(fe_mul(ld_fe(a, i), fe_to_internal(ld_fe(b, i))), ld_fe(c, i));
  st_fe(a, i, fe_mul(v, den));
}

template <class P>
__global__ void __launch_bounds__(256) k_bitrev_swap(Fe<P>* __restrict__ a, size_t n, int logn) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t r = brev_bits((uint32_t)i, logn);
  if (r > i) {
    uint32_t* w = reinterpret_cast<uint32_t*>(a);
    FeG<P> x = feg_load<P>(w + i * P::NG), y = feg_load<P>(w + r * P::NG);
    feg_store<P>(w + i * P::NG, y);
    feg_store<P>(w + r * P::NG, x);
  }
}

// out[brev(i)] = in[i] (out-of-place bit-reversal permutation; out != in)
template <class P>
__global__ void __launch_bounds__(256) k_bitrev_copy(const Fe<P>* __restrict__ in, Fe<P>* __restrict__ out,
                                                     size_t n, int logn) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t r = brev_bits((uint32_t)i, logn);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(in);
  feg_store<P>(reinterpret_cast<uint32_t*>(out) + r * P::NG, feg_load<P>(src + i * P::NG));
}

// a <- (a*b - c) * den[i] with an element-wise den vector (iciclegnark PolyOps)
template <class P>
__global__ void __launch_bounds__(256) k_poly_ops_vec(Fe<P>* __restrict__ a, const Fe<P>* __restrict__ b,
                                                      const Fe<P>* __restrict__ c, const Fe<P>* __restrict__ den,
                                                      size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fe<P> v = fe_sub(fe_mul(ld_fe(a, i), fe_to_internal(ld_fe(b, i))), ld_fe(c, i));
  st_fe(a, i, fe_mul(v, fe_to_internal(ld_fe(den, i))));
}

// ---------------------------------------------------------------------------
// domain (cached per context)
// ---------------------------------------------------------------------------
struct NttPass {
  int lo, t;
  void* tw_fwd;     // null if lo == 0
  void* tw_inv;
  void* tw_inv_ns;  // n^-1 * tw_inv (top pass only): folds the INTT scaling into a pass
};

// full-size element-wise tables (built on first use, n internal-form elements)
enum NttTab { TAB_G_NAT, TAB_G_BREV, TAB_GI_NAT, TAB_GI_BREV, TAB_H_POST, TAB_COUNT };

template <class C>
struct NttDomain {
  using HFr = typename C::HFr;
  using HF = host::F<HFr>;
  int logn;
  size_t n;
  std::vector<NttPass> passes;  // DIF order (high bits first)
  void* sub_fwd[NTT_TMAX + 1] = {};
  void* sub_inv[NTT_TMAX + 1] = {};
  void* tab[TAB_COUNT] = {};
  HF omega, omega_inv, ninv, g;
  std::vector<void*> allocs;
};

template <class C>
static typename NttDomain<C>::HF host_omega(int logn) {
  using HF = typename NttDomain<C>::HF;
  using HFr = typename C::HFr;
  // omega_max = g^((r-1) >> two_adicity), then square down
  HF g = host::from_u64<HFr>(C::COSET_GEN);
  uint64_t e[4];
  for (int i = 0; i < 4; i++) e[i] = HFr::P[i];
  e[0] -= 1;
  const int s = C::TWO_ADICITY;
  uint64_t q[4];
  for (int i = 0; i < 4; i++) {
    const int src = i + s / 64, off = s % 64;
    const uint64_t lo = src < 4 ? e[src] >> off : 0;
    const uint64_t hi = (off && src + 1 < 4) ? e[src + 1] << (64 - off) : 0;
    q[i] = lo | hi;
  }
  HF w = host::fpow(g, q, 4);
  for (int i = 0; i < C::TWO_ADICITY - logn; i++) w = w * w;
  return w;
}

template <class C>
static int domain_alloc(NttDomain<C>* d, size_t bytes, void** out) {
  GM_HIP(hipMalloc(out, bytes ? bytes : 16));
  d->allocs.push_back(*out);
  return GM_OK;
}

template <class HF, class Fr>
static FeG<Fr> to_dev(const HF& h) {
  FeG<Fr> r;
  static_assert(sizeof(r.w) == sizeof(h.v), "gnark layout");
  memcpy(r.w, h.v, sizeof(r.w));
  return r;
}

template <class C>
static int domain_build(gm_ctx* ctx, int logn, NttDomain<C>** out) {
  using Fr = typename C::Fr;
  using HF = typename NttDomain<C>::HF;
  using HFr = typename C::HFr;
  hipStream_t st = ctx->stream;
  auto* d = new NttDomain<C>();
  d->logn = logn;
  d->n = (size_t)1 << logn;
  d->omega = host_omega<C>(logn);
  d->omega_inv = host::finv(d->omega);
  d->ninv = host::finv(host::from_u64<HFr>(d->n));
  d->g = host::from_u64<HFr>(C::COSET_GEN);
  auto dev = [](const HF& h) { return to_dev<HF, Fr>(h); };
  int rc;
  // pass plan
  if (logn > 0) {
    int np = (logn + NTT_TMAX - 1) / NTT_TMAX;
    int rem = logn, hi_bit = logn;
    for (int p = 0; p < np; p++) {
      int t = (rem + (np - p) - 1) / (np - p);
      rem -= t;
      NttPass ps;
      ps.t = t;
      ps.lo = hi_bit - t;
      hi_bit -= t;
      ps.tw_fwd = ps.tw_inv = ps.tw_inv_ns = nullptr;
      if (ps.lo > 0) {
        size_t sz = (size_t)1 << (ps.lo + ps.t);
        // w_{N'} = omega^(n / N')
        HF wf = d->omega, wi = d->omega_inv;
        for (int i = 0; i < logn - (ps.lo + ps.t); i++) {
          wf = wf * wf;
          wi = wi * wi;
        }
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * sz, &ps.tw_fwd))) return rc;
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * sz, &ps.tw_inv))) return rc;
        const HF one = HF::one();
        hipLaunchKernelGGL(k_gen_pass_tw<Fr>, dim3(blocks_for(sz, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)ps.tw_fwd, ps.lo, ps.t, dev(wf), dev(one));
        hipLaunchKernelGGL(k_gen_pass_tw<Fr>, dim3(blocks_for(sz, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)ps.tw_inv, ps.lo, ps.t, dev(wi), dev(one));
        if (p == 0) {
          if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * sz, &ps.tw_inv_ns))) return rc;
          hipLaunchKernelGGL(k_gen_pass_tw<Fr>, dim3(blocks_for(sz, 256)), dim3(256), 0, st,
                             (Fe<Fr>*)ps.tw_inv_ns, ps.lo, ps.t, dev(wi), dev(d->ninv));
        }
      }
      d->passes.push_back(ps);
      if (!d->sub_fwd[t]) {
        HF wf = d->omega, wi = d->omega_inv;
        for (int i = 0; i < logn - t; i++) {
          wf = wf * wf;
          wi = wi * wi;
        }
        size_t cnt = (size_t)1 << (t - 1);
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * cnt, &d->sub_fwd[t]))) return rc;
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * cnt, &d->sub_inv[t]))) return rc;
        HF one = HF::one();
        hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(cnt, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)d->sub_fwd[t], cnt, dev(wf), dev(one));
        hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(cnt, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)d->sub_inv[t], cnt, dev(wi), dev(one));
      }
    }
  }
  GM_HIP(hipGetLastError());
  *out = d;
  return GM_OK;
}

// Element-wise table `which` of the domain, built on first use:
//   G_NAT[i] = g^i, G_BREV[i] = g^brev(i)                    (forward coset, on load)
//   GI_NAT[i] = g^-i / n, GI_BREV[i] = g^-brev(i) / n        (inverse coset, on store)
//   H_POST[i] = g^-brev(i) / (n (g^n - 1))                   (computeH final INTT)
template <class C>
static int domain_table(gm_ctx* ctx, NttDomain<C>* d, int which, const Fe<typename C::Fr>** out) {
  using Fr = typename C::Fr;
  using HF = typename NttDomain<C>::HF;
  if (!d->tab[which]) {
    int rc;
    if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * d->n, &d->tab[which]))) return rc;
    const HF gi = host::finv(d->g);
    HF base = d->g, mult = HF::one();
    if (which == TAB_GI_NAT || which == TAB_GI_BREV) {
      base = gi;
      mult = d->ninv;
    } else if (which == TAB_H_POST) {
      uint64_t e[1] = {d->n};
      base = gi;
      mult = d->ninv * host::finv(host::fpow(d->g, e, 1) - HF::one());
    }
    const bool brev = which == TAB_G_BREV || which == TAB_GI_BREV || which == TAB_H_POST;
    auto k = brev ? k_gen_coset<Fr, true> : k_gen_coset<Fr, false>;
    hipLaunchKernelGGL(k, dim3(blocks_for(d->n, 256)), dim3(256), 0, ctx->stream, (Fe<Fr>*)d->tab[which], d->n,
                       d->logn, to_dev<HF, Fr>(base), to_dev<HF, Fr>(mult));
    GM_HIP(hipGetLastError());
  }
  *out = (const Fe<Fr>*)d->tab[which];
  return GM_OK;
}

template <class C>
static int get_domain(gm_ctx* ctx, int logn, NttDomain<C>** out) {
  const int key = C::id * 64 + logn;
  auto it = ctx->ntt_domains.find(key);
  if (it != ctx->ntt_domains.end()) {
    *out = reinterpret_cast<NttDomain<C>*>(it->second);
    return GM_OK;
  }
  NttDomain<C>* d = nullptr;
  int rc = domain_build<C>(ctx, logn, &d);
  if (rc) return rc;
  ctx->ntt_domains[key] = d;
  *out = d;
  return GM_OK;
}

static int log2_exact(size_t n) {
  int l = 0;
  while (((size_t)1 << l) < n) l++;
  return ((size_t)1 << l) == n ? l : -1;
}

// Fused element-wise work attached to a transform (see k_ntt_pass).
template <class Fr>
struct NttFuse {
  const Fe<Fr>* pre = nullptr;   // first pass, on load
  const Fe<Fr>* post = nullptr;  // last pass, on store
  const Fe<Fr>* pb = nullptr;    // first pass, a <- a*b - c
  const Fe<Fr>* pc = nullptr;
  bool scale_ninv = false;       // inverse without coset: fold 1/n into the top pass
};

template <class C>
static int run_passes(gm_ctx* ctx, NttDomain<C>* d, Fe<typename C::Fr>* a, bool inverse, bool dit,
                      const NttFuse<typename C::Fr>& fz) {
  using Fr = typename C::Fr;
  hipStream_t st = ctx->stream;
  const size_t smem = sizeof(Fe<Fr>) * NTT_TILE;
  const int np = (int)d->passes.size();
  for (int k = 0; k < np; k++) {
    const int pi = dit ? np - 1 - k : k;
    const NttPass& ps = d->passes[pi];
    const Fe<Fr>* tw = (const Fe<Fr>*)(inverse ? ((fz.scale_ninv && pi == 0) ? ps.tw_inv_ns : ps.tw_inv)
                                               : ps.tw_fwd);
    const Fe<Fr>* sub = (const Fe<Fr>*)(inverse ? d->sub_inv[ps.t] : d->sub_fwd[ps.t]);
    const bool first = k == 0, last = k == np - 1;
    const size_t nother = d->n >> ps.t;
    const size_t B = NTT_TILE >> ps.t;
    const unsigned grid = (unsigned)((nother + B - 1) / B);
    ProfScope pscope(ctx, "ntt_pass");
    // radix-4 passes for t >= 2 with strict mad chains in the load / store products
    // (fe_mul CHAIN level 2, profiles/r05an_strict_chain_ab.txt) and growing bounds
    // in both pass kinds (r4_dif_grow / r4_dit_grow, r04g / r04af)
    if (ps.t >= 2) {
      auto k4 = dit ? k_ntt_pass4<Fr, true, 2> : k_ntt_pass4<Fr, false, 2>;
      hipLaunchKernelGGL(k4, dim3(grid), dim3(NTT_TPB), smem, st, a, d->logn, ps.lo, ps.t, 3, tw, sub,
                         first ? fz.pre : nullptr, last ? fz.post : nullptr, first ? fz.pb : nullptr,
                         first ? fz.pc : nullptr);
      continue;
    }
    auto kern = dit ? k_ntt_pass<Fr, true> : k_ntt_pass<Fr, false>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTT_TPB), smem, st, a, d->logn, ps.lo, ps.t, tw, sub,
                       first ? fz.pre : nullptr, last ? fz.post : nullptr, first ? fz.pb : nullptr,
                       first ? fz.pc : nullptr);
  }
  GM_HIP(hipGetLastError());
  return GM_OK;
}

// gnark fft.Domain semantics on n = 2^logn elements, all element-wise factors
// fused into the first / last pass.
template <class C>
static int transform(gm_ctx* ctx, NttDomain<C>* d, void* data, bool inverse, bool dit, bool coset,
                     NttFuse<typename C::Fr> fz) {
  using Fr = typename C::Fr;
  Fe<Fr>* a = reinterpret_cast<Fe<Fr>*>(data);
  int rc;
  // n = 1: every mode is the identity (w = g^0 = 1, 1/n = 1)
  if (d->logn == 0 && !fz.pb) return GM_OK;
  if (coset) {
    // forward: coefficient index of position p is p (DIF) or brev(p) (DIT);
    // inverse: output position p holds coefficient p (DIT) or brev(p) (DIF)
    const int which = inverse ? (dit ? TAB_GI_NAT : TAB_GI_BREV) : (dit ? TAB_G_BREV : TAB_G_NAT);
    if ((rc = domain_table<C>(ctx, d, which, inverse ? &fz.post : &fz.pre))) return rc;
  } else if (inverse && !fz.post) {
    fz.scale_ninv = true;
  }
  if ((rc = run_passes<C>(ctx, d, a, inverse, dit, fz))) return rc;
  if (fz.scale_ninv && d->passes[0].lo == 0) {
    // single pass (logn <= NTT_TMAX): no inter-pass twiddle to fold 1/n into
    ProfScope ps(ctx, "ntt_scale");
    hipLaunchKernelGGL(k_scale_const<Fr>, dim3(blocks_for(d->n, 256)), dim3(256), 0, ctx->stream, a, d->n,
                       to_dev<typename NttDomain<C>::HF, Fr>(d->ninv));
  }
  GM_HIP(hipGetLastError());
  return GM_OK;
}

template <class C>
int ntt_device(gm_ctx* ctx, void* data, size_t n, bool inverse, bool dit, bool coset) {
  const int logn = log2_exact(n);
  if (logn < 0 || logn > C::TWO_ADICITY || logn > 30) {
    set_error("ntt: n must be a power of two within the 2-adicity");
    return GM_ERR_INVALID;
  }
  NttDomain<C>* d;
  int rc = get_domain<C>(ctx, logn, &d);
  if (rc) return rc;
  return transform<C>(ctx, d, data, inverse, dit, coset, NttFuse<typename C::Fr>());
}

template <class C>
int poly_ops_device(gm_ctx* ctx, void* a, const void* b, const void* c, size_t n, const void* den_host) {
  using Fr = typename C::Fr;
  FeG<Fr> den;
  memcpy(den.w, den_host, sizeof(den.w));
  ProfScope ps(ctx, "poly_ops");
  hipLaunchKernelGGL(k_poly_ops<Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                     (Fe<Fr>*)a, (const Fe<Fr>*)b, (const Fe<Fr>*)c, n, den);
  GM_HIP(hipGetLastError());
  return GM_OK;
}

template <class C>
int reverse_device(gm_ctx* ctx, void* a, size_t n) {
  using Fr = typename C::Fr;
  const int logn = log2_exact(n);
  if (logn < 0) {
    set_error("reverse: n must be a power of two");
    return GM_ERR_INVALID;
  }
  ProfScope ps(ctx, "bitrev");
  hipLaunchKernelGGL(k_bitrev_swap<Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                     (Fe<Fr>*)a, n, logn);
  GM_HIP(hipGetLastError());
  return GM_OK;
}

template <class C>
int bitrev_copy_device(gm_ctx* ctx, void* out, const void* in, size_t n) {
  using Fr = typename C::Fr;
  const int logn = log2_exact(n);
  if (logn < 0 || out == in) {
    set_error("bitrev_copy: n must be a power of two and out != in");
    return GM_ERR_INVALID;
  }
  ProfScope ps(ctx, "bitrev");
  hipLaunchKernelGGL(k_bitrev_copy<Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                     (const Fe<Fr>*)in, (Fe<Fr>*)out, n, logn);
  GM_HIP(hipGetLastError());
  return GM_OK;
}

template <class C>
int poly_ops_vec_device(gm_ctx* ctx, void* a, const void* b, const void* c, const void* den, size_t n) {
  using Fr = typename C::Fr;
  ProfScope ps(ctx, "poly_ops");
  hipLaunchKernelGGL(k_poly_ops_vec<Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream, (Fe<Fr>*)a,
                     (const Fe<Fr>*)b, (const Fe<Fr>*)c, (const Fe<Fr>*)den, n);
  GM_HIP(hipGetLastError());
  return GM_OK;
}

// Builds (and caches) the domain tables of size n (GenerateTwiddleFactors).
template <class C>
int ntt_domain_prepare(gm_ctx* ctx, size_t n) {
  const int logn = log2_exact(n);
  if (logn < 0 || logn > C::TWO_ADICITY || logn > 30) {
    set_error("ntt: n must be a power of two within the 2-adicity");
    return GM_ERR_INVALID;
  }
  NttDomain<C>* d;
  return get_domain<C>(ctx, logn, &d);
}

// The domain and the two n-element tables computeH reads (coset powers g^brev(p)
// and the fused tail's factors), built ahead of the first prove -- at key upload,
// as the reference generates its twiddles in setupDevicePointers (icicle.go:68-76)
// -- instead of inside it (2^24: ~15 ms of a first prove's ~25 ms overhead,
// profiles/r05ae_first_prove.txt).
template <class C>
int compute_h_prepare(gm_ctx* ctx, size_t n) {
  const int logn = log2_exact(n);
  if (logn < 1 || logn > C::TWO_ADICITY || logn > 30) {
    set_error("compute_h: n must be a power of two >= 2 within the 2-adicity");
    return GM_ERR_INVALID;
  }
  NttDomain<C>* d;
  const Fe<typename C::Fr>* t;
  int rc;
  if ((rc = get_domain<C>(ctx, logn, &d)) || (rc = domain_table<C>(ctx, d, TAB_G_BREV, &t)) ||
      (rc = domain_table<C>(ctx, d, TAB_H_POST, &t)))
    return rc;
  return GM_OK;
}

// computeH (prove.go:356-399; icicle.go:453-513), all scalings fused:
//   a, b, c: INTT (DIF; 1/n folded into the top-pass twiddles) -> bit-reversed
//            coefficients -> coset NTT (DIT; g^brev(p) applied on load) -> natural
//            evaluations on the coset g*<w>
//   a <- a*b - c (on load of the first pass of the final transform)
//   coset INTT (DIF) with g^-brev(p) / (n (g^n - 1)) on store -> h, bit-reversed
//   (the order pk.G1.Z uses, setup.go:265-267; icicle.go:510 reverses explicitly)
template <class C>
int compute_h_device(gm_ctx* ctx, void* a, void* b, void* c, size_t len, size_t n) {
  if (len > n) {
    set_error("compute_h: len > n");
    return GM_ERR_INVALID;
  }
  const int logn = log2_exact(n);
  if (logn < 1 || logn > C::TWO_ADICITY || logn > 30) {
    set_error("compute_h: n must be a power of two >= 2 within the 2-adicity");
    return GM_ERR_INVALID;
  }
  int rc;
  for (void* v : {a, b, c})
    if ((rc = compute_h_chain<C>(ctx, v, len, n))) return rc;
  return compute_h_finish<C>(ctx, a, b, c, n);
}

// One input's chain of computeH (prove.go:372-378): pad to n, FFTInverse(DIF),
// FFT(DIT, OnCoset) -- independent per vector, so a, b, c may run on three GPUs.
template <class C>
int compute_h_chain(gm_ctx* ctx, void* v, size_t len, size_t n) {
  using Fr = typename C::Fr;
  const int logn = log2_exact(n);
  if (len > n || logn < 1 || logn > C::TWO_ADICITY || logn > 30) {
    set_error("compute_h: n must be a power of two >= 2 within the 2-adicity, len <= n");
    return GM_ERR_INVALID;
  }
  if (len < n) GM_HIP(hipMemsetAsync((char*)v + 32 * len, 0, 32 * (n - len), ctx->stream));
  NttDomain<C>* d;
  int rc;
  if ((rc = get_domain<C>(ctx, logn, &d))) return rc;
  if ((rc = transform<C>(ctx, d, v, true, false, false, NttFuse<Fr>()))) return rc;
  return transform<C>(ctx, d, v, false, true, true, NttFuse<Fr>());
}

// The tail of computeH (prove.go:380-396) on the three chained vectors:
// (a b - c) / (g^n - 1) fused into the coset FFTInverse(DIF) -> h in a.
template <class C>
int compute_h_finish(gm_ctx* ctx, void* a, const void* b, const void* c, size_t n) {
  using Fr = typename C::Fr;
  NttDomain<C>* d;
  int rc;
  if ((rc = get_domain<C>(ctx, log2_exact(n), &d))) return rc;
  NttFuse<Fr> fz;
  fz.pb = (const Fe<Fr>*)b;
  fz.pc = (const Fe<Fr>*)c;
  if ((rc = domain_table<C>(ctx, d, TAB_H_POST, &fz.post))) return rc;
  return transform<C>(ctx, d, a, true, false, false, fz);
}

#define GM_NTT_INST(C)                                                                   \
  template int ntt_device<C>(gm_ctx*, void*, size_t, bool, bool, bool);                   \
  template int poly_ops_device<C>(gm_ctx*, void*, const void*, const void*, size_t,        \
                                  const void*);                                           \
  template int reverse_device<C>(gm_ctx*, void*, size_t);                                 \
  template int compute_h_device<C>(gm_ctx*, void*, void*, void*, size_t, size_t);         \
  template int compute_h_chain<C>(gm_ctx*, void*, size_t, size_t);                         \
  template int compute_h_finish<C>(gm_ctx*, void*, const void*, const void*, size_t);      \
  template int bitrev_copy_device<C>(gm_ctx*, void*, const void*, size_t);                 \
  template int poly_ops_vec_device<C>(gm_ctx*, void*, const void*, const void*, const void*, size_t); \
  template int ntt_domain_prepare<C>(gm_ctx*, size_t);                                           \
  template int compute_h_prepare<C>(gm_ctx*, size_t);
GM_NTT_INST(CurveBN254)
GM_NTT_INST(CurveBLS12377)

void ntt_domains_free(gm_ctx* ctx) {
  for (auto& kv : ctx->ntt_domains) {
    const int curve = kv.first / 64;
    auto free_all = [&](auto* d) {
      for (void* p : d->allocs) hipFree(p);
      delete d;
    };
    if (curve == 0)
      free_all(reinterpret_cast<NttDomain<CurveBN254>*>(kv.second));
    else
      free_all(reinterpret_cast<NttDomain<CurveBLS12377>*>(kv.second));
  }
  ctx->ntt_domains.clear();
}

}  // namespace gm
