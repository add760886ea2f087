#pragma once
#include "../../gnark-icicle_amd/csrc/field.hpp"
namespace gm {
GM_DEV void mad_cc(uint32_t a, uint32_t b, uint64_t& acc, uint32_t& hi) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
  asm("v_addc_co_u32 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(c) : "v"(hi), "s"(c));
}
GM_DEV void mad_cc_s(uint32_t a, uint32_t b_s, uint64_t& acc, uint32_t& hi) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "s"(b_s));
  asm("v_addc_co_u32 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(c) : "v"(hi), "s"(c));
}
// Finely-integrated product scanning Montgomery multiplication.
template <class P>
GM_DEV Fe<P> fe_mul_ps(const Fe<P>& a, const Fe<P>& b) {
  constexpr int N = P::N;
  uint32_t m[N];
  Fe<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint32_t hi = 0;
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k < N - 1 ? k : N - 1); i++) mad_cc(a.v[i], b.v[k - i], acc, hi);
#pragma unroll
    for (int i = (k - N + 1 > 0 ? k - N + 1 : 0); i <= (k - 1 < N - 1 ? k - 1 : N - 1); i++) mad_cc_s(m[i], P::p(k - i), acc, hi);
    if (k < N) {
      m[k] = (uint32_t)acc * P::INV;
      mad_cc_s(m[k], P::p(0), acc, hi);
    } else {
      r.v[k - N] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
  }
  r.v[N - 1] = (uint32_t)acc;
  fe_reduce_once(r);
  return r;
}
}
