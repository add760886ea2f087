// NTT / computeH entry points (see ntt.hip).
#pragma once
#include <cstddef>
#include "curves.hpp"

struct gm_ctx;

namespace gm {
template <class C>
int ntt_device(gm_ctx* ctx, void* data, size_t n, bool inverse, bool dit, bool coset);
template <class C>
int poly_ops_device(gm_ctx* ctx, void* a, const void* b, const void* c, size_t n, const void* den_host);
template <class C>
int reverse_device(gm_ctx* ctx, void* a, size_t n);
template <class C>
int compute_h_device(gm_ctx* ctx, void* a, void* b, void* c, size_t len, size_t n);
// computeH in parts (a, b, c chains may run on different devices): the chain of
// one input (pad, FFTInverse DIF, coset FFT DIT), then the fused tail -> h in a
template <class C>
int compute_h_chain(gm_ctx* ctx, void* v, size_t len, size_t n);
template <class C>
int compute_h_finish(gm_ctx* ctx, void* a, const void* b, const void* c, size_t n);
// out[brev(i)] = in[i] (n = 2^k, out != in)
template <class C>
int bitrev_copy_device(gm_ctx* ctx, void* out, const void* in, size_t n);
// a <- (a*b - c) * den[i] (den: n device elements)
template <class C>
int poly_ops_vec_device(gm_ctx* ctx, void* a, const void* b, const void* c, const void* den, size_t n);
template <class C>
int ntt_domain_prepare(gm_ctx* ctx, size_t n);
// the domain and computeH's tables for n, ahead of the first prove (key upload)
template <class C>
int compute_h_prepare(gm_ctx* ctx, size_t n);
void ntt_domains_free(gm_ctx* ctx);
}  // namespace gm
