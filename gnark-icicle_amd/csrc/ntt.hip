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

// One pass.  sub: w_T^x for x < T/2 (T = 2^t); tw: pass twiddles (null if lo == 0).
template <class P, bool DIT>
__global__ void __launch_bounds__(NTT_TPB) k_ntt_pass(Fe<P>* __restrict__ data, int logn, int lo,
                                                      int t, const Fe<P>* __restrict__ tw,
                                                      const Fe<P>* __restrict__ sub) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Fe<P>* X = reinterpret_cast<Fe<P>*>(smem_raw);   // [T][B]
  Fe<P>* SW = X + NTT_TILE;                         // [T/2]
  const int T = 1 << t;
  const int B = NTT_TILE >> t;
  const size_t nother = (size_t)1 << (logn - t);
  const size_t o0 = (size_t)blockIdx.x * B;
  const size_t lomask = ((size_t)1 << lo) - 1;

  for (int x = threadIdx.x; x < T / 2; x += NTT_TPB) SW[x] = ld_tab(sub, x);

  // load (j, o) -> X[j*B + o]
  for (int q = threadIdx.x; q < NTT_TILE; q += NTT_TPB) {
    int j, ol;
    if (lo == 0) {
      j = q & (T - 1);
      ol = q >> t;
    } else {
      ol = q % B;
      j = q / B;
    }
    const size_t o = o0 + ol;
    if (o >= nother) continue;
    const size_t hi = o >> lo, L = o & lomask;
    const size_t addr = (hi << (lo + t)) + ((size_t)j << lo) + L;
    Fe<P> v = ld_fe(data, addr);
    if (DIT && lo > 0) v = fe_mul(v, ld_tab(tw, ((size_t)j << lo) + L));
    X[j * B + ol] = v;
  }
  __syncthreads();

  const int nbf = (T / 2) * B;
  if (!DIT) {
    for (int m = T / 2; m >= 1; m >>= 1) {
      const int step = T / (2 * m);
      for (int q = threadIdx.x; q < nbf; q += NTT_TPB) {
        const int ol = q % B, k = q / B;
        const int jj = k & (m - 1), j0 = ((k / m) * 2 * m) + jj, j1 = j0 + m;
        Fe<P> u = X[j0 * B + ol], v = X[j1 * B + ol];
        X[j0 * B + ol] = fe_add(u, v);
        X[j1 * B + ol] = fe_mul(fe_sub(u, v), SW[jj * step]);
      }
      __syncthreads();
    }
  } else {
    for (int m = 1; m < T; m <<= 1) {
      const int step = T / (2 * m);
      for (int q = threadIdx.x; q < nbf; q += NTT_TPB) {
        const int ol = q % B, k = q / B;
        const int jj = k & (m - 1), j0 = ((k / m) * 2 * m) + jj, j1 = j0 + m;
        Fe<P> u = X[j0 * B + ol];
        Fe<P> v = fe_mul(X[j1 * B + ol], SW[jj * step]);
        X[j0 * B + ol] = fe_add(u, v);
        X[j1 * B + ol] = fe_sub(u, v);
      }
      __syncthreads();
    }
  }

  for (int q = threadIdx.x; q < NTT_TILE; q += NTT_TPB) {
    int j, ol;
    if (lo == 0) {
      j = q & (T - 1);
      ol = q >> t;
    } else {
      ol = q % B;
      j = q / B;
    }
    const size_t o = o0 + ol;
    if (o >= nother) continue;
    const size_t hi = o >> lo, L = o & lomask;
    const size_t addr = (hi << (lo + t)) + ((size_t)j << lo) + L;
    Fe<P> v = X[j * B + ol];
    if (!DIT && lo > 0) v = fe_mul(v, ld_tab(tw, ((size_t)j << lo) + L));
    st_fe(data, addr, v);
  }
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
__global__ void k_gen_pass_tw(Fe<P>* __restrict__ tw, int lo, int t, FeG<P> wg) {
  const Fe<P> w = fe_to_internal(fe_unpack<P>(wg));
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t size = (size_t)1 << (lo + t);
  if (i >= size) return;
  const uint32_t j = (uint32_t)(i >> lo), L = (uint32_t)(i & (((size_t)1 << lo) - 1));
  const uint64_t e = (uint64_t)L * brev_bits(j, t);
  // e < 2^(lo+t) <= 2^32 for supported sizes
  tw[i] = fe_pow_u32(w, (uint32_t)e);
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

// a[i] *= lo[e & m] * hi[e >> s], e = i or bitrev(i)
template <class P, bool BREV>
__global__ void __launch_bounds__(256) k_scale_pow(Fe<P>* __restrict__ a, size_t n, int logn,
                                                   const Fe<P>* __restrict__ tlo,
                                                   const Fe<P>* __restrict__ thi, int s) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t e = BREV ? brev_bits((uint32_t)i, logn) : (uint32_t)i;
  Fe<P> f = fe_mul(ld_tab(tlo, e & ((1u << s) - 1)), ld_tab(thi, e >> s));
  st_fe(a, i, fe_mul(ld_fe(a, i), f));
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

// ---------------------------------------------------------------------------
// domain (cached per context)
// ---------------------------------------------------------------------------
struct NttPass {
  int lo, t;
  void* tw_fwd;  // null if lo == 0
  void* tw_inv;
};

template <class C>
struct NttDomain {
  using HFr = typename C::HFr;
  using HF = host::F<HFr>;
  int logn;
  size_t n;
  std::vector<NttPass> passes;  // DIF order (high bits first)
  void* sub_fwd[NTT_TMAX + 1] = {};
  void* sub_inv[NTT_TMAX + 1] = {};
  // coset tables: g^x (lo/hi), n^-1 g^-x (lo/hi), size 2^s and 2^(logn - s)
  int cs;
  void *g_lo, *g_hi, *gi_lo, *gi_hi;
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
static int domain_alloc(NttDomain<C>* d, size_t bytes, void** out, hipStream_t st) {
  (void)st;
  GM_HIP(hipMalloc(out, bytes ? bytes : 16));
  d->allocs.push_back(*out);
  return GM_OK;
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
  auto dev = [](const HF& h) {
    FeG<Fr> r;
    static_assert(sizeof(r.w) == sizeof(h.v), "gnark layout");
    memcpy(r.w, h.v, sizeof(r.w));
    return r;
  };
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
      ps.tw_fwd = ps.tw_inv = nullptr;
      if (ps.lo > 0) {
        size_t sz = (size_t)1 << (ps.lo + ps.t);
        // w_{N'} = omega^(n / N')
        HF wf = d->omega, wi = d->omega_inv;
        for (int i = 0; i < logn - (ps.lo + ps.t); i++) {
          wf = wf * wf;
          wi = wi * wi;
        }
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * sz, &ps.tw_fwd, st))) return rc;
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * sz, &ps.tw_inv, st))) return rc;
        hipLaunchKernelGGL(k_gen_pass_tw<Fr>, dim3(blocks_for(sz, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)ps.tw_fwd, ps.lo, ps.t, dev(wf));
        hipLaunchKernelGGL(k_gen_pass_tw<Fr>, dim3(blocks_for(sz, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)ps.tw_inv, ps.lo, ps.t, dev(wi));
      }
      d->passes.push_back(ps);
      if (!d->sub_fwd[t]) {
        HF wf = d->omega, wi = d->omega_inv;
        for (int i = 0; i < logn - t; i++) {
          wf = wf * wf;
          wi = wi * wi;
        }
        size_t cnt = (size_t)1 << (t - 1);
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * cnt, &d->sub_fwd[t], st))) return rc;
        if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * cnt, &d->sub_inv[t], st))) return rc;
        HF one = HF::one();
        hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(cnt, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)d->sub_fwd[t], cnt, dev(wf), dev(one));
        hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(cnt, 256)), dim3(256), 0, st,
                           (Fe<Fr>*)d->sub_inv[t], cnt, dev(wi), dev(one));
      }
    }
  }
  // coset tables
  d->cs = (logn + 1) / 2;
  size_t nlo = (size_t)1 << d->cs, nhi = (size_t)1 << (logn - d->cs);
  HF gi = host::finv(d->g);
  HF g_s = d->g, gi_s = gi;  // g^(2^cs)
  for (int i = 0; i < d->cs; i++) {
    g_s = g_s * g_s;
    gi_s = gi_s * gi_s;
  }
  HF one = HF::one();
  if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * nlo, &d->g_lo, st))) return rc;
  if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * nhi, &d->g_hi, st))) return rc;
  if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * nlo, &d->gi_lo, st))) return rc;
  if ((rc = domain_alloc(d, sizeof(Fe<Fr>) * nhi, &d->gi_hi, st))) return rc;
  hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(nlo, 256)), dim3(256), 0, st, (Fe<Fr>*)d->g_lo,
                     nlo, dev(d->g), dev(one));
  hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(nhi, 256)), dim3(256), 0, st, (Fe<Fr>*)d->g_hi,
                     nhi, dev(g_s), dev(one));
  hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(nlo, 256)), dim3(256), 0, st,
                     (Fe<Fr>*)d->gi_lo, nlo, dev(gi), dev(d->ninv));
  hipLaunchKernelGGL(k_gen_powers<Fr>, dim3(blocks_for(nhi, 256)), dim3(256), 0, st,
                     (Fe<Fr>*)d->gi_hi, nhi, dev(gi_s), dev(one));
  GM_HIP(hipGetLastError());
  *out = d;
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

template <class C>
static int run_passes(gm_ctx* ctx, NttDomain<C>* d, Fe<typename C::Fr>* a, bool inverse, bool dit) {
  using Fr = typename C::Fr;
  hipStream_t st = ctx->stream;
  const size_t smem = sizeof(Fe<Fr>) * (NTT_TILE + (1 << (NTT_TMAX - 1)));
  const int np = (int)d->passes.size();
  for (int k = 0; k < np; k++) {
    const NttPass& ps = dit ? d->passes[np - 1 - k] : d->passes[k];
    const Fe<Fr>* tw = (const Fe<Fr>*)(inverse ? ps.tw_inv : ps.tw_fwd);
    const Fe<Fr>* sub = (const Fe<Fr>*)(inverse ? d->sub_inv[ps.t] : d->sub_fwd[ps.t]);
    const size_t nother = d->n >> ps.t;
    const size_t B = NTT_TILE >> ps.t;
    const unsigned grid = (unsigned)((nother + B - 1) / B);
    ProfScope pscope(ctx, "ntt_pass");
    if (dit)
      hipLaunchKernelGGL((k_ntt_pass<Fr, true>), dim3(grid), dim3(NTT_TPB), smem, st, a, d->logn,
                         ps.lo, ps.t, tw, sub);
    else
      hipLaunchKernelGGL((k_ntt_pass<Fr, false>), dim3(grid), dim3(NTT_TPB), smem, st, a, d->logn,
                         ps.lo, ps.t, tw, sub);
  }
  GM_HIP(hipGetLastError());
  return GM_OK;
}

template <class C>
int ntt_device(gm_ctx* ctx, void* data, size_t n, bool inverse, bool dit, bool coset) {
  using Fr = typename C::Fr;
  const int logn = log2_exact(n);
  if (logn < 0 || logn > C::TWO_ADICITY || logn > 30) {
    set_error("ntt: n must be a power of two within the 2-adicity");
    return GM_ERR_INVALID;
  }
  NttDomain<C>* d;
  int rc = get_domain<C>(ctx, logn, &d);
  if (rc) return rc;
  hipStream_t st = ctx->stream;
  Fe<Fr>* a = reinterpret_cast<Fe<Fr>*>(data);
  const unsigned g = blocks_for(n, 256);
  if (!inverse) {
    if (coset) {
      ProfScope ps(ctx, "ntt_scale");
      if (dit)
        hipLaunchKernelGGL((k_scale_pow<Fr, true>), dim3(g), dim3(256), 0, st, a, n, logn,
                           (const Fe<Fr>*)d->g_lo, (const Fe<Fr>*)d->g_hi, d->cs);
      else
        hipLaunchKernelGGL((k_scale_pow<Fr, false>), dim3(g), dim3(256), 0, st, a, n, logn,
                           (const Fe<Fr>*)d->g_lo, (const Fe<Fr>*)d->g_hi, d->cs);
    }
    if ((rc = run_passes<C>(ctx, d, a, false, dit))) return rc;
  } else {
    if ((rc = run_passes<C>(ctx, d, a, true, dit))) return rc;
    ProfScope ps(ctx, "ntt_scale");
    if (coset) {
      // DIF output is bit-reversed: coefficient index = bitrev(i)
      if (dit)
        hipLaunchKernelGGL((k_scale_pow<Fr, false>), dim3(g), dim3(256), 0, st, a, n, logn,
                           (const Fe<Fr>*)d->gi_lo, (const Fe<Fr>*)d->gi_hi, d->cs);
      else
        hipLaunchKernelGGL((k_scale_pow<Fr, true>), dim3(g), dim3(256), 0, st, a, n, logn,
                           (const Fe<Fr>*)d->gi_lo, (const Fe<Fr>*)d->gi_hi, d->cs);
    } else {
      FeG<Fr> k;
      memcpy(k.w, d->ninv.v, sizeof(k.w));
      hipLaunchKernelGGL(k_scale_const<Fr>, dim3(g), dim3(256), 0, st, a, n, k);
    }
  }
  GM_HIP(hipGetLastError());
  return GM_OK;
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

// computeH (prove.go:356-399): INTT(DIF) -> coset NTT(DIT) for a, b, c;
// (a*b - c) * den; coset INTT(DIF) -> h bit-reversed.
template <class C>
int compute_h_device(gm_ctx* ctx, void* a, void* b, void* c, size_t len, size_t n) {
  using HFr = typename C::HFr;
  using HF = host::F<HFr>;
  if (len > n) {
    set_error("compute_h: len > n");
    return GM_ERR_INVALID;
  }
  hipStream_t st = ctx->stream;
  if (len < n) {
    for (void* v : {a, b, c}) GM_HIP(hipMemsetAsync((char*)v + 32 * len, 0, 32 * (n - len), st));
  }
  int rc;
  for (void* v : {a, b, c}) {
    if ((rc = ntt_device<C>(ctx, v, n, true, false, false))) return rc;
    if ((rc = ntt_device<C>(ctx, v, n, false, true, true))) return rc;
  }
  HF g = host::from_u64<HFr>(C::COSET_GEN);
  uint64_t e[1] = {n};
  HF den = host::finv(host::fpow(g, e, 1) - HF::one());
  if ((rc = poly_ops_device<C>(ctx, a, b, c, n, den.v))) return rc;
  return ntt_device<C>(ctx, a, n, true, false, true);
}

#define GM_NTT_INST(C)                                                                   \
  template int ntt_device<C>(gm_ctx*, void*, size_t, bool, bool, bool);                   \
  template int poly_ops_device<C>(gm_ctx*, void*, const void*, const void*, size_t,        \
                                  const void*);                                           \
  template int reverse_device<C>(gm_ctx*, void*, size_t);                                 \
  template int compute_h_device<C>(gm_ctx*, void*, void*, void*, size_t, size_t);
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
