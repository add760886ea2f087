// C-ABI implementation (include/gnark_mi355x.h) and the Groth16 prover
// orchestration that replaces icicle_bn254.Prove
// (backend/groth16/bn254/icicle/icicle.go:133-422), re-derived from the current
// CPU prover groth16_bn254.Prove (backend/groth16/bn254/prove.go:62-325) as
// SURVEY.md §0.3 prescribes: only the MSMs and NTTs move to the device.
#include <cstdlib>
#include <cstring>
#include <thread>
#include <string>
#include <vector>

#include "curves.hpp"
#include "msm.hpp"
#include "ntt.hpp"
#include "runtime.hpp"

namespace gm {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// ---------------------------------------------------------------------------
// synthetic-input kernels (bench / tests)
// ---------------------------------------------------------------------------
GM_DEV uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// n Montgomery (gnark-layout) scalars: random canonical value below 2^BITS,
// reduced once (2^BITS < 2r for both scalar fields), then x*Rg.
template <class Fr>
__global__ void k_random_scalars(uint32_t* out, size_t n, uint64_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t st = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
  FeG<Fr> g;
  for (int q = 0; q < Fr::NG / 2; q++) {
    uint64_t v = splitmix64(st);
    g.w[2 * q] = (uint32_t)v;
    g.w[2 * q + 1] = (uint32_t)(v >> 32);
  }
  const int top = Fr::BITS - 32 * (Fr::NG - 1);
  g.w[Fr::NG - 1] &= (top >= 32) ? 0xffffffffu : ((1u << top) - 1);
  Fe<Fr> k = fe_unpack<Fr>(g);
  fe_reduce_once(k);
  feg_store<Fr>(out + i * Fr::NG, fe_pack(fe_canonical_to_gnark(k)));
}

// gnark-layout affine point passed by value
template <class F>
struct GPoint {
  uint32_t w[2 * Coord<F>::WORDS];
};

// out[i] = [k_i] base (gnark-layout affine), double-and-add over the canonical scalar.
template <class Fr, class F>
__global__ void __launch_bounds__(128) k_batch_mul_base(const uint32_t* __restrict__ scalars,
                                                        size_t n, GPoint<F> base_g,
                                                        uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FeG<Fr> k = fe_pack(fe_gnark_to_canonical(fe_load_g<Fr>(scalars, i)));
  const Affine<F> base = load_affine_gnark<F>(base_g.w);
  XYZZ<F> acc = xyzz_inf<F>();
  for (int w = Fr::NG - 1; w >= 0; w--) {
    for (int b = 31; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      if ((k.w[w] >> b) & 1) xyzz_add_aff(acc, base);
    }
  }
  Affine<F> r;
  if (xyzz_is_inf(acc)) {
    r.x = FOps<F>::zero();
    r.y = FOps<F>::zero();
  } else {
    F t = fe_inv(fe_mul(acc.zz, acc.zzz));
    r.x = fe_mul(acc.x, fe_mul(t, acc.zzz));  // X / ZZ
    r.y = fe_mul(acc.y, fe_mul(t, acc.zz));   // Y / ZZZ
  }
  store_affine_gnark<F>(out + i * 2 * Coord<F>::WORDS, r);
}

// dst[i] = src[idx[i]] (Fr, 32 bytes) -- device-side scalar compaction
__global__ void k_gather_fr(const uint4* __restrict__ src, const uint32_t* __restrict__ idx, size_t n,
                            uint4* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t j = idx[i];
  dst[2 * i] = src[2 * j];
  dst[2 * i + 1] = src[2 * j + 1];
}

// ---------------------------------------------------------------------------
// dispatch helpers
// ---------------------------------------------------------------------------
template <class C, bool G2>
static int msm_to_host(gm_ctx* ctx, const void* sc, const void* pts, size_t n, void* out_jac,
                       void* out_aff) {
  using HF = typename GroupSel<C, G2>::HF;
  HF j[3];
  int rc = msm_device<C, G2>(ctx, sc, pts, n, j);
  if (rc) return rc;
  if (out_jac) memcpy(out_jac, j, sizeof(j));
  if (out_aff) {
    host::Aff<HF> a = host::to_aff(host::Jac<HF>{j[0], j[1], j[2]});
    memcpy(out_aff, &a, sizeof(a));
  }
  return GM_OK;
}

static int check_curve(int curve) {
  if (curve != GM_BN254 && curve != GM_BLS12_377) {
    set_error("unknown curve id");
    return GM_ERR_INVALID;
  }
  return GM_OK;
}

static size_t fp_bytes(int curve) { return curve == GM_BN254 ? 32 : 48; }

}  // namespace gm

using namespace gm;

// ===========================================================================
// Groth16 proving key on device
// ===========================================================================
struct gm_g16_pk {
  int curve;
  size_t n, nb_wires, nb_public, nbA, nbB, nbK;
  void *A, *B, *Z, *K, *B2;       // device point arrays
  void *idxA, *idxB, *idxK;       // device index maps (compaction)
  size_t zlo = 0, nbZ = 0;        // this shard's slice of h / pk.G1.Z (whole: 0, n-1)
  bool precomp = false;           // GM_PK_PRECOMPUTE: fixed-base window copies
  MsmPrecomp preA, preB, preZ, preK;  // layouts (B and B2 share preB)
  std::vector<uint8_t> alpha, beta, delta, beta2, delta2;  // host affine
};

extern "C" {

const char* gm_last_error(void) { return g_last_error.c_str(); }
int gm_version(void) { return 1; }

int gm_init(int device, gm_ctx** out) {
  if (!out) return GM_ERR_INVALID;
  int ndev = 0;
  GM_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("gm_init: device index out of range");
    return GM_ERR_INVALID;
  }
  GM_HIP(hipSetDevice(device));
  auto* c = new gm_ctx();
  c->device = device;
  // GM_MSM_SLICE: entries per thread in the bucket accumulation (tuning; default 64)
  if (const char* sl = getenv("GM_MSM_SLICE")) c->msm_slice = atoi(sl) > 0 ? atoi(sl) : 0;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking);
  if (e != hipSuccess) {
    set_error(std::string("hipStreamCreate: ") + hipGetErrorString(e));
    delete c;
    return GM_ERR_DEVICE;
  }
  *out = c;
  return GM_OK;
}

int gm_destroy(gm_ctx* ctx) {
  if (!ctx) return GM_OK;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  if (ctx->aux) hipStreamSynchronize(ctx->aux);
  ntt_domains_free(ctx);
  for (auto& ch : ctx->chunks) hipFree(ch.base);
  ctx->chunks.clear();
  for (auto e : ctx->event_pool) hipEventDestroy(e);
  for (auto& p : ctx->pending) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  hipStreamDestroy(ctx->stream);
  if (ctx->aux) hipStreamDestroy(ctx->aux);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  delete ctx;
  return GM_OK;
}

int gm_synchronize(gm_ctx* ctx) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

int gm_profile_enable(gm_ctx* ctx, int on) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  ctx->profiling = on != 0;
  return GM_OK;
}
int gm_profile_reset(gm_ctx* ctx) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  ctx->stats.clear();
  return GM_OK;
}
int gm_profile_get(gm_ctx* ctx, const char* name, double* total_ms, uint64_t* count) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  auto it = ctx->stats.find(name);
  if (it == ctx->stats.end()) {
    *total_ms = 0;
    *count = 0;
    return GM_OK;
  }
  *total_ms = it->second.total_ms;
  *count = it->second.count;
  return GM_OK;
}
int gm_profile_dump(gm_ctx* ctx, char* buf, size_t cap) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  hipStreamSynchronize(ctx->stream);
  prof_collect(ctx);
  std::string s;
  for (auto& kv : ctx->stats)
    s += kv.first + " " + std::to_string(kv.second.total_ms) + " " + std::to_string(kv.second.count) + "\n";
  if (cap) {
    size_t m = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), m);
    buf[m] = 0;
  }
  return GM_OK;
}
int gm_set_msm_window(gm_ctx* ctx, int c) {
  if (c != 0 && (c < 2 || c > 24)) return GM_ERR_INVALID;
  ctx->msm_c_override = c;
  return GM_OK;
}

// ---- memory -----------------------------------------------------------------
int gm_malloc(gm_ctx* ctx, size_t bytes, void** dev_out) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  hipError_t e = hipMalloc(dev_out, bytes ? bytes : 16);
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  return GM_OK;
}
int gm_free(gm_ctx* ctx, void* dev) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  GM_HIP(hipFree(dev));
  return GM_OK;
}
int gm_memcpy_h2d(gm_ctx* ctx, void* dev, const void* host, size_t bytes) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
int gm_memcpy_d2h(gm_ctx* ctx, void* host, const void* dev, size_t bytes) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
int gm_memcpy_d2d(gm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
int gm_copy_to_device(gm_ctx* ctx, const void* host, size_t bytes, void** dev_out) {
  int rc = gm_malloc(ctx, bytes, dev_out);
  if (rc) return rc;
  return gm_memcpy_h2d(ctx, *dev_out, host, bytes);
}
int gm_copy_points_to_device(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n,
                             void** dev_out) {
  if (int rc = check_curve(curve)) return rc;
  return gm_copy_to_device(ctx, host_points, n * fp_bytes(curve) * (g2 ? 4 : 2), dev_out);
}

// ---- MSM ------------------------------------------------------------------------
int gm_msm(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* points_dev,
           size_t n, void* out_jac, void* out_affine) {
  if (!ctx) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  if (curve == GM_BN254)
    rc = g2 ? msm_to_host<CurveBN254, true>(ctx, scalars_dev, points_dev, n, out_jac, out_affine)
            : msm_to_host<CurveBN254, false>(ctx, scalars_dev, points_dev, n, out_jac, out_affine);
  else
    rc = g2 ? msm_to_host<CurveBLS12377, true>(ctx, scalars_dev, points_dev, n, out_jac, out_affine)
            : msm_to_host<CurveBLS12377, false>(ctx, scalars_dev, points_dev, n, out_jac, out_affine);
  prof_collect(ctx);
  return rc;
}

int gm_msm_host_scalars(gm_ctx* ctx, int curve, int g2, const void* scalars_host,
                        const void* points_dev, size_t n, void* out_jac, void* out_affine) {
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  Arena arena(ctx);
  DevBuf s;
  int rc;
  if ((rc = s.alloc(arena, 32 * n))) return rc;
  GM_HIP(hipMemcpyAsync(s.p, scalars_host, 32 * n, hipMemcpyHostToDevice, ctx->stream));
  return gm_msm(ctx, curve, g2, s.p, points_dev, n, out_jac, out_affine);
}

int gm_points_upload(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n, void** out) {
  if (!ctx || !out) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  const size_t gb = fp_bytes(curve) * (g2 ? 4 : 2) * n;
  const size_t ib = n * (curve == GM_BN254 ? (g2 ? msm_internal_point_bytes<CurveBN254, true>()
                                                 : msm_internal_point_bytes<CurveBN254, false>())
                                           : (g2 ? msm_internal_point_bytes<CurveBLS12377, true>()
                                                 : msm_internal_point_bytes<CurveBLS12377, false>()));
  Arena arena(ctx);
  DevBuf tmp;
  int rc;
  if ((rc = tmp.alloc(arena, gb))) return rc;
  hipError_t e = hipMalloc(out, ib ? ib : 16);
  if (e != hipSuccess) {
    set_error(std::string("gm_points_upload hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  GM_HIP(hipMemcpyAsync(tmp.p, host_points, gb, hipMemcpyHostToDevice, ctx->stream));
  if (curve == GM_BN254)
    rc = g2 ? msm_prepare_points<CurveBN254, true>(ctx, tmp.p, n, *out)
            : msm_prepare_points<CurveBN254, false>(ctx, tmp.p, n, *out);
  else
    rc = g2 ? msm_prepare_points<CurveBLS12377, true>(ctx, tmp.p, n, *out)
            : msm_prepare_points<CurveBLS12377, false>(ctx, tmp.p, n, *out);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}

extern "C++" {
template <class C, bool G2>
static int msm_prepared_t(gm_ctx* ctx, const void* sc, const void* pts, size_t n, void* out_jac, void* out_aff,
                          const MsmPrecomp* pre = nullptr) {
  using HF = typename GroupSel<C, G2>::HF;
  HF j[3];
  int rc = msm_device<C, G2>(ctx, sc, pts, n, j, true, pre);
  if (rc) return rc;
  if (out_jac) memcpy(out_jac, j, sizeof(j));
  if (out_aff) {
    host::Aff<HF> a = host::to_aff(host::Jac<HF>{j[0], j[1], j[2]});
    memcpy(out_aff, &a, sizeof(a));
  }
  return GM_OK;
}
}  // extern "C++"

int gm_msm_prepared(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* prepared, size_t n,
                    void* out_jac, void* out_affine) {
  if (!ctx) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  if (curve == GM_BN254)
    rc = g2 ? msm_prepared_t<CurveBN254, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine)
            : msm_prepared_t<CurveBN254, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine);
  else
    rc = g2 ? msm_prepared_t<CurveBLS12377, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine)
            : msm_prepared_t<CurveBLS12377, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine);
  prof_collect(ctx);
  return rc;
}

// ---- fixed-base precomputed point sets -------------------------------------------
static int make_precomp(int curve, size_t n, int window, MsmPrecomp* out) {
  const int bits = curve == GM_BN254 ? CurveBN254::FR_BITS : CurveBLS12377::FR_BITS;
  if (window == 0) {
    *out = msm_choose_precomp(n, bits);
    return GM_OK;
  }
  if (window < 2 || window > 24) {
    set_error("precompute: window must be 0 (auto) or in [2, 24]");
    return GM_ERR_INVALID;
  }
  out->c = (uint32_t)window;
  out->W = (uint32_t)((bits + 1 + window - 1) / window);
  out->stride = n;
  return GM_OK;
}

int gm_precompute_layout(int curve, size_t n, int window, int* c_out, int* copies_out) {
  if (int rc = check_curve(curve)) return rc;
  MsmPrecomp p;
  if (int rc = make_precomp(curve, n, window, &p)) return rc;
  if (c_out) *c_out = (int)p.c;
  if (copies_out) *copies_out = (int)p.W;
  return GM_OK;
}

int gm_points_upload_precomputed(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n, int window,
                                 void** out) {
  if (!ctx || !out) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  MsmPrecomp pre;
  if (int rc = make_precomp(curve, n, window, &pre)) return rc;
  if ((size_t)pre.W * n >= (size_t(1) << 31)) {
    set_error("precompute: copies * n must be < 2^31");
    return GM_ERR_INVALID;
  }
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  const size_t gb = fp_bytes(curve) * (g2 ? 4 : 2) * n;
  const size_t ib = (size_t)pre.W * n *
                    (curve == GM_BN254 ? (g2 ? msm_internal_point_bytes<CurveBN254, true>()
                                             : msm_internal_point_bytes<CurveBN254, false>())
                                       : (g2 ? msm_internal_point_bytes<CurveBLS12377, true>()
                                             : msm_internal_point_bytes<CurveBLS12377, false>()));
  Arena arena(ctx);
  DevBuf tmp;
  int rc;
  if ((rc = tmp.alloc(arena, gb ? gb : 16))) return rc;
  hipError_t e = hipMalloc(out, ib ? ib : 16);
  if (e != hipSuccess) {
    set_error(std::string("gm_points_upload_precomputed hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  if (gb) GM_HIP(hipMemcpyAsync(tmp.p, host_points, gb, hipMemcpyHostToDevice, ctx->stream));
  if (curve == GM_BN254)
    rc = g2 ? msm_precompute_points<CurveBN254, true>(ctx, tmp.p, n, pre, *out)
            : msm_precompute_points<CurveBN254, false>(ctx, tmp.p, n, pre, *out);
  else
    rc = g2 ? msm_precompute_points<CurveBLS12377, true>(ctx, tmp.p, n, pre, *out)
            : msm_precompute_points<CurveBLS12377, false>(ctx, tmp.p, n, pre, *out);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}

int gm_msm_precomputed(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* prepared,
                       size_t prepared_n, int window, size_t n, void* out_jac, void* out_affine) {
  if (!ctx) return GM_ERR_INVALID;
  if (int rc = check_curve(curve)) return rc;
  if (n > prepared_n) {
    set_error("msm_precomputed: n exceeds the prepared point count");
    return GM_ERR_INVALID;
  }
  MsmPrecomp pre;
  if (int rc = make_precomp(curve, prepared_n, window, &pre)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc;
  if (curve == GM_BN254)
    rc = g2 ? msm_prepared_t<CurveBN254, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre)
            : msm_prepared_t<CurveBN254, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre);
  else
    rc = g2 ? msm_prepared_t<CurveBLS12377, true>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre)
            : msm_prepared_t<CurveBLS12377, false>(ctx, scalars_dev, prepared, n, out_jac, out_affine, &pre);
  prof_collect(ctx);
  return rc;
}

int gm_kzg_commit(gm_ctx* ctx, int curve, const void* srs, size_t srs_len, const void* coeffs_host, size_t n,
                  void* digest_affine) {
  if (!ctx || !digest_affine) return GM_ERR_INVALID;
  if (n > srs_len) {
    set_error("kzg commit: polynomial larger than the SRS");
    return GM_ERR_INVALID;
  }
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  Arena arena(ctx);
  DevBuf s;
  int rc;
  if ((rc = s.alloc(arena, 32 * (n ? n : 1)))) return rc;
  if (n) GM_HIP(hipMemcpyAsync(s.p, coeffs_host, 32 * n, hipMemcpyHostToDevice, ctx->stream));
  return gm_msm_prepared(ctx, curve, 0, s.p, srs, n, nullptr, digest_affine);
}

// ---- NTT --------------------------------------------------------------------------
int gm_ntt(gm_ctx* ctx, int curve, void* data_dev, size_t n, int inverse, int dit, int coset) {
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? ntt_device<CurveBN254>(ctx, data_dev, n, inverse, dit, coset)
                             : ntt_device<CurveBLS12377>(ctx, data_dev, n, inverse, dit, coset);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}
int gm_poly_ops(gm_ctx* ctx, int curve, void* a, const void* b, const void* c, size_t n,
                const void* den_host) {
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? poly_ops_device<CurveBN254>(ctx, a, b, c, n, den_host)
                             : poly_ops_device<CurveBLS12377>(ctx, a, b, c, n, den_host);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}
int gm_reverse_scalars(gm_ctx* ctx, int curve, void* data_dev, size_t n) {
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? reverse_device<CurveBN254>(ctx, data_dev, n)
                             : reverse_device<CurveBLS12377>(ctx, data_dev, n);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}
int gm_groth16_compute_h(gm_ctx* ctx, int curve, void* a, void* b, void* c, size_t len, size_t n) {
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? compute_h_device<CurveBN254>(ctx, a, b, c, len, n)
                             : compute_h_device<CurveBLS12377>(ctx, a, b, c, len, n);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

// ---- host group helpers ---------------------------------------------------------------
extern "C++" {
template <class HF>
static void jac_add_t(const void* p, const void* q, void* out) {
  host::Jac<HF> a, b;
  memcpy(&a, p, sizeof(a));
  memcpy(&b, q, sizeof(b));
  host::Jac<HF> r = host::jadd(a, b);
  memcpy(out, &r, sizeof(r));
}
template <class HF>
static void jac_aff_t(const void* p, void* out) {
  host::Jac<HF> a;
  memcpy(&a, p, sizeof(a));
  host::Aff<HF> r = host::to_aff(a);
  memcpy(out, &r, sizeof(r));
}
}  // extern "C++"

int gm_jac_add(int curve, int g2, const void* p, const void* q, void* out) {
  if (int rc = check_curve(curve)) return rc;
  if (curve == GM_BN254)
    g2 ? jac_add_t<CurveBN254::HG2F>(p, q, out) : jac_add_t<CurveBN254::HG1F>(p, q, out);
  else
    g2 ? jac_add_t<CurveBLS12377::HG2F>(p, q, out) : jac_add_t<CurveBLS12377::HG1F>(p, q, out);
  return GM_OK;
}
int gm_jac_to_affine(int curve, int g2, const void* p, void* out) {
  if (int rc = check_curve(curve)) return rc;
  if (curve == GM_BN254)
    g2 ? jac_aff_t<CurveBN254::HG2F>(p, out) : jac_aff_t<CurveBN254::HG1F>(p, out);
  else
    g2 ? jac_aff_t<CurveBLS12377::HG2F>(p, out) : jac_aff_t<CurveBLS12377::HG1F>(p, out);
  return GM_OK;
}

// ---- synthetic inputs -------------------------------------------------------------------
static const uint64_t GEN_BN_G1[] = GM_BN254_G1_GEN64;
static const uint64_t GEN_BN_G2[] = GM_BN254_G2_GEN64;
static const uint64_t GEN_BLS_G1[] = GM_BLS12377_G1_GEN64;
static const uint64_t GEN_BLS_G2[] = GM_BLS12377_G2_GEN64;

int gm_generator(int curve, int g2, void* out) {
  if (int rc = check_curve(curve)) return rc;
  const uint64_t* src = curve == GM_BN254 ? (g2 ? GEN_BN_G2 : GEN_BN_G1) : (g2 ? GEN_BLS_G2 : GEN_BLS_G1);
  memcpy(out, src, fp_bytes(curve) * (g2 ? 4 : 2));
  return GM_OK;
}

int gm_random_scalars(gm_ctx* ctx, int curve, uint64_t seed, size_t n, void* scalars_dev) {
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  if (curve == GM_BN254)
    hipLaunchKernelGGL(k_random_scalars<Bn254Fr>, dim3(blocks_for(n, 256)), dim3(256), 0, ctx->stream,
                       (uint32_t*)scalars_dev, n, seed);
  else
    hipLaunchKernelGGL(k_random_scalars<Bls377Fr>, dim3(blocks_for(n, 256)), dim3(256), 0,
                       ctx->stream, (uint32_t*)scalars_dev, n, seed);
  GM_HIP(hipGetLastError());
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}

extern "C++" {
template <class C, bool G2>
static int batch_mul_t(gm_ctx* ctx, const void* base, const void* sc, size_t n, void* out) {
  using DF = typename GroupSel<C, G2>::DF;
  GPoint<DF> b;
  memcpy(&b, base, sizeof(b));
  hipLaunchKernelGGL((k_batch_mul_base<typename C::Fr, DF>), dim3(blocks_for(n, 128)), dim3(128), 0,
                     ctx->stream, (const uint32_t*)sc, n, b, (uint32_t*)out);
  GM_HIP(hipGetLastError());
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
}  // extern "C++"

int gm_batch_mul_base(gm_ctx* ctx, int curve, int g2, const void* base, const void* sc, size_t n,
                      void* out) {
  if (int rc = check_curve(curve)) return rc;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  if (curve == GM_BN254)
    return g2 ? batch_mul_t<CurveBN254, true>(ctx, base, sc, n, out)
              : batch_mul_t<CurveBN254, false>(ctx, base, sc, n, out);
  return g2 ? batch_mul_t<CurveBLS12377, true>(ctx, base, sc, n, out)
            : batch_mul_t<CurveBLS12377, false>(ctx, base, sc, n, out);
}

// ---- Groth16 ------------------------------------------------------------------------------
int gm_g16_pk_upload(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, gm_g16_pk** out) {
  return gm_g16_pk_upload_ex(ctx, curve, h, 0u, out);
}

int gm_g16_pk_upload_ex(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, gm_g16_pk** out) {
  return gm_g16_pk_upload_shard(ctx, curve, h, flags, 0, 1, out);
}

// [lo, hi) of rank's contiguous shard of n items (gnark_mi355x.shard_range)
static void shard_of(size_t n, int rank, int world, size_t* lo, size_t* hi) {
  const size_t q = n / (size_t)world, r = n % (size_t)world;
  *lo = (size_t)rank * q + std::min((size_t)rank, r);
  *hi = *lo + q + ((size_t)rank < r ? 1 : 0);
}

int gm_g16_pk_upload_shard(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, int rank, int world,
                           gm_g16_pk** out) {
  if (int rc = check_curve(curve)) return rc;
  if (flags & ~(unsigned)GM_PK_PRECOMPUTE) {
    set_error("pk upload: unknown flags");
    return GM_ERR_INVALID;
  }
  if (!h || !out || h->domain_size < 2) return GM_ERR_INVALID;
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("pk upload: bad rank / world");
    return GM_ERR_INVALID;
  }
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  auto* pk = new gm_g16_pk();
  pk->curve = curve;
  pk->n = h->domain_size;
  pk->nb_wires = h->nb_wires;
  pk->nb_public = h->nb_public;
  size_t loA, hiA, loB, hiB, loK, hiK, loZ, hiZ;
  shard_of(h->nbA, rank, world, &loA, &hiA);
  shard_of(h->nbB, rank, world, &loB, &hiB);
  shard_of(h->nbK, rank, world, &loK, &hiK);
  shard_of(pk->n - 1, rank, world, &loZ, &hiZ);
  pk->nbA = hiA - loA;
  pk->nbB = hiB - loB;
  pk->nbK = hiK - loK;
  pk->zlo = loZ;
  pk->nbZ = hiZ - loZ;
  pk->precomp = (flags & GM_PK_PRECOMPUTE) != 0;
  const int frbits = curve == GM_BN254 ? CurveBN254::FR_BITS : CurveBLS12377::FR_BITS;
  if (pk->precomp) {
    pk->preA = msm_choose_precomp(pk->nbA, frbits);
    pk->preB = msm_choose_precomp(pk->nbB, frbits);
    pk->preZ = msm_choose_precomp(pk->nbZ, frbits);
    pk->preK = msm_choose_precomp(pk->nbK, frbits);
  }
  const size_t g1b = 2 * fp_bytes(curve), g2b = 4 * fp_bytes(curve);
  auto up = [&](const void* src, size_t bytes, void** dst) -> int {
    hipError_t e = hipMalloc(dst, bytes ? bytes : 16);
    if (e != hipSuccess) {
      set_error(std::string("pk upload hipMalloc: ") + hipGetErrorString(e));
      return GM_ERR_OOM;
    }
    if (bytes) {
      e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        set_error(std::string("pk upload hipMemcpy: ") + hipGetErrorString(e));
        return GM_ERR_DEVICE;
      }
    }
    return GM_OK;
  };
  int rc;
  // upload gnark-layout points, convert once into the device-internal layout
  // (radix-2^29 Montgomery) the MSM kernels consume (setupDevicePointers).
  // (with GM_PK_PRECOMPUTE also the W-1 window-shifted copies, msm_precompute_points)
  auto up_pts = [&](const void* src, size_t count, bool g2, const MsmPrecomp& pre, void** dst) -> int {
    void* tmp = nullptr;
    int r = up(src, (g2 ? g2b : g1b) * count, &tmp);
    if (r) return r;
    size_t ib = 0;
    if (curve == GM_BN254) ib = g2 ? msm_internal_point_bytes<CurveBN254, true>() : msm_internal_point_bytes<CurveBN254, false>();
    else ib = g2 ? msm_internal_point_bytes<CurveBLS12377, true>() : msm_internal_point_bytes<CurveBLS12377, false>();
    const size_t copies = pk->precomp ? pre.W : 1;
    hipError_t e = hipMalloc(dst, ib * (count ? count * copies : 1));
    if (e != hipSuccess) {
      hipFree(tmp);
      set_error(std::string("pk upload hipMalloc: ") + hipGetErrorString(e));
      return GM_ERR_OOM;
    }
    if (pk->precomp) {
      if (curve == GM_BN254)
        r = g2 ? msm_precompute_points<CurveBN254, true>(ctx, tmp, count, pre, *dst)
               : msm_precompute_points<CurveBN254, false>(ctx, tmp, count, pre, *dst);
      else
        r = g2 ? msm_precompute_points<CurveBLS12377, true>(ctx, tmp, count, pre, *dst)
               : msm_precompute_points<CurveBLS12377, false>(ctx, tmp, count, pre, *dst);
    } else if (curve == GM_BN254) {
      r = g2 ? msm_prepare_points<CurveBN254, true>(ctx, tmp, count, *dst)
             : msm_prepare_points<CurveBN254, false>(ctx, tmp, count, *dst);
    } else {
      r = g2 ? msm_prepare_points<CurveBLS12377, true>(ctx, tmp, count, *dst)
             : msm_prepare_points<CurveBLS12377, false>(ctx, tmp, count, *dst);
    }
    hipStreamSynchronize(ctx->stream);
    hipFree(tmp);
    return r;
  };
  auto fail = [&](int code) {
    for (void* q : {pk->A, pk->B, pk->Z, pk->K, pk->B2, pk->idxA, pk->idxB, pk->idxK})
      if (q) hipFree(q);
    delete pk;
    return code;
  };
  // point arrays: the caller passes this shard's slice (first point = index lo)
  if ((rc = up_pts(h->g1_A, pk->nbA, false, pk->preA, &pk->A)) ||
      (rc = up_pts(h->g1_B, pk->nbB, false, pk->preB, &pk->B)) ||
      (rc = up_pts(h->g1_Z, pk->nbZ, false, pk->preZ, &pk->Z)) ||
      (rc = up_pts(h->g1_K, pk->nbK, false, pk->preK, &pk->K)) ||
      (rc = up_pts(h->g2_B, pk->nbB, true, pk->preB, &pk->B2)))
    return fail(rc);
  // compaction maps (prove.go:157-178: drop wire i when InfinityA[i] / InfinityB[i])
  std::vector<uint32_t> ia, ib, ik;
  for (size_t i = 0; i < pk->nb_wires; i++) {
    if (!h->infA[i]) ia.push_back((uint32_t)i);
    if (!h->infB[i]) ib.push_back((uint32_t)i);
  }
  for (size_t i = 0; i < h->nbK; i++) {
    const size_t w = h->k_wires ? (size_t)h->k_wires[i] : pk->nb_public + i;
    if (w >= pk->nb_wires || w < pk->nb_public) {
      set_error("pk upload: K wire index out of range");
      return fail(GM_ERR_INVALID);
    }
    ik.push_back((uint32_t)w);
  }
  if (ia.size() != h->nbA || ib.size() != h->nbB || pk->nb_public + h->nbK > pk->nb_wires) {
    set_error("pk upload: infinity masks inconsistent with nbA/nbB/nbK");
    return fail(GM_ERR_INVALID);
  }
  // this shard's slices of the compaction maps
  if ((rc = up(ia.data() + loA, 4 * pk->nbA, &pk->idxA)) || (rc = up(ib.data() + loB, 4 * pk->nbB, &pk->idxB)) ||
      (rc = up(ik.data() + loK, 4 * pk->nbK, &pk->idxK)))
    return fail(rc);
  auto cp = [](std::vector<uint8_t>& v, const void* s, size_t b) {
    v.resize(b);
    memcpy(v.data(), s, b);
  };
  cp(pk->alpha, h->g1_alpha, g1b);
  cp(pk->beta, h->g1_beta, g1b);
  cp(pk->delta, h->g1_delta, g1b);
  cp(pk->beta2, h->g2_beta, g2b);
  cp(pk->delta2, h->g2_delta, g2b);
  *out = pk;
  return GM_OK;
}

int gm_g16_pk_free(gm_ctx* ctx, gm_g16_pk* pk) {
  if (!pk) return GM_OK;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  for (void* p : {pk->A, pk->B, pk->Z, pk->K, pk->B2, pk->idxA, pk->idxB, pk->idxK})
    if (p) hipFree(p);
  delete pk;
  return GM_OK;
}

extern "C++" {
// computeH on the context's auxiliary stream, after everything already queued
// on the main stream (the caller's a, b, c uploads).  The NTT passes overlap the
// A, B and K MSMs, whose sorts, reductions and host round trips leave the VALUs
// idle; wait() makes the main stream wait for h before the Z MSM.  The
// destructor drains the auxiliary stream on every exit path.
struct AuxComputeH {
  gm_ctx* ctx;
  hipEvent_t ev_in = nullptr, ev_h = nullptr;
  explicit AuxComputeH(gm_ctx* c) : ctx(c) {}
  template <class C>
  int start(void* a, void* b, void* c, size_t nc, size_t n) {
    // GM_G16_OVERLAP=0: computeH in order on the main stream (A/B measurements)
    static const bool overlap = !getenv("GM_G16_OVERLAP") || atoi(getenv("GM_G16_OVERLAP")) != 0;
    if (!overlap) return compute_h_device<C>(ctx, a, b, c, nc, n);
    GM_HIP(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    GM_HIP(hipEventCreateWithFlags(&ev_h, hipEventDisableTiming));
    GM_HIP(hipEventRecord(ev_in, ctx->stream));
    GM_HIP(hipStreamWaitEvent(ctx->aux, ev_in, 0));
    hipStream_t main = ctx->stream;
    ctx->stream = ctx->aux;
    int rc = compute_h_device<C>(ctx, a, b, c, nc, n);
    ctx->stream = main;
    if (rc) return rc;
    GM_HIP(hipEventRecord(ev_h, ctx->aux));
    return GM_OK;
  }
  int wait() {
    if (ev_h) GM_HIP(hipStreamWaitEvent(ctx->stream, ev_h, 0));
    return GM_OK;
  }
  ~AuxComputeH() {
    hipStreamSynchronize(ctx->aux);
    if (ev_in) hipEventDestroy(ev_in);
    if (ev_h) hipEventDestroy(ev_h);
  }
};
}  // extern "C++"

extern "C++" {
template <class C>
static int g16_prove_t(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a, void* b,
                       void* c, size_t nc, const void* r_mont, const void* s_mont, void* ar_out,
                       void* bs_out, void* krs_out) {
  using HF1 = typename C::HG1F;
  using HF2 = typename C::HG2F;
  using HFr = typename C::HFr;
  using J1 = host::Jac<HF1>;
  using J2 = host::Jac<HF2>;
  hipStream_t st = ctx->stream;
  const size_t n = pk->n;
  int rc;

  // device-side scalar compaction (icicle.go:231-278 do this on the host + H2D)
  Arena arena(ctx);
  DevBuf wA, wB, wK;
  if ((rc = wA.alloc(arena, 32 * pk->nbA)) || (rc = wB.alloc(arena, 32 * pk->nbB)) ||
      (rc = wK.alloc(arena, 32 * pk->nbK)))
    return rc;
  {
    ProfScope ps(ctx, "gather_scalars");
    hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(pk->nbA, 256)), dim3(256), 0, st,
                       (const uint4*)wires_dev, (const uint32_t*)pk->idxA, pk->nbA, (uint4*)wA.p);
    hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(pk->nbB, 256)), dim3(256), 0, st,
                       (const uint4*)wires_dev, (const uint32_t*)pk->idxB, pk->nbB, (uint4*)wB.p);
    hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(pk->nbK, 256)), dim3(256), 0, st,
                       (const uint4*)wires_dev, (const uint32_t*)pk->idxK, pk->nbK, (uint4*)wK.p);
  }
  GM_HIP(hipGetLastError());
  // r, s, kr = -rs; deltas (icicle.go:280-295)
  host::F<HFr> r, s;
  memcpy(r.v, r_mont, 32);
  memcpy(s.v, s_mont, 32);
  host::F<HFr> kr = -(r * s);
  host::F<HFr> rc_ = host::from_mont(r), sc_ = host::from_mont(s), krc = host::from_mont(kr);
  host::Aff<HF1> alpha, beta, delta;
  memcpy(&alpha, pk->alpha.data(), sizeof(alpha));
  memcpy(&beta, pk->beta.data(), sizeof(beta));
  memcpy(&delta, pk->delta.data(), sizeof(delta));
  // [r]delta, [s]delta, [kr]delta (BatchScalarMultiplicationG1, prove.go:195) and
  // [s]delta2 do not depend on the device results: computed on a host thread
  // while the GPU runs computeH and the MSMs.
  J1 dj = host::to_jac(delta);
  host::Aff<HF2> beta2, delta2;
  memcpy(&beta2, pk->beta2.data(), sizeof(beta2));
  memcpy(&delta2, pk->delta2.data(), sizeof(delta2));
  J1 d0, d1, d2;
  J2 sd2;
  std::thread deltas([&] {
    d0 = host::jmul(dj, rc_.v, 4);
    d1 = host::jmul(dj, sc_.v, 4);
    d2 = host::jmul(dj, krc.v, 4);
    sd2 = host::jmul(host::to_jac(delta2), sc_.v, 4);
  });
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } joiner{deltas};
  // H (computeH, icicle.go:453-513 / prove.go:356-399) -> bit-reversed h in `a`,
  // on the auxiliary stream, overlapped with the A, B and K MSMs
  AuxComputeH hjob(ctx);
  if ((rc = hjob.start<C>(a, b, c, nc, n))) return rc;
  HF1 t1[3];
  const MsmPrecomp* pA = pk->precomp ? &pk->preA : nullptr;
  const MsmPrecomp* pB = pk->precomp ? &pk->preB : nullptr;
  const MsmPrecomp* pK = pk->precomp ? &pk->preK : nullptr;
  const MsmPrecomp* pZ = pk->precomp ? &pk->preZ : nullptr;
  // MSM results are combined below only after the delta thread has finished
  if ((rc = msm_device<C, false>(ctx, wA.p, pk->A, pk->nbA, t1, true, pA))) return rc;
  deltas.join();
  // Ar = MSM(wA, A) + alpha + r delta   (computeAR1 icicle.go:312-324)
  J1 ar = host::jadd(host::jadd_aff(J1{t1[0], t1[1], t1[2]}, alpha), d0);
  // The G1 and G2 B-MSMs (prove.go:217,293) share scalars and layout: one
  // sorted digit plan serves both.
  HF2 t2[3];
  J1 bs1;
  {
    Arena parena(ctx);
    MsmPlan planB;
    if ((rc = msm_plan<C>(ctx, parena, wB.p, pk->nbB, pB, planB))) return rc;
    // Bs1 = MSM(wB, B) + beta + s delta   (computeBS1 icicle.go:299-310)
    if ((rc = msm_run<C, false>(ctx, planB, pk->B, t1))) return rc;
    bs1 = host::jadd(host::jadd_aff(J1{t1[0], t1[1], t1[2]}, beta), d1);
    // Bs = MSM_G2(wB, B2) + s delta2 + beta2   (computeBS2 icicle.go:377-393)
    if ((rc = msm_run<C, true>(ctx, planB, pk->B2, t2))) return rc;
  }
  // [s]Ar and [r]Bs1 on a host thread while the GPU runs the K and Z MSMs
  J1 s_ar, r_bs1;
  std::thread cross([&] {
    s_ar = host::jmul(ar, sc_.v, 4);
    r_bs1 = host::jmul(bs1, rc_.v, 4);
  });
  Joiner joiner2{cross};
  // Krs = MSM(wK, K) + kr delta + MSM(h[:n-1], Z) + s Ar + r Bs1   (computeKRS icicle.go:326-375)
  if ((rc = msm_device<C, false>(ctx, wK.p, pk->K, pk->nbK, t1, true, pK))) return rc;
  J1 krs = host::jadd(J1{t1[0], t1[1], t1[2]}, d2);
  if ((rc = hjob.wait())) return rc;
  if ((rc = msm_device<C, false>(ctx, (char*)a + 32 * pk->zlo, pk->Z, pk->nbZ, t1, true, pZ))) return rc;
  krs = host::jadd(krs, J1{t1[0], t1[1], t1[2]});
  cross.join();
  krs = host::jadd(krs, s_ar);
  krs = host::jadd(krs, r_bs1);
  J2 bs = host::jadd(J2{t2[0], t2[1], t2[2]}, sd2);
  bs = host::jadd_aff(bs, beta2);
  host::Aff<HF1> ara = host::to_aff(ar), krsa = host::to_aff(krs);
  host::Aff<HF2> bsa = host::to_aff(bs);
  memcpy(ar_out, &ara, sizeof(ara));
  memcpy(krs_out, &krsa, sizeof(krsa));
  memcpy(bs_out, &bsa, sizeof(bsa));
  return GM_OK;
}

}  // extern "C++"

int gm_g16_prove_device(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a, void* b,
                        void* c, size_t nc, const void* r, const void* s, void* ar_out,
                        void* bs_out, void* krs_out) {
  if (!ctx || !pk) return GM_ERR_INVALID;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = pk->curve == GM_BN254
               ? g16_prove_t<CurveBN254>(ctx, pk, wires_dev, a, b, c, nc, r, s, ar_out, bs_out, krs_out)
               : g16_prove_t<CurveBLS12377>(ctx, pk, wires_dev, a, b, c, nc, r, s, ar_out, bs_out,
                                            krs_out);
  prof_collect(ctx);
  return rc;
}

int gm_g16_prove(gm_ctx* ctx, gm_g16_pk* pk, const void* wires, const void* a, const void* b,
                 const void* c, size_t nc, const void* r, const void* s, void* ar_out, void* bs_out,
                 void* krs_out) {
  if (!ctx || !pk) return GM_ERR_INVALID;
  if (nc > pk->n) {
    set_error("prove: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  Arena arena(ctx);
  DevBuf w, da, db, dc;
  int rc;
  if ((rc = w.alloc(arena, 32 * pk->nb_wires)) || (rc = da.alloc(arena, 32 * pk->n)) ||
      (rc = db.alloc(arena, 32 * pk->n)) || (rc = dc.alloc(arena, 32 * pk->n)))
    return rc;
  GM_HIP(hipMemcpyAsync(w.p, wires, 32 * pk->nb_wires, hipMemcpyHostToDevice, st));
  GM_HIP(hipMemcpyAsync(da.p, a, 32 * nc, hipMemcpyHostToDevice, st));
  GM_HIP(hipMemcpyAsync(db.p, b, 32 * nc, hipMemcpyHostToDevice, st));
  GM_HIP(hipMemcpyAsync(dc.p, c, 32 * nc, hipMemcpyHostToDevice, st));
  return gm_g16_prove_device(ctx, pk, w.p, da.p, db.p, dc.p, nc, r, s, ar_out, bs_out, krs_out);
}

// ---- sharded Groth16 (BASELINE config 4) -------------------------------
int gm_g16_partial_bytes(int curve, size_t* out) {
  if (int rc = check_curve(curve)) return rc;
  if (out) *out = 4 * 3 * fp_bytes(curve) + 3 * 2 * fp_bytes(curve);
  return GM_OK;
}
}  // extern "C"

extern "C++" {
// The five raw MSM sums of this shard: computeH (whole domain), then the A, B,
// K, Z (h slice) G1 MSMs and the B G2 MSM over the shard's slices.
template <class C>
static int g16_partial_t(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a, void* b, void* c, size_t nc,
                         uint8_t* out) {
  using HF1 = typename C::HG1F;
  using HF2 = typename C::HG2F;
  hipStream_t st = ctx->stream;
  int rc;
  Arena arena(ctx);
  DevBuf wA, wB, wK;
  if ((rc = wA.alloc(arena, 32 * (pk->nbA ? pk->nbA : 1))) || (rc = wB.alloc(arena, 32 * (pk->nbB ? pk->nbB : 1))) ||
      (rc = wK.alloc(arena, 32 * (pk->nbK ? pk->nbK : 1))))
    return rc;
  {
    ProfScope ps(ctx, "gather_scalars");
    if (pk->nbA)
      hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(pk->nbA, 256)), dim3(256), 0, st, (const uint4*)wires_dev,
                         (const uint32_t*)pk->idxA, pk->nbA, (uint4*)wA.p);
    if (pk->nbB)
      hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(pk->nbB, 256)), dim3(256), 0, st, (const uint4*)wires_dev,
                         (const uint32_t*)pk->idxB, pk->nbB, (uint4*)wB.p);
    if (pk->nbK)
      hipLaunchKernelGGL(k_gather_fr, dim3(blocks_for(pk->nbK, 256)), dim3(256), 0, st, (const uint4*)wires_dev,
                         (const uint32_t*)pk->idxK, pk->nbK, (uint4*)wK.p);
  }
  GM_HIP(hipGetLastError());
  AuxComputeH hjob(ctx);
  if ((rc = hjob.start<C>(a, b, c, nc, pk->n))) return rc;
  const MsmPrecomp* pA = pk->precomp ? &pk->preA : nullptr;
  const MsmPrecomp* pB = pk->precomp ? &pk->preB : nullptr;
  const MsmPrecomp* pK = pk->precomp ? &pk->preK : nullptr;
  const MsmPrecomp* pZ = pk->precomp ? &pk->preZ : nullptr;
  HF1 t[3];
  constexpr size_t J1 = sizeof(t);
  if ((rc = msm_device<C, false>(ctx, wA.p, pk->A, pk->nbA, t, true, pA))) return rc;
  memcpy(out, t, J1);
  HF2 t2[3];
  {
    Arena parena(ctx);
    MsmPlan planB;
    if ((rc = msm_plan<C>(ctx, parena, wB.p, pk->nbB, pB, planB))) return rc;
    if ((rc = msm_run<C, false>(ctx, planB, pk->B, t))) return rc;
    memcpy(out + J1, t, J1);
    if ((rc = msm_run<C, true>(ctx, planB, pk->B2, t2))) return rc;
    memcpy(out + 4 * J1, t2, sizeof(t2));
  }
  if ((rc = msm_device<C, false>(ctx, wK.p, pk->K, pk->nbK, t, true, pK))) return rc;
  memcpy(out + 2 * J1, t, J1);
  if ((rc = hjob.wait())) return rc;
  if ((rc = msm_device<C, false>(ctx, (char*)a + 32 * pk->zlo, pk->Z, pk->nbZ, t, true, pZ))) return rc;
  memcpy(out + 3 * J1, t, J1);
  return GM_OK;
}

// Proof elements from the summed MSMs (icicle.go:295-391 / prove.go:195-305):
//   Ar  = sum_A + alpha + [r]delta
//   Bs1 = sum_B + beta + [s]delta
//   Krs = sum_K + [-rs]delta + sum_Z + [s]Ar + [r]Bs1
//   Bs  = sum_B2 + [s]delta2 + beta2
template <class C>
static int g16_finish_t(const gm_g16_pk_host* h, const uint8_t* sums, const void* r_mont, const void* s_mont,
                        void* ar_out, void* bs_out, void* krs_out) {
  using HF1 = typename C::HG1F;
  using HF2 = typename C::HG2F;
  using HFr = typename C::HFr;
  using J1 = host::Jac<HF1>;
  using J2 = host::Jac<HF2>;
  host::F<HFr> r, s;
  memcpy(r.v, r_mont, 32);
  memcpy(s.v, s_mont, 32);
  host::F<HFr> kr = -(r * s);
  host::F<HFr> rc_ = host::from_mont(r), sc_ = host::from_mont(s), krc = host::from_mont(kr);
  host::Aff<HF1> alpha, beta, delta;
  host::Aff<HF2> beta2, delta2;
  memcpy(&alpha, h->g1_alpha, sizeof(alpha));
  memcpy(&beta, h->g1_beta, sizeof(beta));
  memcpy(&delta, h->g1_delta, sizeof(delta));
  memcpy(&beta2, h->g2_beta, sizeof(beta2));
  memcpy(&delta2, h->g2_delta, sizeof(delta2));
  J1 sum[4];
  J2 sum2;
  for (int k = 0; k < 4; k++) memcpy(&sum[k], sums + k * sizeof(J1), sizeof(J1));
  memcpy(&sum2, sums + 4 * sizeof(J1), sizeof(J2));
  const J1 dj = host::to_jac(delta);
  J1 ar = host::jadd(host::jadd_aff(sum[0], alpha), host::jmul(dj, rc_.v, 4));
  J1 bs1 = host::jadd(host::jadd_aff(sum[1], beta), host::jmul(dj, sc_.v, 4));
  J1 krs = host::jadd(sum[2], host::jmul(dj, krc.v, 4));
  krs = host::jadd(krs, sum[3]);
  krs = host::jadd(krs, host::jmul(ar, sc_.v, 4));
  krs = host::jadd(krs, host::jmul(bs1, rc_.v, 4));
  J2 bs = host::jadd(sum2, host::jmul(host::to_jac(delta2), sc_.v, 4));
  bs = host::jadd_aff(bs, beta2);
  host::Aff<HF1> ara = host::to_aff(ar), krsa = host::to_aff(krs);
  host::Aff<HF2> bsa = host::to_aff(bs);
  memcpy(ar_out, &ara, sizeof(ara));
  memcpy(krs_out, &krsa, sizeof(krsa));
  memcpy(bs_out, &bsa, sizeof(bsa));
  return GM_OK;
}
}  // extern "C++"

extern "C" {
int gm_g16_prove_partial(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a_dev, void* b_dev, void* c_dev,
                         size_t nc, void* partial_out) {
  if (!ctx || !pk || !partial_out) return GM_ERR_INVALID;
  if (nc > pk->n) {
    set_error("prove: more constraints than the domain size");
    return GM_ERR_INVALID;
  }
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = pk->curve == GM_BN254
               ? g16_partial_t<CurveBN254>(ctx, pk, wires_dev, a_dev, b_dev, c_dev, nc, (uint8_t*)partial_out)
               : g16_partial_t<CurveBLS12377>(ctx, pk, wires_dev, a_dev, b_dev, c_dev, nc, (uint8_t*)partial_out);
  prof_collect(ctx);
  return rc;
}

int gm_g16_finish(int curve, const gm_g16_pk_host* h, const void* sums, const void* r, const void* s, void* ar_out,
                  void* bs_out, void* krs_out) {
  if (int rc = check_curve(curve)) return rc;
  if (!h || !sums || !r || !s || !ar_out || !bs_out || !krs_out) return GM_ERR_INVALID;
  return curve == GM_BN254
             ? g16_finish_t<CurveBN254>(h, (const uint8_t*)sums, r, s, ar_out, bs_out, krs_out)
             : g16_finish_t<CurveBLS12377>(h, (const uint8_t*)sums, r, s, ar_out, bs_out, krs_out);
}
}  // extern "C"
