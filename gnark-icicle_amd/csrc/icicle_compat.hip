// iciclegnark-semantics entry points (include/gnark_mi355x.h, "iciclegnark
// call-for-call binding"): the operations backend/groth16/bn254/icicle/icicle.go
// calls, with iciclegnark v0.1.0's buffer ownership and element order, so a cgo
// shim can bind them name for name without changing icicle.go.
//
// Order contract that icicle.go's computeH (icicle.go:453-513) relies on:
//   INttOnDevice(in)  natural-order evaluations -> NEW buffer of natural-order
//                     coefficients (the input is left bit-reversed, as iciclegnark
//                     reverses it in place before interpolating);
//   NttOnDevice(out, in) natural-order coefficients -> natural-order evaluations
//                     written to out;
//   ReverseScalars(h) after the final coset INttOnDevice turns h into the
//                     bit-reversed order of pk.G1.Z (setup.go:265-267).
// The fused path (gm_groth16_compute_h / gm_g16_prove) produces the same h with
// no extra permutation passes.
#include "curves.hpp"
#include "ntt.hpp"
#include "runtime.hpp"

using namespace gm;

namespace {

int check_curve_id(int curve) {
  if (curve != GM_BN254 && curve != GM_BLS12_377) {
    set_error("unknown curve id");
    return GM_ERR_INVALID;
  }
  return GM_OK;
}

template <class C>
int intt_fresh(gm_ctx* ctx, void* in, size_t n, bool coset, void* out) {
  // in (natural) -> bit-reversed copy in out -> DIT inverse (bit-reversed in,
  // natural out); then mirror iciclegnark's in-place reversal of the input.
  int rc;
  if ((rc = bitrev_copy_device<C>(ctx, out, in, n))) return rc;
  if ((rc = ntt_device<C>(ctx, out, n, true, true, coset))) return rc;
  return reverse_device<C>(ctx, in, n);
}

template <class C>
int ntt_into(gm_ctx* ctx, void* out, const void* in, size_t n, bool coset) {
  int rc;
  if (out == in) {
    if ((rc = reverse_device<C>(ctx, out, n))) return rc;
  } else if ((rc = bitrev_copy_device<C>(ctx, out, in, n))) {
    return rc;
  }
  return ntt_device<C>(ctx, out, n, false, true, coset);
}

}  // namespace

extern "C" {

int gm_icicle_generate_twiddles(gm_ctx* ctx, int curve, size_t n, int inverse, void** token_out) {
  (void)inverse;  // one cached domain serves both directions
  if (!ctx || !token_out) return GM_ERR_INVALID;
  if (int rc = check_curve_id(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? ntt_domain_prepare<CurveBN254>(ctx, n) : ntt_domain_prepare<CurveBLS12377>(ctx, n);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  // a real (freeable) allocation standing for the twiddle table handle
  hipError_t e = hipMalloc(token_out, 64);
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  return GM_OK;
}

int gm_icicle_intt_on_device(gm_ctx* ctx, int curve, void* in_dev, size_t n, int coset, void** out_dev) {
  if (!ctx || !in_dev || !out_dev) return GM_ERR_INVALID;
  if (int rc = check_curve_id(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  void* out = nullptr;
  hipError_t e = hipMalloc(&out, 32 * (n ? n : 1));
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return GM_ERR_OOM;
  }
  int rc = curve == GM_BN254 ? intt_fresh<CurveBN254>(ctx, in_dev, n, coset != 0, out)
                             : intt_fresh<CurveBLS12377>(ctx, in_dev, n, coset != 0, out);
  if (rc == GM_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) {
    set_error("gm_icicle_intt_on_device: stream synchronisation failed");
    rc = GM_ERR_DEVICE;
  }
  prof_collect(ctx);
  if (rc) {
    hipFree(out);
    return rc;
  }
  *out_dev = out;
  return GM_OK;
}

int gm_icicle_ntt_on_device(gm_ctx* ctx, int curve, void* out_dev, const void* in_dev, size_t n, int coset) {
  if (!ctx || !in_dev || !out_dev) return GM_ERR_INVALID;
  if (int rc = check_curve_id(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? ntt_into<CurveBN254>(ctx, out_dev, in_dev, n, coset != 0)
                             : ntt_into<CurveBLS12377>(ctx, out_dev, in_dev, n, coset != 0);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

int gm_icicle_poly_ops(gm_ctx* ctx, int curve, void* a_dev, const void* b_dev, const void* c_dev,
                       const void* den_dev, size_t n) {
  if (!ctx || !a_dev || !b_dev || !c_dev || !den_dev) return GM_ERR_INVALID;
  if (int rc = check_curve_id(curve)) return rc;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = curve == GM_BN254 ? poly_ops_vec_device<CurveBN254>(ctx, a_dev, b_dev, c_dev, den_dev, n)
                             : poly_ops_vec_device<CurveBLS12377>(ctx, a_dev, b_dev, c_dev, den_dev, n);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

}  // extern "C"
