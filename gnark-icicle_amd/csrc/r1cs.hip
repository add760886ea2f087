// R1CS resident on the device: solution.A / .B / .C from the wires alone.
//
// gnark's solver fills a[i] = <L_i, w>, b[i] = <R_i, w>, c[i] = <O_i, w> as a
// by-product of solving (constraint/bn254/solver.go:540-620, terms valued by
// computeTerm :144-173).  The prover only needs them for computeH
// (prove.go:141-150), so with the constraint system on the device (uploaded
// once, like the proving key) a proof needs the wires alone over PCIe: 32 B per
// wire instead of 32 B per wire + 96 B per constraint (icicle.go:463-484 copies
// all four vectors).
//
// Layout: per matrix m (L, R, O) a CSR of terms: rowptr[m][i]..rowptr[m][i+1]
// index cid / vid; vid == GM_R1CS_CONST marks a constant term (Term.IsConstant,
// constraint/term.go:35-40).  Coefficients: gnark's CoeffTable (coeff.go:30-44),
// kept in gnark form (constants) and internal form (products).
#include <cstring>
#include <string>
#include <vector>

#include "curves.hpp"
#include "groth16.hpp"
#include "runtime.hpp"

struct gm_r1cs {
  int curve = 0;
  size_t nc = 0, nb_wires = 0, ncoeffs = 0;
  uint32_t* rowptr[3] = {nullptr, nullptr, nullptr};
  uint32_t* cid[3] = {nullptr, nullptr, nullptr};
  uint32_t* vid[3] = {nullptr, nullptr, nullptr};
  void* coeff_g = nullptr;  // gnark form (Montgomery, u64 limbs)
  void* coeff_i = nullptr;  // internal form (radix 2^29)
  size_t nnz[3] = {0, 0, 0};
};

namespace gm {
namespace {

// constant-table ids of gnark's CoeffTable (constraint/coeff.go: CoeffIdZero .. MinusTwo)
constexpr uint32_t CID_ZERO = 0, CID_ONE = 1;

template <class Fr>
__global__ void k_coeff_internal(const Fe<Fr>* __restrict__ g, size_t n, Fe<Fr>* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = fe_to_internal(fe_load_g<Fr>(g, i));
}

// One thread per (constraint, matrix): the row's terms summed in gnark form
// (mul(w_gnark, c_internal) = (w c)_gnark; additions are form-agnostic).
template <class Fr>
__global__ void __launch_bounds__(256) k_r1cs_eval(const uint32_t* __restrict__ rp0, const uint32_t* __restrict__ rp1,
                                                   const uint32_t* __restrict__ rp2, const uint32_t* __restrict__ c0,
                                                   const uint32_t* __restrict__ c1, const uint32_t* __restrict__ c2,
                                                   const uint32_t* __restrict__ v0, const uint32_t* __restrict__ v1,
                                                   const uint32_t* __restrict__ v2, const Fe<Fr>* __restrict__ cg,
                                                   const Fe<Fr>* __restrict__ ci, const Fe<Fr>* __restrict__ w,
                                                   size_t nc, Fe<Fr>* __restrict__ a, Fe<Fr>* __restrict__ b,
                                                   Fe<Fr>* __restrict__ c) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 3 * nc) return;
  const int m = (int)(t / nc);
  const size_t i = t - (size_t)m * nc;
  const uint32_t* rp = m == 0 ? rp0 : (m == 1 ? rp1 : rp2);
  const uint32_t* cid = m == 0 ? c0 : (m == 1 ? c1 : c2);
  const uint32_t* vid = m == 0 ? v0 : (m == 1 ? v1 : v2);
  Fe<Fr>* out = m == 0 ? a : (m == 1 ? b : c);
  Fe<Fr> acc = fe_zero<Fr>();
  for (uint32_t q = rp[i]; q < rp[i + 1]; q++) {
    const uint32_t k = cid[q], v = vid[q];
    if (k == CID_ZERO) continue;
    Fe<Fr> term;
    if (v == GM_R1CS_CONST) term = fe_load_g<Fr>(cg, k);
    else if (k == CID_ONE) term = fe_load_g<Fr>(w, v);
    else term = fe_mul(fe_load_g<Fr>(w, v), ci[k]);
    acc = fe_add(acc, term);
  }
  fe_store_g<Fr>(out, i, acc);
}

void r1cs_release(gm_r1cs* r) {
  for (int m = 0; m < 3; m++)
    for (void* p : {(void*)r->rowptr[m], (void*)r->cid[m], (void*)r->vid[m]})
      if (p) hipFree(p);
  if (r->coeff_g) hipFree(r->coeff_g);
  if (r->coeff_i) hipFree(r->coeff_i);
  delete r;
}

}  // namespace

template <class C>
int r1cs_eval_t(gm_ctx* ctx, const gm_r1cs* r, const void* wires_dev, void* a, void* b, void* c) {
  using Fr = typename C::Fr;
  if (!r->nc) return GM_OK;
  ProfScope ps(ctx, "r1cs_eval");
  hipLaunchKernelGGL(k_r1cs_eval<Fr>, dim3(blocks_for(3 * r->nc, 256)), dim3(256), 0, ctx->stream, r->rowptr[0],
                     r->rowptr[1], r->rowptr[2], r->cid[0], r->cid[1], r->cid[2], r->vid[0], r->vid[1], r->vid[2],
                     (const Fe<Fr>*)r->coeff_g, (const Fe<Fr>*)r->coeff_i, (const Fe<Fr>*)wires_dev, r->nc,
                     (Fe<Fr>*)a, (Fe<Fr>*)b, (Fe<Fr>*)c);
  GM_HIP(hipGetLastError());
  return GM_OK;
}

int r1cs_eval_device(gm_ctx* ctx, const gm_r1cs* r, const void* wires_dev, void* a, void* b, void* c) {
  return r->curve == GM_BN254 ? r1cs_eval_t<CurveBN254>(ctx, r, wires_dev, a, b, c)
                              : r1cs_eval_t<CurveBLS12377>(ctx, r, wires_dev, a, b, c);
}

size_t r1cs_nb_constraints(const gm_r1cs* r) { return r->nc; }
size_t r1cs_nb_wires(const gm_r1cs* r) { return r->nb_wires; }

}  // namespace gm

using namespace gm;

extern "C" {

int gm_r1cs_upload(gm_ctx* ctx, int curve, size_t nb_constraints, size_t nb_wires, const uint32_t* const* rowptr,
                   const uint32_t* const* cid, const uint32_t* const* vid, const void* coeffs, size_t ncoeffs,
                   gm_r1cs** out) {
  if (int rc = check_curve_id(curve)) return rc;
  if (!ctx || !rowptr || !cid || !vid || !out || (ncoeffs && !coeffs)) return GM_ERR_INVALID;
  if (nb_constraints >= (size_t(1) << 31) || nb_wires >= (size_t(1) << 32) - 1 || ncoeffs < 2) {
    set_error("r1cs upload: sizes out of range (CoeffTable holds at least zero and one)");
    return GM_ERR_INVALID;
  }
  // host validation: monotone row pointers, ids inside the tables (the kernel
  // indexes with them unchecked)
  size_t nnz[3];
  for (int m = 0; m < 3; m++) {
    if (!rowptr[m] || rowptr[m][0] != 0) {
      set_error("r1cs upload: row pointers must start at 0");
      return GM_ERR_INVALID;
    }
    for (size_t i = 0; i < nb_constraints; i++)
      if (rowptr[m][i + 1] < rowptr[m][i]) {
        set_error("r1cs upload: row pointers not monotone");
        return GM_ERR_INVALID;
      }
    nnz[m] = rowptr[m][nb_constraints];
    if (nnz[m] && (!cid[m] || !vid[m])) return GM_ERR_INVALID;
    for (size_t q = 0; q < nnz[m]; q++) {
      if (cid[m][q] >= ncoeffs || (vid[m][q] != GM_R1CS_CONST && vid[m][q] >= nb_wires)) {
        set_error("r1cs upload: term " + std::to_string(q) + " of matrix " + std::to_string(m) +
                  " has a coefficient or wire id out of range");
        return GM_ERR_INVALID;
      }
    }
  }
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  auto* r = new gm_r1cs();
  r->curve = curve;
  r->nc = nb_constraints;
  r->nb_wires = nb_wires;
  r->ncoeffs = ncoeffs;
  auto fail = [&](int code) {
    r1cs_release(r);
    return code;
  };
  auto up = [&](const void* src, size_t bytes, void** dst) -> int {
    if (hipMalloc(dst, bytes ? bytes : 16) != hipSuccess) {
      set_error("r1cs upload: hipMalloc failed");
      return GM_ERR_OOM;
    }
    if (bytes && hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      set_error("r1cs upload: hipMemcpy failed");
      return GM_ERR_DEVICE;
    }
    return GM_OK;
  };
  int rc;
  for (int m = 0; m < 3; m++) {
    r->nnz[m] = nnz[m];
    if ((rc = up(rowptr[m], 4 * (nb_constraints + 1), (void**)&r->rowptr[m])) ||
        (rc = up(cid[m], 4 * nnz[m], (void**)&r->cid[m])) || (rc = up(vid[m], 4 * nnz[m], (void**)&r->vid[m])))
      return fail(rc);
  }
  if ((rc = up(coeffs, 32 * ncoeffs, &r->coeff_g))) return fail(rc);
  if (hipMalloc(&r->coeff_i, 36 * ncoeffs + 64) != hipSuccess) return fail(GM_ERR_OOM);
  if (curve == GM_BN254)
    hipLaunchKernelGGL(k_coeff_internal<Bn254Fr>, dim3(blocks_for(ncoeffs, 256)), dim3(256), 0, ctx->stream,
                       (const Fe<Bn254Fr>*)r->coeff_g, ncoeffs, (Fe<Bn254Fr>*)r->coeff_i);
  else
    hipLaunchKernelGGL(k_coeff_internal<Bls377Fr>, dim3(blocks_for(ncoeffs, 256)), dim3(256), 0, ctx->stream,
                       (const Fe<Bls377Fr>*)r->coeff_g, ncoeffs, (Fe<Bls377Fr>*)r->coeff_i);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess) return fail(GM_ERR_DEVICE);
  *out = r;
  return GM_OK;
}

int gm_r1cs_free(gm_ctx* ctx, gm_r1cs* r) {
  if (!r) return GM_OK;
  if (ctx) {
    gm::CtxLock g(ctx);
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
  }
  r1cs_release(r);
  return GM_OK;
}

int gm_r1cs_eval(gm_ctx* ctx, const gm_r1cs* r, const void* wires_dev, void* a_dev, void* b_dev, void* c_dev) {
  if (!ctx || !r || (r->nc && (!wires_dev || !a_dev || !b_dev || !c_dev))) return GM_ERR_INVALID;
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  int rc = r1cs_eval_device(ctx, r, wires_dev, a_dev, b_dev, c_dev);
  if (rc) return rc;
  GM_HIP(hipStreamSynchronize(ctx->stream));
  prof_collect(ctx);
  return GM_OK;
}

}  // extern "C"
