// Element-wise test hooks for the device field / curve layer (used by the
// parity tests to pin each arithmetic primitive against the oracle).  Not on
// the proving path.
#include <chrono>
#include <vector>

#include "curves.hpp"
#include "runtime.hpp"
#include "../../include/gnark_mi355x_testhooks.h"

namespace gm {

// gnark-layout element i -> internal, and back
template <class F>
struct ElemIO {
  GM_DEV static F load(const uint8_t* p, size_t i) {
    return Coord<F>::load_internal(reinterpret_cast<const uint32_t*>(p) + i * Coord<F>::WORDS);
  }
  GM_DEV static void store(uint8_t* p, size_t i, const F& v) {
    Coord<F>::store_gnark(reinterpret_cast<uint32_t*>(p) + i * Coord<F>::WORDS, v);
  }
};

template <class F>
__global__ void k_field_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F x = ElemIO<F>::load(a, i), y = ElemIO<F>::load(b, i), r;
  switch (op) {
    case 0: r = fe_mul(x, y); break;
    case 1: r = fe_add(x, y); break;
    case 2: r = fe_sub(x, y); break;
    case 3: r = fe_neg(x); break;
    case 4: r = fe_inv(x); break;
    case 5: r = fe_sqr(x); break;
    default: r = x; break;
  }
  ElemIO<F>::store(out, i, r);
}

template <class F>
GM_DEV Affine<F> to_affine_dev(const XYZZ<F>& a) {
  Affine<F> r;
  if (xyzz_is_inf(a)) {
    r.x = FOps<F>::zero();
    r.y = FOps<F>::zero();
    return r;
  }
  F t = fe_inv(fe_mul(a.zz, a.zzz));
  r.x = fe_mul(a.x, fe_mul(t, a.zzz));
  r.y = fe_mul(a.y, fe_mul(t, a.zz));
  return r;
}

template <class F>
GM_DEV XYZZ<F> from_affine_dev(const Affine<F>& p) {
  XYZZ<F> r = xyzz_inf<F>();
  xyzz_add_aff(r, p);
  return r;
}

template <class F>
__global__ void k_point_op(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int PW = 2 * Coord<F>::WORDS;
  Affine<F> p = load_affine_gnark<F>(a + i * PW), q = load_affine_gnark<F>(b + i * PW);
  XYZZ<F> r;
  switch (op) {
    case 0: r = from_affine_dev(p); xyzz_add_aff(r, q); break;          // mixed add
    case 1: r = xyzz_dbl(from_affine_dev(p)); break;                      // double
    case 2: r = xyzz_add(from_affine_dev(p), from_affine_dev(q)); break;  // full add
    case 3: r = xyzz_mul_small(from_affine_dev(p), 1000003u); break;      // small scalar mul
    default: r = from_affine_dev(p); break;
  }
  store_affine_gnark<F>(out + i * PW, to_affine_dev(r));
}

}  // namespace gm

using namespace gm;

extern "C++" {
template <class C>
static int field_op_t(gm_ctx* ctx, int kind, int op, const void* a, const void* b, void* out, size_t n) {
  auto g = dim3(blocks_for(n, 64)), t = dim3(64);
  auto A = (const uint8_t*)a, B = (const uint8_t*)b;
  auto O = (uint8_t*)out;
  if (kind == 0) hipLaunchKernelGGL(k_field_op<Fe<typename C::Fr>>, g, t, 0, ctx->stream, op, A, B, O, n);
  else if (kind == 1) hipLaunchKernelGGL(k_field_op<typename C::G1F>, g, t, 0, ctx->stream, op, A, B, O, n);
  else hipLaunchKernelGGL(k_field_op<typename C::G2F>, g, t, 0, ctx->stream, op, A, B, O, n);
  GM_HIP(hipGetLastError());
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
template <class C, bool G2>
static int point_op_t(gm_ctx* ctx, int op, const void* a, const void* b, void* out, size_t n) {
  using DF = typename GroupSel<C, G2>::DF;
  hipLaunchKernelGGL(k_point_op<DF>, dim3(blocks_for(n, 64)), dim3(64), 0, ctx->stream, op,
                     (const uint32_t*)a, (const uint32_t*)b, (uint32_t*)out, n);
  GM_HIP(hipGetLastError());
  GM_HIP(hipStreamSynchronize(ctx->stream));
  return GM_OK;
}
}

extern "C" {
int gm_test_field_op(gm_ctx* ctx, int curve, int kind, int op, const void* a_dev, const void* b_dev,
                     void* out_dev, size_t n) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  if (kind < 0 || kind > 2) return GM_ERR_INVALID;
  return curve == GM_BN254 ? field_op_t<CurveBN254>(ctx, kind, op, a_dev, b_dev, out_dev, n)
                           : field_op_t<CurveBLS12377>(ctx, kind, op, a_dev, b_dev, out_dev, n);
}
int gm_test_point_op(gm_ctx* ctx, int curve, int g2, int op, const void* a_dev, const void* b_dev,
                     void* out_dev, size_t n) {
  gm::CtxLock g(ctx);
  GM_HIP(hipSetDevice(ctx->device));
  if (curve == GM_BN254)
    return g2 ? point_op_t<CurveBN254, true>(ctx, op, a_dev, b_dev, out_dev, n)
              : point_op_t<CurveBN254, false>(ctx, op, a_dev, b_dev, out_dev, n);
  return g2 ? point_op_t<CurveBLS12377, true>(ctx, op, a_dev, b_dev, out_dev, n)
            : point_op_t<CurveBLS12377, false>(ctx, op, a_dev, b_dev, out_dev, n);
}
}

/* The solver-side cost of staging the reference benchmark circuit's level shape
 * (backend/groth16/groth16_test.go:120-156: a chain of squarings; the solver runs
 * it as one one-instruction level after another, constraint/bn254/solver.go:
 * 471-484).  Level j finishes constraint j and solves wire nb_inputs + j (the
 * last level, the final assertion, solves no wire).  mode 0: one put per level
 * and vector; mode 1: the Go hook's pattern (integration/go/icicle_bn254/
 * staged.go): ids appended to pending lists, handed over every `flush_at` ids and
 * at the end.  abc = 0: wires only (resident constraint system).  The put range
 * of the witness inputs comes first.  *ns_per_level = host time / levels. */
extern "C" int gm_test_stage_replay_chain(gm_g16_stage* st, const void* wires, size_t nb_inputs, const void* a,
                                          const void* b, const void* c, size_t nb_constraints, int mode, int abc,
                                          size_t flush_at, double* ns_per_level) {
  if (!st || !wires || !ns_per_level || (abc && (!a || !b || !c)) || nb_constraints == 0 || flush_at == 0)
    return GM_ERR_INVALID;
  const auto t0 = std::chrono::steady_clock::now();
  int rc = gm_g16_stage_put_range(st, GM_STAGE_WIRES, 0, nb_inputs, wires);
  std::vector<uint32_t> pw, pc;
  pw.reserve(flush_at);
  pc.reserve(flush_at);
  auto put_abc = [&](const uint32_t* ids, size_t k) {
    int r = gm_g16_stage_put_indexed(st, GM_STAGE_A, a, ids, k);
    if (!r) r = gm_g16_stage_put_indexed(st, GM_STAGE_B, b, ids, k);
    if (!r) r = gm_g16_stage_put_indexed(st, GM_STAGE_C, c, ids, k);
    return r;
  };
  for (size_t j = 0; j < nb_constraints && !rc; j++) {
    const uint32_t cid = (uint32_t)j, wid = (uint32_t)(nb_inputs + j);
    const bool solves = j + 1 < nb_constraints;
    if (mode == 0) {
      if (solves) rc = gm_g16_stage_put_indexed(st, GM_STAGE_WIRES, wires, &wid, 1);
      if (!rc && abc) rc = put_abc(&cid, 1);
      continue;
    }
    if (solves) pw.push_back(wid);
    if (pw.size() >= flush_at) {
      rc = gm_g16_stage_put_indexed(st, GM_STAGE_WIRES, wires, pw.data(), pw.size());
      pw.clear();
    }
    if (!abc || rc) continue;
    pc.push_back(cid);
    if (pc.size() >= flush_at) {
      rc = put_abc(pc.data(), pc.size());
      pc.clear();
    }
  }
  if (!rc && !pw.empty()) rc = gm_g16_stage_put_indexed(st, GM_STAGE_WIRES, wires, pw.data(), pw.size());
  if (!rc && !pc.empty()) rc = put_abc(pc.data(), pc.size());
  *ns_per_level = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() /
                  (double)nb_constraints;
  return rc;
}
