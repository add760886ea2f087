// Device-resident Groth16 proving key shared by groth16.hip (upload, prove)
// and pk_io.hip (WriteDump streaming, device-layout cache, staged inputs).
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

#include "../../include/gnark_mi355x.h"
#include "msm.hpp"

struct gm_g16_pk {
  int curve;
  size_t n, nb_wires, nb_public, nbA, nbB, nbK;
  void *A = nullptr, *B = nullptr, *Z = nullptr, *K = nullptr, *B2 = nullptr;  // device point arrays
  void *idxA = nullptr, *idxB = nullptr, *idxK = nullptr;  // device compaction maps (wire - wlo)
  size_t zlo = 0, nbZ = 0;      // this key's slice of h / pk.G1.Z (whole key: 0, n-1)
  size_t wlo = 0, whi = 0;      // wires the maps address: [wlo, whi) (whole key: 0, nb_wires)
  bool precomp = false;         // GM_PK_PRECOMPUTE: fixed-base window copies
  gm::MsmPrecomp preA, preB, preZ, preK;  // layouts (B and B2 share preB)
  std::vector<uint8_t> alpha, beta, delta, beta2, delta2;  // host affine
  // Shared wire plan: when the A, B (+ B2) and K arrays each cover (nearly)
  // every wire of [wlo, whi), their MSMs read ONE digit / sort plan over the
  // wire slice instead of one per array (g16_sums_t).  wmap[X][i] = array X's
  // point index for wire wlo + i, or MSM_SKIP; nullptr = identity.
  bool wshare[3] = {false, false, false};  // A, B, K
  void* wmap[3] = {nullptr, nullptr, nullptr};
  gm::MsmPrecomp preW;  // the wire plan's geometry (precomp: same c / W / narrow as the shared arrays)
};

namespace gm {

// point arrays of a key, in WriteDump order (marshal.go:430-444)
enum PkArray { PK_A = 0, PK_B = 1, PK_Z = 2, PK_K = 3, PK_B2 = 4 };

struct Ranges {
  size_t loA, hiA, loB, hiB, loK, hiK, loZ, hiZ;
  bool rebase;  // index maps relative to the lowest wire they address (gm_multi keys)
};

// Fills the device-internal array `dst` (already allocated: count points, times
// pre->W copies when pre != nullptr) with `count` points of key array `which`.
using PointSource = std::function<int(int which, size_t count, bool g2, const MsmPrecomp* pre, void* dst)>;

int check_curve_id(int curve);
size_t internal_point_bytes(int curve, bool g2);
void pk_release(gm_g16_pk* pk);
// gnark-layout points on the device -> internal layout at dst (+ window copies)
int prepare_points_into(gm_ctx* ctx, int curve, bool g2, const void* gnark_dev, size_t count,
                        const MsmPrecomp* pre, void* dst);
// Arrays (A, B, K) that qualify for the shared wire plan, from the counts alone
// (upload and cache load decide alike): each covers >= 31/32 of the `span`
// wires, and at least two of them do.  GM_G16_WIRE_PLAN=0 disables it.
void wire_plan_choice(size_t span, size_t nbA, size_t nbB, size_t nbK, bool out[3]);
// Builds pk's wire maps from the key's local compaction maps (wire - wlo per
// point of A, B, K; host memory) and sets pk->wshare / wmap / preW.
int pk_setup_wire_plan(gm_ctx* ctx, gm_g16_pk* pk, const uint32_t* ia, const uint32_t* ib, const uint32_t* ik);
// a, b, c = <L_i, w>, <R_i, w>, <O_i, w> of a device-resident R1CS (r1cs.hip),
// queued on ctx->stream
int r1cs_eval_device(gm_ctx* ctx, const gm_r1cs* r, const void* wires_dev, void* a, void* b, void* c);
size_t r1cs_nb_constraints(const gm_r1cs* r);
size_t r1cs_nb_wires(const gm_r1cs* r);
// src == nullptr: points from the host pointers in h
int pk_upload_ranges(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, const Ranges& rg,
                     gm_g16_pk** out, const PointSource* src);

}  // namespace gm
