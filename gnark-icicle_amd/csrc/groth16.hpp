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
  // every wire of [wlo, whi), they are stored wire-indexed -- point i of a copy
  // belongs to wire wlo + i, infinity where the wire has none -- and their MSMs
  // read ONE digit / sort plan over the wire slice instead of one per array
  // (g16_sums_t).  The compaction maps idxX stay as they are.
  bool wshare[3] = {false, false, false};  // A, B (and B2), K
  gm::MsmPrecomp preW;  // the wire plan's geometry (precomp: c / W / narrow of the shared arrays, stride = span)
  // staging buffers of the last freed gm_g16_stage of this key (pk_io.hip): the
  // next gm_g16_stage_begin on the same context reuses them instead of
  // allocating 4 vectors and the pinned ring per proof
  gm_g16_stage* spare_stage = nullptr;
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
void stage_spare_release(gm_g16_pk* pk);  // pk_io.hip
// computeH's NTT domain and tables for the key's n, built at upload (best effort;
// GM_G16_PREPARE_H=0 leaves them to the first prove)
void pk_prepare_h(gm_ctx* ctx, const gm_g16_pk* pk);
// gnark-layout points on the device -> internal layout at dst (+ window copies)
int prepare_points_into(gm_ctx* ctx, int curve, bool g2, const void* gnark_dev, size_t count,
                        const MsmPrecomp* pre, void* dst);
// Arrays (A, B, K) that qualify for the shared wire plan, from the counts alone
// (upload and cache load decide alike): each covers >= 31/32 of the `span`
// wires, and at least two of them do.  GM_G16_WIRE_PLAN=0 disables it.
void wire_plan_choice(size_t span, size_t nbA, size_t nbB, size_t nbK, bool out[3]);
// Wire maps of the chosen arrays from their local compaction maps (wire - wlo
// per point): map[x][i] = point index of wire i or MSM_SKIP.  An array whose
// map would repeat a wire drops out; fewer than two left: none shares.
void wire_plan_maps(size_t span, const uint32_t* const idx[3], const size_t cnt[3], bool want[3],
                    std::vector<uint32_t> map[3]);
// points per window copy of array which (PK_A..PK_B2): the wire span when the
// array is wire-indexed (shared plan), else its own count
inline size_t pk_array_points(const gm_g16_pk* pk, int which) {
  const size_t span = pk->whi - pk->wlo;
  switch (which) {
    case 0: return pk->wshare[0] ? span : pk->nbA;
    case 1:
    case 4: return pk->wshare[1] ? span : pk->nbB;
    case 2: return pk->nbZ;
    default: return pk->wshare[2] ? span : pk->nbK;
  }
}
// a, b, c = <L_i, w>, <R_i, w>, <O_i, w> of a device-resident R1CS (r1cs.hip),
// queued on ctx->stream
int r1cs_eval_device(gm_ctx* ctx, const gm_r1cs* r, const void* wires_dev, void* a, void* b, void* c);
size_t r1cs_nb_constraints(const gm_r1cs* r);
// proof from device-resident wires through a device-resident R1CS (groth16.hip);
// a, b, c: n-element device buffers the evaluation writes
int g16_prove_r1cs_device(gm_ctx* ctx, gm_g16_pk* pk, const gm_r1cs* r1, const void* wires_dev, void* a, void* b,
                          void* c, const void* r, const void* s, void* ar_out, void* bs_out, void* krs_out);
bool r1cs_matches_key(const gm_g16_pk* pk, const gm_r1cs* r1);
size_t r1cs_nb_wires(const gm_r1cs* r);
// src == nullptr: points from the host pointers in h
int pk_upload_ranges(gm_ctx* ctx, int curve, const gm_g16_pk_host* h, unsigned flags, const Ranges& rg,
                     gm_g16_pk** out, const PointSource* src);

}  // namespace gm
