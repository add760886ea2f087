// MSM entry points (see msm_impl.hpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "curves.hpp"

struct gm_ctx;

namespace gm {
struct Arena;
// Counting sort of the MSM digits (msm_impl.hpp k_msm_digits, msm_sort.hip).
// T buckets; coarse bin H = bucket >> F (NC bins, ~2K entries each for uniform
// digits, finished in LDS); pass-1 bin = bucket >> (F + G) (NS bins).  G = 0:
// two levels; G > 0: a middle pass splits each of the NS super-bins into its
// 2^G coarse bins (large MSMs).  M = upper bound on the entries.  Coarse bins
// above S2_BIG entries are split into parts.
constexpr uint32_t S2_BIG = 1u << 16;
constexpr uint32_t S2_STAGE = 6144;  // bins up to this many entries are sorted in LDS
struct SortGeom {
  uint32_t T = 0, F = 0, G = 0, NC = 0, NS = 0;
  size_t M = 0;
};
// Digits (k_msm_digits output: window-major, plus the pass-1 bin counts
// `scount`, NS words) -> sorted keys / values and offsets[0..T].  Scratch comes
// from `arena`.
int msm_sort_digits(gm_ctx* ctx, Arena& arena, const SortGeom& g, size_t n, uint32_t W, uint32_t nb,
                    uint32_t shared_stride, const uint32_t* dig, const uint32_t* scount, uint32_t* keys_out,
                    uint32_t* vals_out, uint32_t* offsets);

// Fixed-base precomputation of a resident point set (a proving key's arrays):
// W copies of the n points, copy w = [2^(c w)] P_i at index w * stride + i, so
// every window's digits land in ONE shared set of 2^(c-1) buckets.  The
// accumulation work is unchanged (one mixed add per non-zero digit), but the
// bucket reduction runs once instead of W times, which lets c grow (fewer
// windows).  c == 0 means plain points (no precomputation).
// Version of the precomputed-copy rule below (part of the device-layout cache
// fingerprint, pk_io.hip): bump when the copies' content or order changes.
// Layout 2: the last `narrow` windows are c - 1 bits wide so that the windows
// cover exactly bits + 1 bits: with one shared bucket set, a narrow TOP window
// (e.g. 13 of 22 bits at 2^24) would pile n / 2^12 entries on each of the
// lowest 2^12 buckets (long slice spans, tree fixups, hot sort bins); spreading
// the excess one bit per window keeps every bucket within ~2x of the mean.
constexpr uint32_t PRECOMP_LAYOUT = 2;
struct MsmPrecomp {
  uint32_t c = 0, W = 0;
  uint32_t narrow = 0;  // windows W - narrow .. W - 1 are c - 1 bits wide
  size_t stride = 0;
};
// narrow windows of a (c, W) layout over `bits`-bit scalars: c W - narrow =
// bits + 1 (signed digits), at least one full-width window
inline uint32_t precomp_narrow(uint32_t c, uint32_t W, int bits) {
  const long long e = (long long)c * W - (bits + 1);
  if (e <= 0) return 0;
  return (uint32_t)(e < (long long)W - 1 ? e : (long long)W - 1);
}

// Window size and copy count for a precomputed set of n points of a
// `bits`-bit scalar field: minimises n*W accumulation adds + ~3 adds per bucket.
MsmPrecomp msm_choose_precomp(size_t n, int bits);

// Host wire-map sentinel "this wire has no point" (groth16.hip, the shared wire
// plan): k_expand_points writes an all-zero (infinity) point into the expanded
// array's slot for such a wire.  It is never an entry value of a plan -- the
// accumulation kernels have no skip branch, so an entry carrying it would fail
// the bounds check (err = 2).  Valid point indices stay below 2^31 - 1
// (msm_plan bounds n and W * stride by 2^31).
constexpr uint32_t MSM_SKIP = 0x7fffffffu;

// Sorted signed-digit plan of one scalar vector: depends only on the scalars
// and the point layout, so MSMs that share scalars and layout (Groth16's G1 and
// G2 B-MSMs, prove.go:217,293) sort once.  Buffers live in the caller's Arena.
struct MsmPlan {
  uint32_t c = 0, W = 0, nb = 0, total = 0;
  uint32_t Wred = 0;  // windows reduced separately: W (plain) or 1 (shared buckets)
  size_t n = 0, M = 0;  // M: upper bound on the sorted entries (n * W); offsets[total] = actual
  size_t npts = 0;    // points addressable through the plan (bounds check)
  int bits = 0;       // scalar bits the digits cover (FR_BITS; 127 for a GLV split)
  uint32_t wn = 0;    // first narrow window (window_geom; W when all are c bits)
  uint32_t* keys = nullptr;     // sorted bucket keys (window-major bucket index), offsets[total] entries
  uint32_t* vals = nullptr;     // point index | sign << 31
  uint32_t* offsets = nullptr;  // total + 1 bucket start offsets
};
// glv (plain layout, BN254 and BLS12-377): each scalar k is split
// k = k1 + k2 lambda with |k1|, |k2| < 2^127, over 2n points
// [P_0..P_{n-1}, phi(P_0)..phi(P_{n-1})] (msm_device_launch builds them): half
// the windows, so half the buckets to reduce, for the same number of bucket adds.
template <class C>
int msm_plan(gm_ctx* ctx, Arena& arena, const void* scalars_dev, size_t n, const MsmPrecomp* pre,
             MsmPlan& plan, bool glv = false);
// GLV for an MSM of n points on ctx: the context's setting (gm_set_msm_glv)
// or, by default, on for n up to 2^21 (G1 and G2)
bool msm_glv_on(const gm_ctx* ctx, bool g2, size_t n);
template <class C, bool G2>
int msm_run(gm_ctx* ctx, const MsmPlan& plan, const void* points_internal,
            typename GroupSel<C, G2>::HF (&jac_out)[3]);

// An MSM whose device work is queued and whose host tail (consistency and
// long-span checks, host Horner) is deferred to msm_finish, so that the tail of
// one MSM overlaps the device work of the next.  Its buffers live in the Arena
// given to msm_launch, which must outlive msm_finish.
struct MsmTail {
  size_t n = 0, M = 0;
  uint32_t c = 0, W = 0, Wr = 0, nb = 0, total = 0, L = 0, nseg = 0, K = 0, Q = 2;
  uint32_t wn = 0;  // first narrow (c - 1 bit) window of the plan (window_geom)
  const uint32_t* keys = nullptr;
  const uint32_t* offsets = nullptr;
  void *buckets = nullptr, *pfirst = nullptr, *plast = nullptr, *nodes_a = nullptr, *nodes_b = nullptr;
  void *wsum = nullptr, *errw = nullptr;
  uint8_t* stage = nullptr;  // pinned readback: 16 B (error, max span) + the exported nodes
  gm_ctx* stage_ctx = nullptr;  // owner of `stage` (tail_pinned_acquire), released by msm_finish
  int stage_idx = -1;
  hipEvent_t done = nullptr;
  void release_stage();  // runtime.hpp: returns `stage` to the context
  MsmTail() = default;
  MsmTail(const MsmTail&) = delete;
  MsmTail& operator=(const MsmTail&) = delete;
  ~MsmTail() {
    if (done) hipEventDestroy(done);
    release_stage();
  }
};
template <class C, bool G2>
int msm_launch(gm_ctx* ctx, Arena& arena, const MsmPlan& plan, const void* points_internal, MsmTail& t);
template <class C, bool G2>
int msm_finish(gm_ctx* ctx, MsmTail& t, typename GroupSel<C, G2>::HF (&jac_out)[3]);
// plan + launch (points converted into `arena` first unless points_internal)
template <class C, bool G2>
// inputs_read (optional) is recorded on ctx->stream once the caller's scalars
// and points have been read for the last time (after the digits / conversion).
int msm_device_launch(gm_ctx* ctx, Arena& arena, const void* scalars_dev, const void* points_dev, size_t n,
                      bool points_internal, const MsmPrecomp* pre, MsmTail& t,
                      hipEvent_t inputs_read = nullptr);

// out = sum_i int(scalars[i]) * points[i] as a host Jacobian triple (X, Y, Z).
// points_dev is gnark-layout affine points, or (points_internal) an array of
// device-internal points prepared by msm_prepare_points /
// msm_precompute_points (e.g. a device-resident proving key); `pre` describes a
// precomputed set.
template <class C, bool G2>
int msm_device(gm_ctx* ctx, const void* scalars_dev, const void* points_dev, size_t n,
               typename GroupSel<C, G2>::HF (&jac_out)[3], bool points_internal = false,
               const MsmPrecomp* pre = nullptr);
// Converts n gnark-layout affine points into the internal layout (dst holds
// n * msm_internal_point_bytes<C, G2>() bytes).
template <class C, bool G2>
int msm_prepare_points(gm_ctx* ctx, const void* gnark_points, size_t n, void* dst);
// Same, plus the W - 1 shifted copies of `pre` (dst holds
// pre.W * pre.stride * msm_internal_point_bytes<C, G2>() bytes, stride >= n).
template <class C, bool G2>
int msm_precompute_points(gm_ctx* ctx, const void* gnark_points, size_t n, const MsmPrecomp& pre, void* dst);
template <class C, bool G2>
size_t msm_internal_point_bytes();
}  // namespace gm
