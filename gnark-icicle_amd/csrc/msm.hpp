// MSM entry points (see msm.hip).
#pragma once
#include <cstddef>
#include <cstdint>
#include "curves.hpp"

struct gm_ctx;

namespace gm {
struct Arena;
// Sorts M (key, value) u32 pairs by the low end_bit key bits (msm_sort.hip).
int msm_sort_pairs(gm_ctx* ctx, Arena& arena, const uint32_t* keys_in, uint32_t* keys_out,
                   const uint32_t* vals_in, uint32_t* vals_out, size_t M, int end_bit);
// out = sum_i int(scalars[i]) * points[i] as a host Jacobian triple (X, Y, Z).
// points_dev is gnark-layout affine points, or (points_internal) an array of
// device-internal Affine<F> (radix-2^29 Montgomery) prepared by
// msm_prepare_points (e.g. a device-resident proving key).
template <class C, bool G2>
int msm_device(gm_ctx* ctx, const void* scalars_dev, const void* points_dev, size_t n,
               typename GroupSel<C, G2>::HF (&jac_out)[3], bool points_internal = false);
// Converts n gnark-layout affine points into the internal layout (dst holds
// n * msm_internal_point_bytes<C, G2>() bytes).
template <class C, bool G2>
int msm_prepare_points(gm_ctx* ctx, const void* gnark_points, size_t n, void* dst);
template <class C, bool G2>
size_t msm_internal_point_bytes();
}  // namespace gm
