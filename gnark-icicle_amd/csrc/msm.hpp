// MSM entry points (see msm.hip).
#pragma once
#include <cstddef>
#include "curves.hpp"

struct gm_ctx;

namespace gm {
// out = sum_i int(scalars[i]) * points[i] as a host Jacobian triple (X, Y, Z).
template <class C, bool G2>
int msm_device(gm_ctx* ctx, const void* scalars_dev, const void* points_dev, size_t n,
               typename GroupSel<C, G2>::HF (&jac_out)[3]);
}  // namespace gm
