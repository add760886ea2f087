// Pippenger MSM instantiation: CurveBN254 G1 (templates in msm_impl.hpp).
#include "msm_impl.hpp"

namespace gm {
GM_MSM_INSTANTIATE(CurveBN254, false)
GM_MSM_INSTANTIATE_PLAN(CurveBN254)
}  // namespace gm
