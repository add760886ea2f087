// Pippenger MSM instantiation: CurveBN254 G2 (templates in msm_impl.hpp).
#include "msm_impl.hpp"

namespace gm {
GM_MSM_INSTANTIATE(CurveBN254, true)
}  // namespace gm
