// Pippenger MSM instantiation: CurveBLS12377 G1 (templates in msm_impl.hpp).
#include "msm_impl.hpp"

namespace gm {
GM_MSM_INSTANTIATE(CurveBLS12377, false)
GM_MSM_INSTANTIATE_PLAN(CurveBLS12377)
}  // namespace gm
