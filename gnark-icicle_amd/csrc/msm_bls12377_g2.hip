// Pippenger MSM instantiation: CurveBLS12377 G2 (templates in msm_impl.hpp).
// Lane-pair kernels capped at three waves per SIMD (168 VGPRs, some spills):
// same-box A/B at 2^22, accumulation 48.2 -> 46.7 ms.  (BN254 G2 keeps two
// waves: 5.34 vs 5.64 ms at three.)
#ifndef GM_PAIR_WPE
#define GM_PAIR_WPE 3
#endif
#include "msm_impl.hpp"

namespace gm {
GM_MSM_INSTANTIATE(CurveBLS12377, true)
}  // namespace gm
