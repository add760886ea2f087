// Pippenger MSM instantiation: CurveBLS12377 G2 (templates in msm_impl.hpp).
// Lane-pair kernels at two waves per SIMD (256 VGPRs, no spill).  Since the
// lane-pair product is one unsigned reduction (r04) this beats the three-wave
// cap, which spills 130 VGPRs: 2^22 MSM 41.0-41.1 vs 46.3-46.4 ms same box
// (profiles/r04e_g2_ab.txt; r02 measured the opposite for the old product).
#ifndef GM_PAIR_WPE
#define GM_PAIR_WPE 2
#endif
#include "msm_impl.hpp"

namespace gm {
GM_MSM_INSTANTIATE(CurveBLS12377, true)
}  // namespace gm
