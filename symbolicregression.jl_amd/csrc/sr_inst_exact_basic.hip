// Exact-check (Julia-order range sum) kernels for BASIC-tier operator sets (round 5): the same pass
// without the FULL tier's 38 further operators in the dispatch (f32: 121 -> 84 VGPRs).
#include "sr_tile_impl.h"
SR_INSTANTIATE_W(float, 4, SR_MODE_EXACT, false, SR_TIER_BASIC, 1)
SR_INSTANTIATE_W(float, 4, SR_MODE_EXACT, true, SR_TIER_BASIC, 1)
SR_INSTANTIATE_W(float, 4, SR_MODE_EXACT, false, SR_TIER_BASIC, 4)
SR_INSTANTIATE_W(float, 4, SR_MODE_EXACT, true, SR_TIER_BASIC, 4)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, false, SR_TIER_BASIC, 1)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, true, SR_TIER_BASIC, 1)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, false, SR_TIER_BASIC, 4)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, true, SR_TIER_BASIC, 4)
