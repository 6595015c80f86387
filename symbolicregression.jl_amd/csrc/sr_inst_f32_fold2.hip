// f32 FOLD-mode kernels (round 6): the classic LDS-stack builds (full view and gathered views, BASIC
// tier at 8 rows per lane, FULL tier at 4), for the launches of a large call that run them.
#include "sr_tile_impl.h"
SR_INSTANTIATE_WL(float, 8, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, SR_LOSS_L2)
SR_INSTANTIATE_WL(float, 8, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, -1)
SR_INSTANTIATE_WL(float, 8, SR_MODE_FOLD, true, SR_TIER_BASIC, 4, -1)
SR_INSTANTIATE(float, 4, SR_MODE_FOLD, false, SR_TIER_FULL)
SR_INSTANTIATE(float, 4, SR_MODE_FOLD, true, SR_TIER_FULL)
