// f32 loss kernels over the full dataset: BASIC tier at 8 rows/lane (default) and 4 (tuning),
// FULL tier at 4 rows/lane.
#include "sr_tile_impl.h"
SR_INSTANTIATE(float, 8, SR_MODE_LOSS, false, SR_TIER_BASIC)
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_BASIC)
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_FULL)
