// f32 loss kernels over the full dataset: BASIC tier at 8 rows/lane (one build per elementwise loss;
// 4 rows/lane and the 8-wave L2 build for tuning; 16 rows/lane: sr_inst_f32_r16.hip), FULL tier at 4 rows/lane.
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS(float, 8, false)
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_BASIC)
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_FULL)
SR_INSTANTIATE_WL(float, 8, SR_MODE_LOSS, false, SR_TIER_BASIC, 8, SR_LOSS_L2)
