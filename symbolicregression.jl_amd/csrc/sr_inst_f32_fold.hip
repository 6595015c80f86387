// f32 FOLD-mode kernels (round 6): the complete trees' loss programs again, composing the reference's
// in-order loss fold per row tile (sr_fold_dev.h) — the register-stack builds of the large-call path.
#include "sr_tile_impl.h"
SR_INSTANTIATE_WLV(float, 16, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, SR_LOSS_L2, true)
SR_INSTANTIATE_WLV(float, 16, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, -1, true)
