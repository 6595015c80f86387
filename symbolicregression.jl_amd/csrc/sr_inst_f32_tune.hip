// Tuning variants of the hot kernel (f32, BASIC tier, full dataset), selected with SR_AMD_VARIANT:
//   1 = R4 no prefetch, 2 = R8 prefetch.  The default (0) is R4 + prefetch (sr_inst_f32_loss.hip).
#include "sr_interp_impl.h"
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_BASIC, 0)
SR_INSTANTIATE(float, 8, SR_MODE_LOSS, false, SR_TIER_BASIC, 1)
