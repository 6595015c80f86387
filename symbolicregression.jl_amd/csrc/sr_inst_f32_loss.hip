// Explicit kernel instantiations: float, loss mode (hot path), both operator tiers.
#include "sr_interp_impl.h"
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_BASIC, 1)
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, false, SR_TIER_FULL, 1)
