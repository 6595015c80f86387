// Explicit kernel instantiations: float, loss mode (hot path), both operator tiers.
#include "sr_interp_impl.h"
SR_INSTANTIATE(float, SR_MODE_LOSS, false, SR_TIER_BASIC)
SR_INSTANTIATE(float, SR_MODE_LOSS, false, SR_TIER_FULL)
