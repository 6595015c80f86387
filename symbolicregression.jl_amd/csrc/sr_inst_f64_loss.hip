// Explicit kernel instantiations: double, loss mode (hot path), both operator tiers.
#include "sr_interp_impl.h"
SR_INSTANTIATE(double, 2, SR_MODE_LOSS, false, SR_TIER_BASIC, 1)
SR_INSTANTIATE(double, 2, SR_MODE_LOSS, false, SR_TIER_FULL, 1)
