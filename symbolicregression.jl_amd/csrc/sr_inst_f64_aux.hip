// Explicit kernel instantiations: double, prediction and exact-check modes (full operator tier).
#include "sr_interp_impl.h"
SR_INSTANTIATE(double, 2, SR_MODE_PRED, false, SR_TIER_FULL, 1)
SR_INSTANTIATE(double, 2, SR_MODE_PRED, true, SR_TIER_FULL, 1)
SR_INSTANTIATE(double, 2, SR_MODE_EXACT, false, SR_TIER_FULL, 1)
SR_INSTANTIATE(double, 2, SR_MODE_EXACT, true, SR_TIER_FULL, 1)
template size_t sr_interp_lds_bytes<double>(int, int, int);
