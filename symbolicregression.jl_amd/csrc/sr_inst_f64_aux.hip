// f64 prediction and exact-check (Julia-order range sum) kernels (FULL tier, 2 rows/lane).
#include "sr_tile_impl.h"
SR_INSTANTIATE(double, 2, SR_MODE_PRED, false, SR_TIER_FULL)
SR_INSTANTIATE(double, 2, SR_MODE_PRED, true, SR_TIER_FULL)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, false, SR_TIER_FULL, 1)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, true, SR_TIER_FULL, 1)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, false, SR_TIER_FULL, 4)
SR_INSTANTIATE_W(double, 2, SR_MODE_EXACT, true, SR_TIER_FULL, 4)
SR_INSTANTIATE_DERIVED(double)
