// f64 loss kernels over the full dataset: BASIC tier at 4 rows/lane, FULL tier at 2.
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS(double, 4, false)
SR_INSTANTIATE(double, 2, SR_MODE_LOSS, false, SR_TIER_FULL)
