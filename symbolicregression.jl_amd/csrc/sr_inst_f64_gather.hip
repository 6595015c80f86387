// f64 loss kernels over a row view (SubDataset / minibatch).
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS(double, 4, true)
SR_INSTANTIATE(double, 2, SR_MODE_LOSS, true, SR_TIER_FULL)
