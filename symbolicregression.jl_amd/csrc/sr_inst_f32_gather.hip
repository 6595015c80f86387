// f32 loss kernels over a row view (SubDataset / minibatch).
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS(float, 8, true)
SR_INSTANTIATE(float, 4, SR_MODE_LOSS, true, SR_TIER_FULL)
