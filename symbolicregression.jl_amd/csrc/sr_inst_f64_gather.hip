// Explicit kernel instantiations: double, loss mode over a SubDataset row view (minibatching).
#include "sr_interp_impl.h"
SR_INSTANTIATE(double, 2, SR_MODE_LOSS, true, SR_TIER_BASIC, 1)
SR_INSTANTIATE(double, 2, SR_MODE_LOSS, true, SR_TIER_FULL, 1)
