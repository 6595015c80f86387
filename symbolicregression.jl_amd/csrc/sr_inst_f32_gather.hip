// Explicit kernel instantiations: float, loss mode over a SubDataset row view (minibatching).
#include "sr_interp_impl.h"
SR_INSTANTIATE(float, SR_MODE_LOSS, true, SR_TIER_BASIC)
SR_INSTANTIATE(float, SR_MODE_LOSS, true, SR_TIER_FULL)
