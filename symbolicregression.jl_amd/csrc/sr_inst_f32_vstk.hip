// f32 register-stack loss kernels (BASIC tier, operand stack in VGPRs): 8, 16 and 32 rows per lane,
// one build per elementwise loss.
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS_VSTK(float, 8, false)
SR_INSTANTIATE_LOSS_VSTK(float, 16, false)
SR_INSTANTIATE_LOSS_VSTK(float, 32, false)
