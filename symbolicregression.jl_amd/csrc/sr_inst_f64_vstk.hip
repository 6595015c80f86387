// f64 register-stack loss kernels (BASIC tier, operand stack in VGPRs): 8 rows per lane (twice the
// classic f64 kernel's), one build per elementwise loss; and a 4-row build (SR_AMD_VSTK_ROWS=-4).
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS_VSTK(double, 8, false)
SR_INSTANTIATE_LOSS_VSTK(double, 4, false)
