// f32 register-stack loss kernels (BASIC tier, operand stack in VGPRs): 8, 16 and 32 rows per lane,
// one build per elementwise loss.
// (A/B: SR_VSTK_TRIG_COPIES = 2 / 4 / 8 interleaved trig-table copies in these kernels' LDS, sr_libm.h)
#if defined(SR_VSTK_TRIG_COPIES)
#define SR_TRIG_COPIES SR_VSTK_TRIG_COPIES
#endif
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS_VSTK(float, 8, false)
SR_INSTANTIATE_LOSS_VSTK(float, 16, false)
SR_INSTANTIATE_LOSS_VSTK(float, 32, false)
