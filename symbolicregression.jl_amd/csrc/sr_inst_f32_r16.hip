// f32 BASIC-tier loss kernels at 16 rows/lane (one build per elementwise loss): twice the rows per
// dispatched instruction of the 8-rows/lane kernels, for large views.
#include "sr_tile_impl.h"
SR_INSTANTIATE_LOSS(float, 16, false)
