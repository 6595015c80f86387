// sr_grad_f64.hip — the Float64 forward-mode constant-gradient kernels (sr_grad_impl.h).
#include "sr_grad_impl.h"

template hipError_t sr_launch_grad_any<double>(const SrGradArgs<double>&, int, bool, int, int, hipStream_t);
