// sr_grad.hip — forward-mode constant-gradient kernels (f32 / f64, 1 / 2 / 4 / 8 / 16 tangents per pass)
// and their launcher used by the C ABI (sr_eval_grad_batch).
#include "sr_grad_impl.h"

template <typename T>
hipError_t sr_launch_grad_any(const SrGradArgs<T>& a, int kt, bool gather, int n_blocks, hipStream_t s) {
  if (gather) {
    if (kt == 1) return sr_launch_grad<T, 1, 4, true>(a, n_blocks, s);
    if (kt == 2) return sr_launch_grad<T, 2, 4, true>(a, n_blocks, s);
    if (kt == 4) return sr_launch_grad<T, 4, 4, true>(a, n_blocks, s);
    if (kt == 8) return sr_launch_grad<T, 8, 4, true>(a, n_blocks, s);
    return sr_launch_grad<T, 16, 4, true>(a, n_blocks, s);
  }
  if (kt == 1) return sr_launch_grad<T, 1, 4, false>(a, n_blocks, s);
  if (kt == 2) return sr_launch_grad<T, 2, 4, false>(a, n_blocks, s);
  if (kt == 4) return sr_launch_grad<T, 4, 4, false>(a, n_blocks, s);
  if (kt == 8) return sr_launch_grad<T, 8, 4, false>(a, n_blocks, s);
  return sr_launch_grad<T, 16, 4, false>(a, n_blocks, s);
}

hipError_t sr_launch_grad_reduce(const double* part, int n_row_blocks, int n_vals, double* out, hipStream_t s) {
  if (n_vals <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_grad_reduce_kernel, dim3(unsigned((n_vals + 3) / 4)), dim3(256), 0, s, part, n_row_blocks,
                     n_vals, out);  // (4 waves per block, one value per wave)
  return hipGetLastError();
}

template hipError_t sr_launch_grad_any<float>(const SrGradArgs<float>&, int, bool, int, hipStream_t);
template hipError_t sr_launch_grad_any<double>(const SrGradArgs<double>&, int, bool, int, hipStream_t);
