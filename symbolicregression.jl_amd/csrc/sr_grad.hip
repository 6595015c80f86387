// sr_grad.hip — forward-mode constant-gradient kernels (f32 / f64, 1 / 2 / 4 / 8 / 16 tangents per pass)
// and their launcher used by the C ABI (sr_eval_grad_batch).
#include "sr_grad_impl.h"

template <typename T, bool GATHER, int KT>
hipError_t sr_launch_grad_rows(const SrGradArgs<T>& a, int rows, int n_blocks, hipStream_t s) {
  constexpr int RD = sr_grad_rows_per_lane(KT);
  if (rows == RD) return sr_launch_grad<T, KT, 4, GATHER, RD>(a, n_blocks, s);
  if constexpr (RD != 1) {
    if (rows == 1) return sr_launch_grad<T, KT, 4, GATHER, 1>(a, n_blocks, s);
  }
  return hipErrorInvalidValue;
}

template <typename T>
hipError_t sr_launch_grad_any(const SrGradArgs<T>& a, int kt, bool gather, int rows, int n_blocks, hipStream_t s) {
  auto go = [&](auto g) -> hipError_t {
    constexpr bool G = decltype(g)::value;
    switch (kt) {
      case 1: return sr_launch_grad_rows<T, G, 1>(a, rows, n_blocks, s);
      case 2: return sr_launch_grad_rows<T, G, 2>(a, rows, n_blocks, s);
      case 4: return sr_launch_grad_rows<T, G, 4>(a, rows, n_blocks, s);
      case 8: return sr_launch_grad_rows<T, G, 8>(a, rows, n_blocks, s);
      case 16: return sr_launch_grad_rows<T, G, 16>(a, rows, n_blocks, s);
      default: return hipErrorInvalidValue;
    }
  };
  return gather ? go(std::true_type{}) : go(std::false_type{});
}

hipError_t sr_launch_grad_reduce(const double* part, int n_row_blocks, int n_vals, double* out, hipStream_t s) {
  if (n_vals <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_grad_reduce_kernel, dim3(unsigned((n_vals + 3) / 4)), dim3(256), 0, s, part, n_row_blocks,
                     n_vals, out);  // (4 waves per block, one value per wave)
  return hipGetLastError();
}

template hipError_t sr_launch_grad_any<float>(const SrGradArgs<float>&, int, bool, int, int, hipStream_t);
template hipError_t sr_launch_grad_any<double>(const SrGradArgs<double>&, int, bool, int, int, hipStream_t);
