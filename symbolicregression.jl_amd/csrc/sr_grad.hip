// sr_grad.hip — forward-mode constant-gradient kernels (Float32; 1 / 2 / 4 / 8 / 16 tangents per pass),
// their partial reduction, and the launcher used by the C ABI (sr_eval_grad_batch).
#include "sr_grad_impl.h"

// Σ over row blocks of the [row block][item][KT] partials -> out[item][KT], one wave per value: lane
// l folds row blocks l, l + 64, ... in order and a fixed butterfly adds the lanes (deterministic; a
// thread per value walking ~160 row blocks serially took 46 us per launch in C3's searches).
__global__ void __launch_bounds__(256) sr_grad_reduce_kernel(const double* __restrict__ part, int n_row_blocks,
                                                              int n_vals, double* __restrict__ out) {
  const int lane = int(threadIdx.x) & 63;
  const int i = int(int64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64);
  if (i >= n_vals) return;  // wave-uniform
  double s = 0.0;
  for (int b = lane; b < n_row_blocks; b += 64) s += part[size_t(b) * n_vals + i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[i] = s;
}

hipError_t sr_launch_grad_reduce(const double* part, int n_row_blocks, int n_vals, double* out, hipStream_t s) {
  if (n_vals <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_grad_reduce_kernel, dim3(unsigned((n_vals + 3) / 4)), dim3(256), 0, s, part, n_row_blocks,
                     n_vals, out);  // (4 waves per block, one value per wave)
  return hipGetLastError();
}

template hipError_t sr_launch_grad_any<float>(const SrGradArgs<float>&, int, bool, int, int, hipStream_t);
// (Float64: sr_grad_f64.hip, a translation unit of its own so the two compile in parallel)
