// sr_aux.hip — small kernels around the interpreter: fixed-order partial reduction, dataset
// transpose/padding, and the runtime dispatcher over the explicitly instantiated interpreters.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sr_eval.h"

template <typename T>
__device__ __forceinline__ T sr_wave_sum_aux(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// One wave per tree: Σ over row blocks in a fixed lane/stride order (bit-reproducible), OR of flags.
__global__ void __launch_bounds__(256) sr_reduce_partials_kernel(const double* __restrict__ part_sum,
                                                                  const uint32_t* __restrict__ part_flag,
                                                                  int n_trees, int n_row_blocks,
                                                                  const uint8_t* __restrict__ static_bad,
                                                                  double* __restrict__ out_sum,
                                                                  uint32_t* __restrict__ out_flag) {
  const int tree = int((int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (tree >= n_trees) return;
  const double* ps = part_sum + size_t(tree) * n_row_blocks;
  const uint32_t* pf = part_flag + size_t(tree) * n_row_blocks;
  double s = 0.0;
  uint32_t f = 0u;
  for (int i = lane; i < n_row_blocks; i += 64) {
    s += ps[i];
    f |= pf[i];
  }
  s = sr_wave_sum_aux<double>(s);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) f |= __shfl_xor(f, off, 64);
  if (lane == 0) {
    if (static_bad && static_bad[tree]) f |= SR_FLAG_STATIC | SR_FLAG_NONFINITE;
    out_sum[tree] = s;
    out_flag[tree] = f;
  }
}

// Julia [nf, n] column-major -> per-feature rows [nf][ld]; padded rows replicate row 0 so that the
// interpreter's validity checks never see a value that is not in the dataset.
template <typename T>
__global__ void sr_transpose_kernel(const T* __restrict__ Xh, int64_t nf, int64_t n, int64_t ld,
                                    T* __restrict__ Xd) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= ld) return;
  const int64_t src = (i < n) ? i : 0;
  for (int64_t f = 0; f < nf; ++f) Xd[f * ld + i] = Xh[src * nf + f];
}

template <typename T>
__global__ void sr_pad_kernel(T* __restrict__ v, int64_t n, int64_t ld, T pad_value, int replicate_first) {
  const int64_t i = n + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= ld) return;
  v[i] = replicate_first ? v[0] : pad_value;
}

hipError_t sr_launch_reduce(const double* part_sum, const uint32_t* part_flag, int n_trees, int n_row_blocks,
                            const uint8_t* static_bad, double* out_sum, uint32_t* out_flag, hipStream_t s) {
  if (n_trees <= 0) return hipSuccess;
  const int64_t blocks = (int64_t(n_trees) * 64 + 255) / 256;
  hipLaunchKernelGGL(sr_reduce_partials_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, part_sum, part_flag,
                     n_trees, n_row_blocks, static_bad, out_sum, out_flag);
  return hipGetLastError();
}

template <typename T>
hipError_t sr_launch_transpose(const T* Xh_dev, int64_t nf, int64_t n, int64_t ld, T* Xd, hipStream_t s) {
  const int64_t blocks = (ld + 255) / 256;
  hipLaunchKernelGGL(sr_transpose_kernel<T>, dim3(unsigned(blocks)), dim3(256), 0, s, Xh_dev, nf, n, ld, Xd);
  return hipGetLastError();
}

template <typename T>
hipError_t sr_launch_pad(T* v, int64_t n, int64_t ld, T pad_value, int replicate_first, hipStream_t s) {
  if (ld <= n) return hipSuccess;
  const int64_t blocks = (ld - n + 255) / 256;
  hipLaunchKernelGGL(sr_pad_kernel<T>, dim3(unsigned(blocks)), dim3(256), 0, s, v, n, ld, pad_value, replicate_first);
  return hipGetLastError();
}

template <typename T>
hipError_t sr_launch_interp(const SrEvalArgs<T>& a, int mode, bool gather, int tier, SrVariant v, int n_blocks,
                            hipStream_t s) {
  constexpr int R = 16 / sizeof(T);
  if (mode == SR_MODE_LOSS) {
    if (tier == SR_TIER_BASIC) {
      if (!gather) {
        if constexpr (sizeof(T) == 4) {
          if (v.rows_per_lane == 8) return sr_dispatch_interp<T, 8, SR_MODE_LOSS, false, SR_TIER_BASIC, 1>(a, n_blocks, s);
          if (v.var == 0) return sr_dispatch_interp<T, 4, SR_MODE_LOSS, false, SR_TIER_BASIC, 0>(a, n_blocks, s);
        }
        return sr_dispatch_interp<T, R, SR_MODE_LOSS, false, SR_TIER_BASIC, 1>(a, n_blocks, s);
      }
      return sr_dispatch_interp<T, R, SR_MODE_LOSS, true, SR_TIER_BASIC, 1>(a, n_blocks, s);
    }
    return gather ? sr_dispatch_interp<T, R, SR_MODE_LOSS, true, SR_TIER_FULL, 1>(a, n_blocks, s)
                  : sr_dispatch_interp<T, R, SR_MODE_LOSS, false, SR_TIER_FULL, 1>(a, n_blocks, s);
  }
  if (mode == SR_MODE_PRED)
    return gather ? sr_dispatch_interp<T, R, SR_MODE_PRED, true, SR_TIER_FULL, 1>(a, n_blocks, s)
                  : sr_dispatch_interp<T, R, SR_MODE_PRED, false, SR_TIER_FULL, 1>(a, n_blocks, s);
  return gather ? sr_dispatch_interp<T, R, SR_MODE_EXACT, true, SR_TIER_FULL, 1>(a, n_blocks, s)
                : sr_dispatch_interp<T, R, SR_MODE_EXACT, false, SR_TIER_FULL, 1>(a, n_blocks, s);
}

template hipError_t sr_launch_interp<float>(const SrEvalArgs<float>&, int, bool, int, SrVariant, int, hipStream_t);
template hipError_t sr_launch_interp<double>(const SrEvalArgs<double>&, int, bool, int, SrVariant, int, hipStream_t);
template hipError_t sr_launch_transpose<float>(const float*, int64_t, int64_t, int64_t, float*, hipStream_t);
template hipError_t sr_launch_transpose<double>(const double*, int64_t, int64_t, int64_t, double*, hipStream_t);
template hipError_t sr_launch_pad<float>(float*, int64_t, int64_t, float, int, hipStream_t);
template hipError_t sr_launch_pad<double>(double*, int64_t, int64_t, double, int, hipStream_t);
