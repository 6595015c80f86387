// sr_aux.hip — small kernels around the interpreter: fixed-order partial reduction, dataset
// transpose/padding, and the runtime dispatcher over the explicitly instantiated tile kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sr_eval.h"
#include "sr_fold.h"
#include "sr_fold_dev.h"


// The result goes to the caller's tree index perm[position].  One wave per tree: lane l folds row blocks l, l + 64, ... in order, then a fixed butterfly adds the
// 64 lane sums (deterministic: the same tree gives the same bits whatever the batch).  A thread per
// tree walking every row block serialises its loads (C3's 196 row blocks: 47 us per call).
__global__ void __launch_bounds__(256) sr_reduce_partials_kernel(const double* __restrict__ part_sum,
                                                                  const uint32_t* __restrict__ part_flag,
                                                                  int n_trees, int n_row_blocks,
                                                                  const uint32_t* __restrict__ perm,
                                                                  const uint8_t* __restrict__ static_bad,
                                                                  double* __restrict__ out_sum,
                                                                  uint32_t* __restrict__ out_flag) {
  const int lane = int(threadIdx.x) & 63;
  const int pos = int(int64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64);
  if (pos >= n_trees) return;  // wave-uniform
  sr_reduce_positions<1, false>(part_sum, part_flag, n_trees, n_row_blocks, pos, 1, 1, perm, static_bad, out_sum,
                                out_flag, lane);
}

// Julia's pairwise `sum` of one view, from its leaf folds: every thread combines one array's
// n_leaves folds by the shared post-order program (leaf index: push it; -1: add the top two, in T),
// the order of Base.mapreduce_impl's recursion; out[a] = isfinite(total).
// Base.mapreduce_impl's combine of one view's leaf folds, level by level: `nodes` holds the
// internal nodes of the recursion tree grouped by height (level_off), each as (left, right) with
// c >= 0 = leaf c and c < 0 = internal node -c-1; a node's two children are always of lower height,
// so a level's nodes are independent.  One workgroup per array; the internal sums go to `scratch`
// ([n_arrays][n_internal], global: the workgroup barrier orders them); the root's isfinite -> out.
template <typename T>
__global__ void __launch_bounds__(256) sr_jsum_levels_kernel(const T* __restrict__ leaf_sums, int n_leaves,
                                                             const int2* __restrict__ nodes, int n_internal,
                                                             const int32_t* __restrict__ level_off, int n_levels,
                                                             T* __restrict__ scratch, uint8_t* __restrict__ out) {
  const int64_t a = blockIdx.x;
  const T* leaf = leaf_sums + a * n_leaves;
  T* in = scratch + a * n_internal;
  for (int lv = 0; lv < n_levels; ++lv) {
    for (int m = level_off[lv] + int(threadIdx.x); m < level_off[lv + 1]; m += int(blockDim.x)) {
      const int2 c = nodes[m];
      const T x = c.x >= 0 ? leaf[c.x] : in[-c.x - 1];
      const T y = c.y >= 0 ? leaf[c.y] : in[-c.y - 1];
      in[m] = x + y;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[a] = __builtin_isfinite(n_internal > 0 ? in[n_internal - 1] : leaf[0]) ? 1 : 0;
}

template <typename T>
hipError_t sr_launch_jsum_levels(const T* leaf_sums, int64_t n_arrays, int n_leaves, const int2* nodes, int n_internal,
                                 const int32_t* level_off, int n_levels, T* scratch, uint8_t* out, hipStream_t s) {
  if (n_arrays <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_jsum_levels_kernel<T>, dim3(unsigned(n_arrays)), dim3(256), 0, s, leaf_sums, n_leaves, nodes,
                     n_internal, level_off, n_levels, scratch, out);
  return hipGetLastError();
}
template hipError_t sr_launch_jsum_levels<float>(const float*, int64_t, int, const int2*, int, const int32_t*, int, float*,
                                                 uint8_t*, hipStream_t);
template hipError_t sr_launch_jsum_levels<double>(const double*, int64_t, int, const int2*, int, const int32_t*, int,
                                                  double*, uint8_t*, hipStream_t);

// Packed row-shard partials for one all-reduce (sr_eval_loss_partials_packed): [5][n] f64 = Σ loss,
// then the NONFINITE / BIG / STATIC / ELEMINF flag bits as 0 / 1.
__global__ void __launch_bounds__(256) sr_pack_partials_kernel(const double* __restrict__ sum,
                                                                const uint32_t* __restrict__ flag, int n,
                                                                double* __restrict__ out) {
  const int t = int(int64_t(blockIdx.x) * blockDim.x + threadIdx.x);
  if (t >= n) return;
  const uint32_t f = flag[t];
  out[t] = sum[t];
  out[size_t(n) + t] = (f & SR_FLAG_NONFINITE) ? 1.0 : 0.0;
  out[2 * size_t(n) + t] = (f & SR_FLAG_BIG) ? 1.0 : 0.0;
  out[3 * size_t(n) + t] = (f & SR_FLAG_STATIC) ? 1.0 : 0.0;
  out[4 * size_t(n) + t] = (f & SR_FLAG_ELEMINF) ? 1.0 : 0.0;
}

hipError_t sr_launch_pack_partials(const double* sum, const uint32_t* flag, int n, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_pack_partials_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, sum, flag, n, out);
  return hipGetLastError();
}

// Row-sharded finalize on the device (sr_eval_loss_sharded): the partials [5][n] summed over every
// rank -> loss[t] = Σ / denom (f64 division, rounded once to T) or +Inf, and comp[t] = 0 incomplete,
// 1 complete, 2 flagged BIG only (the exact Julia-order check over the global rows decides; its loss
// slot holds the finite value), plus SR_COMP_FOLD when the reference's loss fold over the n_terms global
// rows must be computed in order (sr_fold.h).  The same rules as the host's finalize (sr_capi.cpp).
template <typename T>
__global__ void __launch_bounds__(256) sr_finalize_packed_kernel(const double* __restrict__ packed, int n,
                                                                 double denom, int64_t n_terms, T* __restrict__ loss,
                                                                 uint8_t* __restrict__ comp) {
  const int t = int(int64_t(blockIdx.x) * blockDim.x + threadIdx.x);
  if (t >= n) return;
  const bool nonfinite = packed[size_t(n) + t] > 0.0;
  const bool big = packed[2 * size_t(n) + t] > 0.0;
  const bool stat = packed[3 * size_t(n) + t] > 0.0;
  const bool elem_inf = packed[4 * size_t(n) + t] > 0.0;
  const bool ok = !nonfinite && !stat;
  T l = ok ? T(packed[t] / denom) : T(INFINITY);
  uint8_t c = ok ? (big ? uint8_t(2) : uint8_t(1)) : uint8_t(0);
  if (ok) {
    const int cls = n_terms > 0 ? sr_fold_class<T>(packed[t], elem_inf, n_terms) : (elem_inf ? SR_FOLD_INF : SR_FOLD_FINITE);
    if (cls == SR_FOLD_INF) l = T(INFINITY);
    if (cls == SR_FOLD_EXACT) c |= uint8_t(SR_COMP_FOLD);
  }
  loss[t] = l;
  comp[t] = c;
}

template <typename T>
hipError_t sr_launch_finalize_packed(const double* packed, int n, double denom, int64_t n_terms, T* loss, uint8_t* comp,
                                     hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_finalize_packed_kernel<T>, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, packed, n, denom,
                     n_terms, loss, comp);
  return hipGetLastError();
}
template hipError_t sr_launch_finalize_packed<float>(const double*, int, double, int64_t, float*, uint8_t*, hipStream_t);
template hipError_t sr_launch_finalize_packed<double>(const double*, int, double, int64_t, double*, uint8_t*, hipStream_t);

// ---------------------------------------------------------------- the reference's loss fold, exactly
// LossFunctions' mean / weighted sum fold the elementwise losses left to right in T
// (src/LossFunctions.jl:38-58; sr_fold.h).  For the rare trees whose overflow the bounds of sr_fold.h
// cannot decide, these kernels compute that fold bit for bit.  While the running value p stays in one
// binade [2^e, 2^(e+1)) with spacing 2^q, fl(p + l) = p + 2^q (m + r), where l / 2^q = m + f (m integer)
// and r rounds f half-to-even against the parity of p / 2^q + m — so a step depends on the running
// value only through its parity, and runs of steps compose (a pair: the ulps added from an even and
// from an odd start; compose(x, y)(b) = x(b) + y((b + x(b)) & 1)).  The step that leaves the binade is
// the hardware add itself.
//
// Round 5: the whole GPU folds, not one workgroup per tree.  The rows are cut into segments of
// seg_len rows and three launches run:
//   segsum  (one workgroup per tree and segment) the f64 sum of each segment's losses;
//   segtab  (the same grid) the composed step of each segment for the binades holding the fold's value
//           at the segment start if that value is within 2^-7 of the f64 prefix sum before it (<= 2
//           binades; the fold's real relative error over 64M rows is ~1e-4);
//   chain   (one workgroup per tree) walks the segments in order: a segment whose table covers the
//           running value's binade and that ends inside it advances in O(1); any other segment (the
//           first, those where the fold crosses a binade, a value outside the speculated window) is
//           folded exactly by the workgroup scan of rounds 3-4 (fold_range).
// Every O(1) advance is an exact composition of the segment's steps, so the result does not depend on
// the segmentation (seg_len = 0: the whole view through fold_range, rounds 3-4's kernel;
// tests/test_gpu_fold.py compares both bit for bit).
template <typename T>
struct SrFoldRows {  // the listed tree's elementwise losses (the interpreter's product, in the same order)
  const T* pr;
  const T* y;
  const T* w;
  const int64_t* row_idx;
  int lk;
  T lp;
  __device__ __forceinline__ T operator()(int64_t i) const {
    const int64_t ri = row_idx ? row_idx[i] : i;
    T e = sr_elem_loss<T>(lk, pr[i], y[ri], lp);
    if (w) e *= w[ri];
    return e;
  }
  // R consecutive losses from row r0 (rows >= hi: 0, which adds nothing).  A full, 16-byte aligned run
  // of a full view is read with 16-byte loads: a thread's R rows are contiguous, so one scalar load per
  // row would make every load instruction touch 64 cache lines (one per lane)
  template <int R>
  __device__ __forceinline__ void rows_from(int64_t r0, int64_t hi, T (&ev)[R]) const {
    constexpr int C = 16 / int(sizeof(T));
    using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
    const bool vec = !row_idx && r0 + R <= hi && ((reinterpret_cast<uintptr_t>(pr + r0) | reinterpret_cast<uintptr_t>(y + r0) |
                                                  (w ? reinterpret_cast<uintptr_t>(w + r0) : 0)) & 15u) == 0;
    if (vec) {
#pragma unroll
      for (int c = 0; c < R / C; ++c) {
        const V pv = *reinterpret_cast<const V*>(pr + r0 + c * C);
        const V yv = *reinterpret_cast<const V*>(y + r0 + c * C);
        const T* pp = reinterpret_cast<const T*>(&pv);
        const T* yy = reinterpret_cast<const T*>(&yv);
        T wv[C];
        if (w) {
          const V wq = *reinterpret_cast<const V*>(w + r0 + c * C);
#pragma unroll
          for (int j = 0; j < C; ++j) wv[j] = reinterpret_cast<const T*>(&wq)[j];
        }
#pragma unroll
        for (int j = 0; j < C; ++j) {
          T e = sr_elem_loss<T>(lk, pp[j], yy[j], lp);
          if (w) e *= wv[j];
          ev[c * C + j] = e;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) ev[r] = (r0 + r < hi) ? (*this)(r0 + r) : T(0);
    }
  }
};

template <typename T>
__global__ void __launch_bounds__(256) sr_fold_segsum_kernel(SrFoldRows<T> rows, int64_t pred_ld, int64_t n,
                                                             int64_t seg_len, int n_seg, double* __restrict__ segsum) {
  const int seg = int(blockIdx.x), b = int(blockIdx.y), tid = int(threadIdx.x);
  SrFoldRows<T> rw = rows;
  rw.pr = rows.pr + int64_t(b) * pred_ld;
  const int64_t lo = int64_t(seg) * seg_len, hi = lo + seg_len < n ? lo + seg_len : n;
  double acc = 0.0;
  for (int64_t i = lo + tid; i < hi; i += 256) acc += double(rw(i));
  __shared__ double s_w[4];
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((tid & 63) == 0) s_w[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) segsum[int64_t(b) * n_seg + seg] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}

// composed steps of one segment for binades qa and qb: tab[b][seg] = {a0(qa), a1(qa), a0(qb), a1(qb)}
template <typename T, int R>
__global__ void __launch_bounds__(256) sr_fold_segtab_kernel(SrFoldRows<T> rows, int64_t pred_ld, int64_t n,
                                                             int64_t seg_len, int n_seg,
                                                             const double* __restrict__ segsum,
                                                             const double* __restrict__ carry_est,
                                                             int2* __restrict__ tq, int64_t* __restrict__ tab) {
  using Tr = SrFoldTraits<T>;
  using I = typename SrFoldTab<T>::I;
  constexpr I CAP = I(1) << (Tr::mant + 3);
  const int seg = int(blockIdx.x), b = int(blockIdx.y), tid = int(threadIdx.x), lane = tid & 63, wave = tid >> 6;
  SrFoldRows<T> rw = rows;
  rw.pr = rows.pr + int64_t(b) * pred_ld;
  __shared__ double s_d[4];
  __shared__ I s_v[4][4];
  // the f64 prefix before this segment (any order: it only chooses the binades to tabulate)
  const double* ss = segsum + int64_t(b) * n_seg;
  double pre = 0.0;
  for (int j = tid; j < seg; j += 256) pre += ss[j];
  for (int off = 32; off >= 1; off >>= 1) pre += __shfl_xor(pre, off, 64);
  if (lane == 0) s_d[wave] = pre;
  __syncthreads();
  const double S = (carry_est ? carry_est[b] : 0.0) + ((s_d[0] + s_d[1]) + (s_d[2] + s_d[3]));
  const int qa = sr_fold_q<T>(S * (1.0 - 0x1p-7)), qb = sr_fold_q<T>(S * (1.0 + 0x1p-7));
  const bool two = qb != qa;
  const int64_t lo = int64_t(seg) * seg_len, hi = lo + seg_len < n ? lo + seg_len : n;
  I ta0 = 0, ta1 = 0, tb0 = 0, tb1 = 0;  // the segment so far (meaningful in thread 0)
  for (int64_t base = lo; base < hi; base += 256 * R) {
    I a0 = 0, a1 = 0, c0 = 0, c1 = 0;  // this thread's R consecutive rows, binades qa and qb
    const int64_t r0 = base + int64_t(tid) * R;
    T ev[R];
    rw.template rows_from<R>(r0, hi, ev);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      I m;
      int kind;
      SrFoldTab<T>::step(ev[r], qa, m, kind);
      sr_fold_add_i<I>(m, kind, CAP, a0, a1);
    }
    if (two) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        I m;
        int kind;
        SrFoldTab<T>::step(ev[r], qb, m, kind);
        sr_fold_add_i<I>(m, kind, CAP, c0, c1);
      }
    }
    // ordered reduction over the wave's lanes (lane l's rows precede lane l + 1's), then the waves
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      I o0 = __shfl_down(a0, off, 64), o1 = __shfl_down(a1, off, 64);
      if ((lane & (2 * off - 1)) == 0) {
        sr_fold_compose_i<I>(a0, a1, o0, o1, CAP);
        a0 = o0;
        a1 = o1;
      }
      if (two) {
        I p0 = __shfl_down(c0, off, 64), p1 = __shfl_down(c1, off, 64);
        if ((lane & (2 * off - 1)) == 0) {
          sr_fold_compose_i<I>(c0, c1, p0, p1, CAP);
          c0 = p0;
          c1 = p1;
        }
      }
    }
    if (lane == 0) {
      s_v[wave][0] = a0;
      s_v[wave][1] = a1;
      s_v[wave][2] = c0;
      s_v[wave][3] = c1;
    }
    __syncthreads();
    if (tid == 0) {
      for (int v = 0; v < 4; ++v) {
        I y0 = s_v[v][0], y1 = s_v[v][1];
        sr_fold_compose_i<I>(ta0, ta1, y0, y1, CAP);
        ta0 = y0;
        ta1 = y1;
        y0 = s_v[v][2];
        y1 = s_v[v][3];
        sr_fold_compose_i<I>(tb0, tb1, y0, y1, CAP);
        tb0 = y0;
        tb1 = y1;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int64_t o = int64_t(b) * n_seg + seg;
    tq[o] = make_int2(qa, qb);
    tab[4 * o + 0] = int64_t(ta0);
    tab[4 * o + 1] = int64_t(ta1);
    tab[4 * o + 2] = int64_t(two ? tb0 : ta0);
    tab[4 * o + 3] = int64_t(two ? tb1 : ta1);
  }
}

// The workgroup scan of rounds 3-4 over rows [s_k, hi) from the running value s_p (every thread
// calls it; the state lives in LDS): CHUNK rows per round, restarting at each binade crossing.
template <typename T, int R, typename Rows>
__device__ void sr_fold_range(const Rows& elem, int64_t hi, T* s_p, int64_t* s_k, int64_t* s_w0, int64_t* s_w1) {
  using Tr = SrFoldTraits<T>;
  constexpr int NT = 1024;
  constexpr int64_t CHUNK = int64_t(NT) * R;
  constexpr int64_t CAP = int64_t(1) << (Tr::mant + 3);
  constexpr T MIN_NORMAL = sizeof(T) == 4 ? T(1.17549435e-38f) : T(2.2250738585072014e-308);
  const int tid = int(threadIdx.x), lane = tid & 63, wave = tid >> 6;
  for (;;) {
    __syncthreads();
    const T p = *s_p;
    const int64_t k = *s_k;
    __syncthreads();  // every thread has read the state before thread 0 may write it again
    if (k >= hi || !(p <= SrM<T>::big)) break;  // done, or +Inf / NaN (a fold that stays so)
    // p = P 2^q, P < lim: the binade's spacing (subnormals: the fixed spacing up to the first normal)
    int q;
    int64_t lim;
    if (p < MIN_NORMAL) {
      q = Tr::qmin;
      lim = int64_t(1) << Tr::mant;
    } else {
      int ex;
      (void)frexp(double(p), &ex);
      q = ex - 1 - Tr::mant;
      lim = int64_t(1) << (Tr::mant + 1);
    }
    const int64_t P = int64_t(ldexp(double(p), -q));
    // this thread's R consecutive losses and their composed step
    const int64_t base = k + int64_t(tid) * R;
    T ev[R];
    elem.template rows_from<R>(base, hi, ev);
    int64_t a0 = 0, a1 = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const SrFoldStep<T> st = sr_fold_step<T>(ev[r], q, CAP);
      int64_t e0 = sr_fold_inc<T>(st, (0 + a0) & 1), e1 = sr_fold_inc<T>(st, (1 + a1) & 1);
      a0 = a0 + e0 < CAP ? a0 + e0 : CAP;
      a1 = a1 + e1 < CAP ? a1 + e1 : CAP;
    }
    // inclusive scan over the wave's lanes (in row order), then over the waves
    int64_t i0 = a0, i1 = a1;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t l0 = __shfl_up(i0, off, 64), l1 = __shfl_up(i1, off, 64);
      if (lane >= off) sr_fold_compose(l0, l1, i0, i1, CAP);
    }
    if (lane == 63) {
      s_w0[wave] = i0;
      s_w1[wave] = i1;
    }
    __syncthreads();
    int64_t w0 = 0, w1 = 0;  // the waves before this one
    for (int v = 0; v < wave; ++v) {
      int64_t y0 = s_w0[v], y1 = s_w1[v];
      sr_fold_compose(w0, w1, y0, y1, CAP);
      w0 = y0;
      w1 = y1;
    }
    int64_t t0 = 0, t1 = 0;  // the whole chunk
    for (int v = 0; v < NT / 64; ++v) {
      int64_t y0 = s_w0[v], y1 = s_w1[v];
      sr_fold_compose(t0, t1, y0, y1, CAP);
      t0 = y0;
      t1 = y1;
    }
    const int64_t b0 = P & 1;
    const int64_t tot = b0 ? t1 : t0;
    if (P + tot < lim) {  // the whole chunk stays in this binade
      if (tid == 0) {
        *s_p = T(ldexp(double(P + tot), q));
        *s_k = k + CHUNK < hi ? k + CHUNK : hi;
      }
      continue;
    }
    // the step leaving the binade: in the thread whose exclusive prefix is below lim and inclusive
    // prefix is not (prefixes only grow, so exactly one thread)
    int64_t e0 = __shfl_up(i0, 1, 64), e1 = __shfl_up(i1, 1, 64);
    if (lane == 0) e0 = e1 = 0;
    int64_t x0 = w0, x1 = w1;
    sr_fold_compose(x0, x1, e0, e1, CAP);  // exclusive prefix of this thread
    int64_t n0 = w0, n1 = w1, y0 = i0, y1 = i1;
    sr_fold_compose(n0, n1, y0, y1, CAP);  // inclusive
    const int64_t pre = P + (b0 ? e1 : e0), inc = P + (b0 ? y1 : y0);
    if (pre < lim && inc >= lim) {
      int64_t run = pre;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (base + r >= hi) break;
        const int64_t d = sr_fold_inc<T>(sr_fold_step<T>(ev[r], q, CAP), run & 1);
        if (run + d >= lim) {
          *s_p = T(ldexp(double(run), q)) + ev[r];  // the hardware's own rounding of this step
          *s_k = base + r + 1;
          break;
        }
        run += d;
      }
    }
  }
}

template <typename T, int R>
__global__ void __launch_bounds__(1024) sr_fold_chain_kernel(SrFoldRows<T> rows, int64_t pred_ld, int64_t n,
                                                             int64_t seg_len, int n_seg, const int2* __restrict__ tq,
                                                             const int64_t* __restrict__ tab,
                                                             const T* __restrict__ carry, T* __restrict__ out,
                                                             int* __restrict__ n_slow) {
  using Tr = SrFoldTraits<T>;
  constexpr int SB = 512;  // segments per LDS batch of tables
  constexpr T MIN_NORMAL = sizeof(T) == 4 ? T(1.17549435e-38f) : T(2.2250738585072014e-308);
  __shared__ T s_p;
  __shared__ int64_t s_k, s_seg;
  __shared__ int64_t s_w0[16], s_w1[16];
  __shared__ int2 s_tq[SB];
  __shared__ int64_t s_tab[SB * 4];
  const int b = int(blockIdx.x), tid = int(threadIdx.x);
  SrFoldRows<T> rw = rows;
  rw.pr = rows.pr + int64_t(b) * pred_ld;
  if (tid == 0) {
    if (carry) {
      s_p = carry[b];
      s_k = 0;
    } else {  // Statistics.mean / Base.sum over a generator: the first loss starts the fold
      s_p = n > 0 ? rw(0) : T(0);
      s_k = n > 0 ? 1 : 0;
    }
  }
  int slow = 0;
  if (seg_len <= 0) {
    sr_fold_range<T, R>(rw, n, &s_p, &s_k, s_w0, s_w1);
  } else {
    for (int64_t sb = 0; sb < n_seg; sb += SB) {
      const int nb = int(n_seg - sb < SB ? n_seg - sb : SB);
      __syncthreads();  // (thread 0 is done with the previous batch's tables)
      for (int i = tid; i < nb; i += 1024) s_tq[i] = tq[int64_t(b) * n_seg + sb + i];
      for (int i = tid; i < 4 * nb; i += 1024) s_tab[i] = tab[4 * (int64_t(b) * n_seg + sb) + i];
      __syncthreads();
      int64_t s = sb;
      bool stop = false;
      while (s < sb + nb) {
        if (tid == 0) {  // O(1) advances through the segments the tables cover
          T p = s_p;
          int64_t k = s_k, sg = s;
          for (; sg < sb + nb; ++sg) {
            if (!(p <= SrM<T>::big)) break;
            const int64_t lo = sg * seg_len, hi = lo + seg_len < n ? lo + seg_len : n;
            if (k != lo) break;  // (the first segment without a carry starts at row 1)
            int q;
            int64_t lim;
            if (p < MIN_NORMAL) {
              q = Tr::qmin;
              lim = int64_t(1) << Tr::mant;
            } else {
              int ex;
              (void)frexp(double(p), &ex);
              q = ex - 1 - Tr::mant;
              lim = int64_t(1) << (Tr::mant + 1);
            }
            const int2 qq = s_tq[sg - sb];
            const int j = q == qq.x ? 0 : (q == qq.y ? 2 : -1);
            if (j < 0) break;
            const int64_t P = int64_t(ldexp(double(p), -q));
            const int64_t g = s_tab[4 * (sg - sb) + j + int(P & 1)];
            if (P + g >= lim) break;  // the fold crosses a binade inside this segment
            p = T(ldexp(double(P + g), q));
            k = hi;
          }
          s_p = p;
          s_k = k;
          s_seg = sg;
        }
        __syncthreads();
        const int64_t sg = s_seg;
        const T p = s_p;
        __syncthreads();
        if (!(p <= SrM<T>::big)) {
          stop = true;
          break;
        }
        if (sg >= sb + nb) break;
        const int64_t hi = sg * seg_len + seg_len < n ? sg * seg_len + seg_len : n;
        sr_fold_range<T, R>(rw, hi, &s_p, &s_k, s_w0, s_w1);  // this segment, exactly
        ++slow;
        s = sg + 1;
      }
      if (stop) break;
    }
  }
  __syncthreads();
  if (tid == 0) {
    out[b] = s_p;
    if (n_slow) n_slow[b] = slow;
  }
}

template <typename T>
hipError_t sr_launch_fold_segsum(const T* pred, int64_t pred_ld, int n_trees, const T* y, const T* w,
                                 const int64_t* row_idx, int64_t n, int loss_kind, T loss_param, int64_t seg_len,
                                 double* segsum, hipStream_t s) {
  if (n_trees <= 0 || seg_len <= 0 || n <= 0) return hipSuccess;
  const int n_seg = int((n + seg_len - 1) / seg_len);
  const SrFoldRows<T> rows{pred, y, w, row_idx, loss_kind, loss_param};
  hipLaunchKernelGGL(sr_fold_segsum_kernel<T>, dim3(unsigned(n_seg), unsigned(n_trees)), dim3(256), 0, s, rows, pred_ld,
                     n, seg_len, n_seg, segsum);
  return hipGetLastError();
}
template <typename T>
hipError_t sr_launch_fold_segtab(const T* pred, int64_t pred_ld, int n_trees, const T* y, const T* w,
                                 const int64_t* row_idx, int64_t n, int loss_kind, T loss_param, int64_t seg_len,
                                 const double* segsum, const double* carry_est, int2* tq, int64_t* tab, hipStream_t s) {
  if (n_trees <= 0 || seg_len <= 0 || n <= 0) return hipSuccess;
  const int n_seg = int((n + seg_len - 1) / seg_len);
  const SrFoldRows<T> rows{pred, y, w, row_idx, loss_kind, loss_param};
  hipLaunchKernelGGL((sr_fold_segtab_kernel<T, 16>), dim3(unsigned(n_seg), unsigned(n_trees)), dim3(256), 0, s, rows,
                     pred_ld, n, seg_len, n_seg, segsum, carry_est, tq, tab);
  return hipGetLastError();
}
template <typename T>
hipError_t sr_launch_fold(const T* pred, int64_t pred_ld, int n_trees, const T* y, const T* w, const int64_t* row_idx,
                          int64_t n, int loss_kind, T loss_param, int64_t seg_len, const int2* tq, const int64_t* tab,
                          const T* carry, T* out, int* n_slow, hipStream_t s) {
  if (n_trees <= 0) return hipSuccess;
  const int n_seg = seg_len > 0 ? int((n + seg_len - 1) / seg_len) : 0;
  const SrFoldRows<T> rows{pred, y, w, row_idx, loss_kind, loss_param};
  hipLaunchKernelGGL((sr_fold_chain_kernel<T, 8>), dim3(unsigned(n_trees)), dim3(1024), 0, s, rows, pred_ld, n,
                     seg_len, n_seg, tq, tab, carry, out, n_slow);
  return hipGetLastError();
}
template hipError_t sr_launch_fold_segsum<float>(const float*, int64_t, int, const float*, const float*, const int64_t*,
                                                 int64_t, int, float, int64_t, double*, hipStream_t);
template hipError_t sr_launch_fold_segsum<double>(const double*, int64_t, int, const double*, const double*,
                                                  const int64_t*, int64_t, int, double, int64_t, double*, hipStream_t);
template hipError_t sr_launch_fold_segtab<float>(const float*, int64_t, int, const float*, const float*, const int64_t*,
                                                 int64_t, int, float, int64_t, const double*, const double*, int2*,
                                                 int64_t*, hipStream_t);
template hipError_t sr_launch_fold_segtab<double>(const double*, int64_t, int, const double*, const double*,
                                                  const int64_t*, int64_t, int, double, int64_t, const double*,
                                                  const double*, int2*, int64_t*, hipStream_t);
template hipError_t sr_launch_fold<float>(const float*, int64_t, int, const float*, const float*, const int64_t*, int64_t,
                                          int, float, int64_t, const int2*, const int64_t*, const float*, float*, int*,
                                          hipStream_t);
template hipError_t sr_launch_fold<double>(const double*, int64_t, int, const double*, const double*, const int64_t*,
                                           int64_t, int, double, int64_t, const int2*, const int64_t*, const double*,
                                           double*, int*, hipStream_t);

// ---------------------------------------------------------------- every complete tree's fold (round 6)
// The reference's loss of a complete tree IS the in-order fold in T (LossFunctions.jl:38-58), not the
// f64 sum (at 2^20 rows the two differ by ~5e-4 relative, past north_star's 1e-4).  The call's loss
// launch already leaves one f64 partial per (row block, tree); a row block is a fold segment:
//   plan   the f64 prefix before and after each segment (from those partials) brackets the fold's value
//          there within a relative window delta; a segment whose window lies in ONE binade gets that
//          binade's composed step (code q), the first segment and every segment whose window meets a
//          binade edge are slow (their losses are kept, code SLOT0 + slot);
//   steps  small calls: the loss launch stored every tree's losses, and sr_fold_stab_kernel composes
//          each segment's steps from them; large calls: the interpreter runs the complete trees again in
//          FOLD mode (sr_tile_impl.h), composing each tile's steps in registers and storing only the slow
//          segments' losses (plan: sr_fold_plan_kernel, slots from a call-wide counter);
//   walk   one workgroup per tree walks the segments in order: a steps segment advances in O(1) when
//          the running value is in its binade and stays there, a slow one is folded row by row by the
//          workgroup scan (sr_fold_range); anything else fails the tree (SR_FST_FAIL), which the host
//          folds through the prediction pass instead (fold_exact).
// Every O(1) advance is an exact composition, so the result is the reference's fold bit for bit whatever
// the window; delta only trades slow segments against failures.

// A segment's stored losses (the loss launch's store or a FOLD slot): row i of the view at base[i - lo].
template <typename T>
struct SrStoredRows {
  const T* base;
  int64_t lo;
  __device__ __forceinline__ T operator()(int64_t i) const { return base[i - lo]; }
  template <int R>
  __device__ __forceinline__ void rows_from(int64_t r0, int64_t hi, T (&ev)[R]) const {
    constexpr int C = 16 / int(sizeof(T));
    using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
    const T* p = base + (r0 - lo);
    if (r0 + R <= hi && (reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
#pragma unroll
      for (int c = 0; c < R / C; ++c) {
        const V v = *reinterpret_cast<const V*>(p + c * C);
#pragma unroll
        for (int j = 0; j < C; ++j) ev[c * C + j] = reinterpret_cast<const T*>(&v)[j];
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) ev[r] = (r0 + r < hi) ? p[r] : T(0);
    }
  }
};

// Large calls: one wave per launch position; codes [rb][np] (slots of the FOLD mode's slow segments
// from the call's counter; past slot_cap a slow segment gets SKIP, which fails its tree in the walk).
template <typename T>
__global__ void __launch_bounds__(256) sr_fold_plan_kernel(const double* __restrict__ part, int np, int n_rb,
                                                           const uint32_t* __restrict__ perm, SrFoldWho who,
                                                           double delta, SrFoldTabs ft, int* __restrict__ slot_next,
                                                           int slot_cap) {
  const int lane = int(threadIdx.x) & 63;
  const int p = int(blockIdx.x) * 4 + int(threadIdx.x) / 64;
  if (p >= np) return;  // wave-uniform
  const uint32_t t = perm ? perm[p] : uint32_t(p);
  const bool ok = who.eligible<T>(t);
  double run = who.est ? who.est[t] : 0.0;  // (a row shard after the first: the shards before it)
  // (any tree's fold drifts from the f64 prefix more the longer it is: ~2e-3 at most over C2's trees at
  //  2^20 rows, 4x that at 2^22 — the 4-rank rehearsal's 243 fallbacks at 2^-8 — so the window is at least
  //  n 2^-28: 2^-8 up to 2^20 rows, 2^-5 at 2^23)
  {
    const double len_w = double(who.n_terms) * 3.725290298461914e-09;
    if (delta < len_w) delta = len_w < 0.0625 ? len_w : 0.0625;
  }
  // A tree whose losses hardly vary — a huge constant tree, (c - y)^2 with |c| >> |y| — drifts from the
  // f64 prefix systematically: once the running value's ulp exceeds the losses' spread, every step
  // rounds the same way (up to ~1 % at 2^20 rows: C2's failed walks, round 6).  Its window is widened to
  // n 2^-26 (at least 2^-5, at most 2^-2) when its full row blocks' sums agree to 2^-7 (a tree with
  // varied losses: ~10 %; the last block may be shorter and is left out).
  if (ok && part && n_rb >= 3) {
    double mn = 1.7976931348623157e308, mx = 0.0;
    for (int rb = lane; rb < n_rb - 1; rb += 64) {
      const double v = part[size_t(rb) * size_t(np) + size_t(p)];
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    // (the drift grows with the fold's length: ~1 % at 2^20 rows, ~8 % at 2^23)
    const double wide = double(who.n_terms) * 1.4901161193847656e-08 < 0.03125 ? 0.03125
                        : (double(who.n_terms) * 1.4901161193847656e-08 > 0.25 ? 0.25
                                                                               : double(who.n_terms) * 1.4901161193847656e-08);
    if (mx <= mn * (1.0 + 0.0078125) && delta < wide) delta = wide;
  }
  for (int c0 = 0; c0 < n_rb; c0 += 64) {
    const int rb = c0 + lane;
    const bool in = rb < n_rb;
    // (one row block: its sum is the tree's total on this view)
    const double v = !(ok && in) ? 0.0 : (part ? part[size_t(rb) * size_t(np) + size_t(p)] : who.sums[t]);
    double inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double o = __shfl_up(inc, off, 64);
      if (lane >= off) inc += o;
    }
    const double sb = run + (inc - v), sa = run + inc;  // (estimates: they only choose binades)
    run += __shfl(inc, 63, 64);
    int32_t cd = SR_FCODE_SKIP, sqv = SR_FCODE_SKIP;
    bool slow = false;
    if (ok && in) {
      const int qa = sr_fold_q<T>(sb * (1.0 - delta));
      const bool first = rb == 0 && who.first;
      slow = first || qa != sr_fold_q<T>(sa * (1.0 + delta));
      cd = qa;
      if (slow && !first) sqv = qa;  // (the FOLD pass composes its steps under qa and qa + 1 too)
    }
    const uint64_t sm = __builtin_amdgcn_ballot_w64(slow);
    if (sm) {
      int base = 0;
      if (lane == 0) base = atomicAdd(slot_next, __popcll(sm));
      base = __shfl(base, 0, 64);
      const int k = base + __popcll(sm & ((uint64_t(1) << lane) - 1u));
      if (slow) cd = k < slot_cap ? SR_FCODE_SLOT0 + k : SR_FCODE_SKIP;
    }
    if (in) {
      ft.code[size_t(rb) * size_t(np) + size_t(p)] = cd;
      ft.sq[size_t(rb) * size_t(np) + size_t(p)] = sqv;
    }
  }
}

// The fold's first rows one by one (Statistics.mean / Base.sum over a generator: the first loss starts
// the fold), in the hardware's own adds — the running value leaves a binade every few rows here, so a
// round per crossing would cost ~1 us each.  Rows [0, ks), ks <= 256, of a stored segment b; one wave
// (64 lanes): through LDS, lane 0 reads its rows ahead of the adds, 8 at a time (a readlane per row
// costs ~100 cycles of hazards, 11 us for 256 rows).  Wave-uniform result.  The walk's serial start
// and, for stored-loss calls, the pair kernel's first-segment wave (off the walk's critical path).
template <typename T>
__device__ __forceinline__ T sr_fold_serial_start(const T* __restrict__ b, int ks, int lane) {
  __shared__ T s_first[256];
#pragma unroll
  for (int j = 0; j < 4; ++j) s_first[4 * lane + j] = (4 * lane + j < ks) ? b[4 * lane + j] : T(0);
  __syncthreads();
  T f0 = T(0);
  if (lane == 0) {
    f0 = s_first[0];
    int r = 1;
    for (; r + 8 <= ks; r += 8) {
      T u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = s_first[r + j];
#pragma unroll
      for (int j = 0; j < 8; ++j) f0 = f0 + u[j];
    }
    for (; r < ks; ++r) f0 = f0 + s_first[r];
  }
  return sr_fold_lane(f0, 0);
}
template <typename T>
__device__ __forceinline__ int sr_fold_serial_rows(int64_t rb_rows, int64_t n) {
  const int64_t m = rb_rows < n ? rb_rows : n;
  return int(m < 256 ? m : 256);
}

// Small calls: the loss launch stored every position's losses ([position][pos_stride], pos_stride =
// n_rb x rb_rows, so segment rb of position p is slot p n_rb + rb); one wave per (segment, position)
// decides its code and composes a steps segment's pair in row order (a slow segment's under its lower
// window binade and the next).  (One wave, no barriers: round 6 measured the 256-thread form at ~11 us
// a search call, most of it barriers and idle waves for 512-row segments.)
template <typename T, int R>
__device__ typename SrFoldTab<T>::Pair sr_fold_stab_pair_wave(const SrStoredRows<T>& rw, int64_t lo, int64_t hi, int q,
                                                              int lane) {
  using I = typename SrFoldTab<T>::I;
  constexpr I CAP = I(1) << (SrFoldTraits<T>::mant + 3);
  I ta0 = 0, ta1 = 0;  // the segment so far (uniform)
  for (int64_t base = lo; base < hi; base += 64 * R) {
    I a0 = 0, a1 = 0;
    T ev[R];
    rw.template rows_from<R>(base + int64_t(lane) * R, hi, ev);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      I m;
      int kind;
      SrFoldTab<T>::step(ev[r], q, m, kind);
      sr_fold_add_i<I>(m, kind, CAP, a0, a1);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // ordered over the lanes: lane 0 ends with the pass
      I o0 = __shfl_down(a0, off, 64), o1 = __shfl_down(a1, off, 64);
      if ((lane & (2 * off - 1)) == 0) {
        sr_fold_compose_i<I>(a0, a1, o0, o1, CAP);
        a0 = o0;
        a1 = o1;
      }
    }
    I y0 = sr_fold_lane(a0, 0), y1 = sr_fold_lane(a1, 0);
    sr_fold_compose_i<I>(ta0, ta1, y0, y1, CAP);
    ta0 = y0;
    ta1 = y1;
  }
  return SrFoldTab<T>::pair(ta0, ta1);
}
template <typename T, int R>
__global__ void __launch_bounds__(64) sr_fold_stab_kernel(const double* __restrict__ part, int np, int n_rb,
                                                          int64_t rb_rows, int64_t n, const uint32_t* __restrict__ perm,
                                                          SrFoldWho who, double delta, const T* __restrict__ losses,
                                                          SrFoldTabs ft, const uint32_t* __restrict__ part_flag,
                                                          const uint8_t* __restrict__ static_bad,
                                                          double* __restrict__ red_sum, uint32_t* __restrict__ red_flag) {
  using Pair = typename SrFoldTab<T>::Pair;
  int32_t* __restrict__ code = ft.code;
  const int rb = int(blockIdx.x), p = int(blockIdx.y), lane = int(threadIdx.x);
  const uint32_t t = perm ? perm[p] : uint32_t(p);
  const size_t o = size_t(rb) * size_t(np) + size_t(p);
  bool elig;
  if (red_sum) {
    // the call's reduce, here instead of its own launch: every wave of the tree folds the partials with
    // the reduce launch's arithmetic (sr_reduce_positions: lane-strided in order, then the xor
    // butterfly), so all agree bit for bit; the first segment's wave writes the tree's Σ and flags
    double S = 0.0;
    uint32_t fl = 0u;
    for (int i = lane; i < n_rb; i += 64) {
      const size_t oi = size_t(i) * size_t(np) + size_t(p);
      S += part[oi];
      fl |= part_flag[oi];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      S += __shfl_xor(S, off, 64);
      fl |= __shfl_xor(fl, off, 64);
    }
    if (static_bad && static_bad[t]) fl |= SR_FLAG_STATIC | SR_FLAG_NONFINITE;
    if (rb == 0 && lane == 0) {
      red_sum[t] = S;
      red_flag[t] = fl;
    }
    elig = sr_fold_eligible<T>(S, fl, who.n_terms);
  } else {
    elig = who.eligible<T>(t);
  }
  if (!elig) {
    if (lane == 0) {
      code[o] = SR_FCODE_SKIP;
      ft.sq[o] = SR_FCODE_SKIP;
    }
    return;
  }
  const int32_t slow_code = SR_FCODE_SLOT0 + p * n_rb + rb;
  if (rb == 0 && who.first) {
    // the fold's start: its first rows one by one, here (the walk reads the value from the segment's
    // pair slot, so its critical path skips them)
    const T f0 = n > 0 ? sr_fold_serial_start<T>(losses + size_t(p) * size_t(n_rb) * size_t(rb_rows),
                                                 sr_fold_serial_rows<T>(rb_rows, n), lane)
                       : T(0);
    if (lane == 0) {
      code[o] = slow_code;
      ft.sq[o] = SR_FCODE_SKIP;
      *reinterpret_cast<T*>(static_cast<Pair*>(ft.tab) + o) = f0;
    }
    return;
  }
  double pre = 0.0;
  for (int i = lane; i < rb; i += 64) pre += part[size_t(i) * size_t(np) + size_t(p)];  // (rb > 0: part is set)
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) pre += __shfl_xor(pre, off, 64);
  const double sb = (who.est ? who.est[t] : 0.0) + pre;  // (an estimate: it only chooses binades)
  const double sa = sb + (part ? part[o] : who.sums[t]);  // (one row block: the view's total; no fused reduce)
  const int q = sr_fold_q<T>(sb * (1.0 - delta));
  const bool slow = q != sr_fold_q<T>(sa * (1.0 + delta));
  const int64_t lo = int64_t(rb) * rb_rows, hi = lo + rb_rows < n ? lo + rb_rows : n;
  const SrStoredRows<T> rw{losses + (size_t(p) * size_t(n_rb) + size_t(rb)) * size_t(rb_rows), lo};
  // a steps segment's pair under q; a slow segment's under q and q + 1 (the walk uses them when the
  // running value stays in one binade there after all)
  const Pair pr = sr_fold_stab_pair_wave<T, R>(rw, lo, hi, q, lane);
  if (lane == 0) static_cast<Pair*>(ft.tab)[o] = pr;
  if (slow) {
    const Pair pr2 = sr_fold_stab_pair_wave<T, R>(rw, lo, hi, q + 1, lane);
    if (lane == 0) static_cast<Pair*>(ft.tab2)[o] = pr2;
  }
  if (lane == 0) {
    code[o] = slow ? slow_code : q;
    ft.sq[o] = slow ? q : SR_FCODE_SKIP;
  }
}
// One pass of a slow segment: 64 x RW rows from b0 (16-byte aligned in the segment's storage, row i at
// base[i - lo]), lane l holding rows b0 + l RW ...  Branch-free and unmasked: a chunk past the view
// loads the view's last chunk (a valid address) and the rows at or past hi are masked where they are
// used, so the loads stay in flight until then (a load under a branch, or one whose value is selected
// right away, waits at once).
template <typename T, int RW>
__device__ __forceinline__ void sr_fold_load(const T* __restrict__ base, int64_t lo, int64_t b0, int64_t hi, int lane,
                                             T (&ev)[RW]) {
  constexpr int C = 16 / int(sizeof(T));
  using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
  const int64_t r0 = b0 + int64_t(lane) * RW;
  const int64_t last = hi - 1 - ((hi - 1 - lo) % C);
#pragma unroll
  for (int c = 0; c < RW / C; ++c) {
    const int64_t rc = r0 + c * C;
    const V v = *reinterpret_cast<const V*>(base + ((rc < last ? rc : last) - lo));
#pragma unroll
    for (int j = 0; j < C; ++j) ev[c * C + j] = reinterpret_cast<const T*>(&v)[j];
  }
}

// One wave folds rows [k, hi) of a slow segment into F exactly (row i's loss at base[i - lo]), 64 x RW
// rows per pass: each lane holds RW consecutive rows.  Per round, under the binade of F: every row's
// step, each lane's composition, an ordered inclusive scan over the lanes; a round that leaves the
// binade ends at the first row whose step reaches it (that lane re-walks its rows from its exclusive
// prefix), the hardware add takes that row, and the next round continues in the SAME registers from the
// row after it (rows before k are identity steps) until the pass is used up.  Fast path (no row of the
// round at an exact half ulp): every step is rint(l 2^-q) whatever the parity, so the compositions are
// plain sums (a DPP scan in T: exact below the binade's limit, monotone past it); otherwise the pair
// composition (sr_fold_add_i / sr_fold_compose_i).
// Software pipelining: ev holds the pass at k's 16-byte boundary on entry (k is the segment's first row
// or row 1); each pass first issues the load of the next one — the segment's next pass, else the first
// pass of the next slow segment (nbase, rows [nlo, nhi); NULL: none) — into nx, so its latency hides
// behind this pass's rounds.  On return ev holds the next slow segment's first pass when nbase was set.
template <typename T, int RW>
__device__ T sr_fold_rows_wave(const T* __restrict__ base, int64_t lo, int64_t k, int64_t hi, T F, int lane,
                               int& rounds, T (&ev)[RW], const T* __restrict__ nbase, int64_t nlo, int64_t nhi) {
  using Tr = SrFoldTraits<T>;
  using I = typename SrFoldTab<T>::I;
  constexpr I CAP = I(1) << (Tr::mant + 3);
  constexpr T CLAMP = T(int64_t(1) << (Tr::mant + 2));
  constexpr int C = 16 / int(sizeof(T));
  T nx[RW];
  while (k < hi) {
    const int64_t b0 = k - ((k - lo) % C);
    const int64_t r0 = b0 + int64_t(lane) * RW;
    const int64_t pass_end = b0 + int64_t(64) * RW;
    {  // (one unconditional load: no next pass re-loads this one)
      const bool same = pass_end < hi;
      const T* pb = same ? base : (nbase ? nbase : base);
      const int64_t plo = same ? lo : (nbase ? nlo : lo), pb0 = same ? pass_end : (nbase ? nlo : b0),
                    phi = same ? hi : (nbase ? nhi : hi);
      sr_fold_load<T, RW>(pb, plo, pb0, phi, lane, nx);
    }
    // the pass's rows before k and at or past hi are identity steps: zeroed once here, and the rows up to
    // each crossing once after it (the rounds read ev as it is)
    {
      const int64_t dk = k - r0, dh = hi - r0;
      const int rk = dk < 0 ? 0 : (dk > RW ? RW : int(dk)), rh = dh < 0 ? 0 : (dh > RW ? RW : int(dh));
#pragma unroll
      for (int r = 0; r < RW; ++r) ev[r] = (r >= rk && r < rh) ? ev[r] : T(0);
    }
    while (k < hi && k < pass_end) {
      ++rounds;
      if (!(F <= SrM<T>::big)) return F;  // +Inf / NaN stays
      const SrFoldBinade<T> bn(F);
      const int q = bn.q;
      const I P = bn.P, lim = bn.lim;
      const bool odd = (P & 1) != 0;
      // fast path: the round's steps are rint(l 2^-q) unless some row is an exact half (6 VALU a row:
      // scale, round, residual, max |residual|, clamp, sum; a NaN loss clamps, its residual is ignored)
      T sr[RW];
      T lsum = T(0), dmax = T(0);
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const T v = sizeof(T) == 4 ? T(ldexpf(float(ev[r]), -q)) : T(ldexp(double(ev[r]), -q));
        const T st = sizeof(T) == 4 ? T(rintf(float(v))) : T(rint(double(v)));
        dmax = sizeof(T) == 4 ? T(fmaxf(float(dmax), fabsf(float(v - st)))) : T(fmax(double(dmax), fabs(double(v - st))));
        sr[r] = sizeof(T) == 4 ? T(fminf(float(st), float(CLAMP))) : T(fmin(double(st), double(CLAMP)));
        lsum += sr[r];
      }
      const bool fast = __builtin_amdgcn_ballot_w64(dmax == T(0.5)) == 0;
      uint64_t cross;
      I xp = 0;  // the crossing lane's exclusive prefix (from the parity of P)
      int cl = 0;
      if (fast) {
        const T inc = sr_fold_scan(lsum);
        cross = __builtin_amdgcn_ballot_w64(T(P) + inc >= T(lim));
        if (cross == 0) {  // the rest of this pass stays in the binade
          F = SrFoldBinade<T>::value(P + I(sr_fold_lane(inc, 63)), q);
          k = pass_end;
          break;
        }
        cl = __builtin_ctzll(cross);
        // (the prefix before the first lane that leaves the binade is exact)
        if (cl > 0) xp = I(sr_fold_lane(inc, cl - 1));
      } else {
        I i0 = 0, i1 = 0;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          I m;
          int kind;
          SrFoldTab<T>::step(ev[r], q, m, kind);
          sr_fold_add_i<I>(m, kind, CAP, i0, i1);
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const I l0 = __shfl_up(i0, off, 64), l1 = __shfl_up(i1, off, 64);
          if (lane >= off) sr_fold_compose_i<I>(l0, l1, i0, i1, CAP);
        }
        const I inc = P + (odd ? i1 : i0);
        cross = __builtin_amdgcn_ballot_w64(inc >= lim);
        if (cross == 0) {
          F = SrFoldBinade<T>::value(sr_fold_lane(inc, 63), q);
          k = pass_end;
          break;
        }
        cl = __builtin_ctzll(cross);
        const I x0 = sr_fold_lane(i0, cl > 0 ? cl - 1 : 0), x1 = sr_fold_lane(i1, cl > 0 ? cl - 1 : 0);
        if (cl > 0) xp = odd ? x1 : x0;
      }
      // the lane whose rows leave the binade
      T nF = T(0);
      int64_t nk = 0;
      if (lane == cl) {
        I run = P + xp;
        bool done = false;
        nF = T(__builtin_nan(""));  // (not reached: the lane's rows do leave the binade)
        nk = pass_end;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const T e = ev[r];
          I d;
          if (fast) {
            d = I(sr[r]);
          } else {
            I m;
            int kind;
            SrFoldTab<T>::step(e, q, m, kind);
            d = m + (kind == 2 ? 1 : (kind == 1 ? ((run + m) & 1) : 0));
          }
          if (!done && run + d >= lim) {
            nF = SrFoldBinade<T>::value(run, q) + e;  // the hardware's own rounding of this step
            nk = r0 + r + 1;
            done = true;
          }
          if (!done) run += d;
        }
      }
      F = sr_fold_lane(nF, cl);
      k = sr_fold_lane(nk, cl);
      {  // the rows up to the crossing are done
        const int64_t dk = k - r0;
        const int rk = dk < 0 ? 0 : (dk > RW ? RW : int(dk));
#pragma unroll
        for (int r = 0; r < RW; ++r) ev[r] = r >= rk ? ev[r] : T(0);
      }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) ev[r] = nx[r];
  }
  return F;
}

// The walk: one wave per launch position (one per workgroup), its segments in row order, 64 at a time.
// Between two slow segments the steps segments share one binade (adjacent windows cannot straddle
// apart), so each such run is ONE composition — a segmented ordered scan of the chunk's pairs over the
// lanes — checked against the running value once: its binade must be the run's and the run must end
// inside it.  A slow segment is folded by sr_fold_rows_wave.  Anything else fails the tree.  carry (at
// the caller's tree index): the fold's value before this view's first row (a row shard after the
// first), or NULL: the first loss starts the fold.  out_val / out_st at the caller's tree index.
template <typename T, int RW>
__global__ void __launch_bounds__(64) sr_fold_walk_kernel(SrFoldTabs ft, SrFoldWho who, int np, int n_rb,
                                                           int64_t rb_rows, int64_t n,
                                                           const T* __restrict__ losses, int64_t slot_rows,
                                                           const uint32_t* __restrict__ perm,
                                                           const T* __restrict__ carry, T* __restrict__ out_val,
                                                           int32_t* __restrict__ out_st, int4* __restrict__ dbg,
                                                           int all_rows) {
  using Tr = SrFoldTraits<T>;
  using I = typename SrFoldTab<T>::I;
  using Pair = typename SrFoldTab<T>::Pair;
  constexpr I CAP = I(1) << (Tr::mant + 3);
  const int32_t* __restrict__ code = ft.code;
  const Pair* __restrict__ tab = static_cast<const Pair*>(ft.tab);
  const Pair* __restrict__ tab2 = static_cast<const Pair*>(ft.tab2);
  const int lane = int(threadIdx.x) & 63;
  const uint64_t clk0 = dbg ? wall_clock64() : 0;
  int n_slow = 0, n_rounds = 0, n_skip = 0;  // (SR_AMD_FOLD_STATS: per-tree walk statistics)
  uint64_t slow_clk = 0;
  const int p = int(blockIdx.x);  // (one wave per workgroup: a finished walk frees its slot at once)
  if (p >= np) return;  // wave-uniform
  const uint32_t t = perm ? perm[p] : uint32_t(p);
  if (who.msum && lane == 0) {  // (every position of the call has its walk workgroup, skipped trees too)
    who.msum[t] = who.sums[t];
    who.mflag[t] = who.flags[t];
  }
  // (all_rows & 16: a call of one row block of at most 256 rows with its losses kept — the serial start
  //  is the whole fold, and no pair kernel ran: eligibility from the call's flags, slot p)
  const bool tiny = (all_rows & 16) != 0;
  const int32_t c_first = tiny ? (who.eligible<T>(t) ? SR_FCODE_SLOT0 + p : SR_FCODE_SKIP) : code[p];
  if (c_first == SR_FCODE_SKIP) {
    if (lane == 0) out_st[t] = SR_FST_NONE;
    return;
  }
  auto seg_base = [&](int32_t c) { return losses + size_t(c - SR_FCODE_SLOT0) * size_t(slot_rows); };
  bool fail = false;
  int why = 0;  // (SR_AMD_FOLD_STATS: the failure site)
  T F = T(0);
  int64_t k = 0;
  if (carry) {
    F = carry[t];
  } else if (c_first >= SR_FCODE_SLOT0 && n > 0 && (all_rows & 4)) {  // (debug: no serial start)
    F = seg_base(c_first)[0];
    k = 1;
  } else if (c_first >= SR_FCODE_SLOT0 && n > 0 && (all_rows & 32)) {  // (the pair kernel's serial start)
    F = *reinterpret_cast<const T*>(tab + p);
    k = sr_fold_serial_rows<T>(rb_rows, n);
  } else if (c_first >= SR_FCODE_SLOT0 && n > 0) {  // the first rows one by one (sr_fold_serial_start)
    F = sr_fold_serial_start<T>(seg_base(c_first), sr_fold_serial_rows<T>(rb_rows, n), lane);
    k = sr_fold_serial_rows<T>(rb_rows, n);
  } else {
    fail = n > 0;  // (the plan keeps the first segment's losses)
    why = 1;
  }
  T ev[RW];  // a slow segment's current pass (have: ev holds the next slow segment's first pass)
  bool have = false;
  // the chunk's four arrays in one round trip (unconditional loads at a valid index, then selects: a
  // load under a branch on another load's value costs a second round trip), the next chunk's issued
  // at the start of this one
  if (tiny) {  // (k == n: the serial start folded every row)
    if (lane == 0) {
      out_val[t] = F;
      out_st[t] = fail ? SR_FST_FAIL : SR_FST_OK;
      if (dbg) dbg[t] = make_int4(1000, 0, 0, int((wall_clock64() - clk0) / 100));
    }
    return;
  }
  auto chunk_at = [&](int c) { return size_t(c + lane < n_rb ? c + lane : n_rb - 1) * size_t(np) + size_t(p); };
  size_t so_n = chunk_at(0);
  int32_t cd_n = code[so_n], sq_n = ft.sq[so_n];
  Pair pa_n = tab[so_n], pb_n = tab2[so_n];
  for (int c0 = 0; c0 < n_rb && !fail; c0 += 64) {
    have = false;
    const int sg = c0 + lane;
    const bool in = sg < n_rb;
    const int32_t cd_l = cd_n, sq_l = sq_n;
    const Pair pa = pa_n, pb = pb_n;
    if (c0 + 64 < n_rb) {
      so_n = chunk_at(c0 + 64);
      cd_n = code[so_n];
      sq_n = ft.sq[so_n];
      pa_n = tab[so_n];
      pb_n = tab2[so_n];
    }
    const int32_t cd = in ? cd_l : SR_FCODE_SKIP;
    const bool slow = in && cd >= SR_FCODE_SLOT0;
    // a steps segment's pair; a slow segment's lower window binade and its steps under that binade
    // (s0, s1) and the next (u0, u1)
    const bool steps = in && !slow && cd != SR_FCODE_SKIP;
    I x0 = steps ? I(pa.x) : I(0), x1 = steps ? I(pa.y) : I(0);
    const int32_t sq = slow ? sq_l : SR_FCODE_SKIP;
    const bool has2 = sq != SR_FCODE_SKIP;
    const I s0 = has2 ? I(pa.x) : I(0), s1 = has2 ? I(pa.y) : I(0);
    const I u0 = has2 ? I(pb.x) : I(0), u1 = has2 ? I(pb.y) : I(0);
    if (__builtin_amdgcn_ballot_w64(in && cd == SR_FCODE_SKIP)) {  // (a plan out of slots)
      fail = true;
      why = 2;
      break;
    }
    const uint64_t slowm = __builtin_amdgcn_ballot_w64(slow);
    // segmented inclusive scan: a run starts at the chunk's first lane and after each slow lane
    bool head = lane == 0 || (lane > 0 && ((slowm >> (lane - 1)) & 1u));
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const I l0 = __shfl_up(x0, off, 64), l1 = __shfl_up(x1, off, 64);
      const bool lh = __shfl_up(int(head), off, 64) != 0;
      if (lane >= off && !head) {
        sr_fold_compose_i<I>(l0, l1, x0, x1, CAP);
        head = lh;
      }
    }
    const int end = n_rb - c0 < 64 ? n_rb - c0 : 64;
    int pos = 0;
    while (pos < end && !fail) {
      const int64_t lo = int64_t(c0 + pos) * rb_rows;
      if ((slowm >> pos) & 1u) {  // a slow segment, row by row
        const int32_t c = sr_fold_lane(cd, pos);
        const int64_t hi = lo + rb_rows < n ? lo + rb_rows : n;
        if (k < lo || k > hi) {
          fail = true;
          why = 3;
          break;
        }
        {  // the running value may not leave a binade in this segment after all: its composed steps
          const int32_t q0 = sr_fold_lane(sq, pos);
          if (k == lo && q0 != SR_FCODE_SKIP && F <= SrM<T>::big && !(all_rows & 2)) {
            const SrFoldBinade<T> bn(F);
            const int qf = bn.q;
            const I P = bn.P, lim = bn.lim;
            const bool odd = (P & 1) != 0;
            const I ga = sr_fold_lane(odd ? s1 : s0, pos), gb = sr_fold_lane(odd ? u1 : u0, pos);
            const I g = qf == q0 ? ga : (qf == q0 + 1 ? gb : lim);
            if (P + g < lim) {
              F = SrFoldBinade<T>::value(P + g, qf);
              k = hi;
              have = false;  // (ev held this segment's prefetched rows)
              ++n_skip;
              ++pos;
              continue;
            }
          }
        }
        if (k == hi) {  // (the first block wholly inside the serial start: nothing left here, nothing loaded)
          have = false;
          ++pos;
          continue;
        }
        const int64_t b0 = k - ((k - lo) % (16 / int64_t(sizeof(T))));  // (the pass sr_fold_rows_wave expects)
        if (!have || b0 != lo) sr_fold_load<T, RW>(seg_base(c), lo, b0, hi, lane, ev);
        // the chunk's next slow segment: its first pass is prefetched during this one
        const uint64_t later = (slowm >> pos) >> 1;
        const int np2 = later ? pos + 1 + __builtin_ctzll(later) : 64;
        const T* nbase = nullptr;
        int64_t nlo = 0, nhi = 0;
        if (np2 < end) {
          nbase = seg_base(sr_fold_lane(cd, np2));
          nlo = int64_t(c0 + np2) * rb_rows;
          nhi = nlo + rb_rows < n ? nlo + rb_rows : n;
        }
        const uint64_t cs0 = dbg ? wall_clock64() : 0;
        F = sr_fold_rows_wave<T, RW>(seg_base(c), lo, k, hi, F, lane, n_rounds, ev, nbase, nlo, nhi);
        if (dbg) slow_clk += wall_clock64() - cs0;
        have = nbase != nullptr;
        ++n_slow;
        k = hi;
        if (!(F <= SrM<T>::big)) {  // (an overflow: not the plan's case)
          fail = true;
          why = 4;
        }
        ++pos;
        continue;
      }
      // the run [pos, e): its composition is the scan's value at lane e - 1
      const uint64_t after = (slowm >> pos) >> 1;
      int e = after ? pos + 1 + __builtin_ctzll(after) : end;
      if (e > end) e = end;
      const int32_t q = sr_fold_lane(cd, pos);
      const I g0 = sr_fold_lane(x0, e - 1), g1 = sr_fold_lane(x1, e - 1);
      if (!(F <= SrM<T>::big)) {
        fail = true;
        why = 7;
        break;
      }
      const SrFoldBinade<T> bn(F);
      const int qf = bn.q;
      const I lim = bn.lim;
      const I P = bn.P;
      const I g = (P & 1) ? g1 : g0;
      if (k != lo || qf != q || P + g >= lim) {
        // the running value left the plan's window (it drifted from the f64 prefix past delta), or the
        // fold crosses a binade inside a run the plan called safe: with every row kept (stored losses,
        // slot p n_rb + row block), the run's segments row by row; otherwise the tree fails
        if (!(all_rows & 1) || k != lo) {
          fail = true;
          why = k != lo ? 7 : (qf < q ? 5 : (qf > q ? 6 : 8));
          break;
        }
        for (int s2 = pos; s2 < e && !fail; ++s2) {
          const int64_t l2 = int64_t(c0 + s2) * rb_rows, h2 = l2 + rb_rows < n ? l2 + rb_rows : n;
          const T* b2 = losses + (size_t(p) * size_t(n_rb) + size_t(c0 + s2)) * size_t(slot_rows);
          sr_fold_load<T, RW>(b2, l2, l2, h2, lane, ev);
          F = sr_fold_rows_wave<T, RW>(b2, l2, k, h2, F, lane, n_rounds, ev, nullptr, 0, 0);
          ++n_slow;
          k = h2;
          if (!(F <= SrM<T>::big)) {
            fail = true;
            why = 4;
          }
        }
        have = false;
        pos = e;
        continue;
      }
      F = SrFoldBinade<T>::value(P + g, q);
      const int64_t hl = int64_t(c0 + e) * rb_rows;
      k = hl < n ? hl : n;
      pos = e;
    }
  }
  if (lane == 0) {
    out_val[t] = F;
    out_st[t] = fail ? SR_FST_FAIL : SR_FST_OK;
    if (dbg) dbg[t] = make_int4(n_slow * 1000 + (n_skip < 999 ? n_skip : 999), n_rounds, fail ? -why : int(slow_clk / 100), int((wall_clock64() - clk0) / 100));  // (us: 100 MHz)
  }
}

template <typename T>
hipError_t sr_launch_fold_plan(const double* part, int np, int n_rb, const uint32_t* perm, const SrFoldWho& who,
                               double delta, SrFoldTabs ft, int* slot_next, int slot_cap, hipStream_t s) {
  if (np <= 0) return hipSuccess;
  hipLaunchKernelGGL(sr_fold_plan_kernel<T>, dim3(unsigned((np + 3) / 4)), dim3(256), 0, s, part, np, n_rb, perm, who,
                     delta, ft, slot_next, slot_cap);
  return hipGetLastError();
}
template <typename T>
hipError_t sr_launch_fold_stab(const double* part, int np, int n_rb, int64_t rb_rows, int64_t n, const uint32_t* perm,
                               const SrFoldWho& who, double delta, const T* losses, SrFoldTabs ft,
                               const uint32_t* part_flag, const uint8_t* static_bad, double* red_sum,
                               uint32_t* red_flag, hipStream_t s) {
  if (np <= 0 || n_rb <= 0) return hipSuccess;
  if (red_sum && (part == nullptr || part_flag == nullptr || red_flag == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((sr_fold_stab_kernel<T, 8>), dim3(unsigned(n_rb), unsigned(np)), dim3(64), 0, s, part, np, n_rb,
                     rb_rows, n, perm, who, delta, losses, ft, part_flag, static_bad, red_sum, red_flag);
  return hipGetLastError();
}
template <typename T>
hipError_t sr_launch_fold_walk(SrFoldTabs ft, const SrFoldWho& who, int np, int n_rb, int64_t rb_rows, int64_t n,
                               const T* losses, int64_t slot_rows, const uint32_t* perm, const T* carry, T* out_val,
                               int32_t* out_st, void* dbg, int all_rows, hipStream_t s) {
  if (np <= 0) return hipSuccess;
  // (row blocks of at most 512 rows, e.g. the search's 100k-row calls: half-width passes, half the
  //  per-round work of a crossing block that a 1,024-row pass would spend on idle lanes)
  if (rb_rows <= 512)
    hipLaunchKernelGGL((sr_fold_walk_kernel<T, sizeof(T) == 4 ? 8 : 4>), dim3(unsigned(np)), dim3(64), 0, s, ft, who, np,
                       n_rb, rb_rows, n, losses, slot_rows, perm, carry, out_val, out_st, static_cast<int4*>(dbg),
                       all_rows);
  else
    hipLaunchKernelGGL((sr_fold_walk_kernel<T, sizeof(T) == 4 ? 16 : 8>), dim3(unsigned(np)), dim3(64), 0, s, ft, who,
                       np, n_rb, rb_rows, n, losses, slot_rows, perm, carry, out_val, out_st, static_cast<int4*>(dbg),
                       all_rows);
  return hipGetLastError();
}
#define SR_INSTANTIATE_FOLD2(T)                                                                                      \
  template hipError_t sr_launch_fold_plan<T>(const double*, int, int, const uint32_t*, const SrFoldWho&, double,   \
                                             SrFoldTabs, int*, int, hipStream_t);                                      \
  template hipError_t sr_launch_fold_stab<T>(const double*, int, int, int64_t, int64_t, const uint32_t*,              \
                                             const SrFoldWho&, double, const T*, SrFoldTabs, const uint32_t*,          \
                                             const uint8_t*, double*, uint32_t*, hipStream_t);                         \
  template hipError_t sr_launch_fold_walk<T>(SrFoldTabs, const SrFoldWho&, int, int, int64_t, int64_t, const T*,      \
                                             int64_t, const uint32_t*, const T*, T*, int32_t*, void*, int, hipStream_t);
SR_INSTANTIATE_FOLD2(float)
SR_INSTANTIATE_FOLD2(double)

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
                            const uint32_t* perm, const uint8_t* static_bad, double* out_sum, uint32_t* out_flag,
                            hipStream_t s) {
  if (n_trees <= 0) return hipSuccess;
  const int64_t blocks = (int64_t(n_trees) + 3) / 4;  // 4 waves (trees) per block
  hipLaunchKernelGGL(sr_reduce_partials_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, part_sum, part_flag,
                     n_trees, n_row_blocks, perm, static_bad, out_sum, out_flag);
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

// Rows per lane of each instantiated kernel (sr_inst_*.hip): f32 BASIC 8 (4 for tuning), f32 FULL 4,
// f64 BASIC 4, f64 FULL 2.  `rows_per_lane` <= 0 picks the default.
template <typename T>
int sr_rows_per_lane(int mode, int tier, int requested) {
  const bool basic = mode == SR_MODE_LOSS && tier == SR_TIER_BASIC;
  if (sizeof(T) == 4) {
    if (basic) return (requested == 4 || requested == 16) ? requested : 8;
    return 4;
  }
  return basic ? 4 : 2;
}
template int sr_rows_per_lane<float>(int, int, int);
template int sr_rows_per_lane<double>(int, int, int);

size_t sr_tile_lds_bytes(int elem_size, int nf, int rows_per_lane, int stack_depth, int trees_per_block,
                         int max_checks, int waves, bool weighted, int code_lds) {
  // = SrLdsPlan (sr_tile_impl.h): X tile, y (+ w), LDS stack, EXACT checked values + running sums,
  // program cache (16-byte instructions)
  const size_t rows = size_t(64) * rows_per_lane;
  return size_t(nf) * rows * elem_size + (weighted ? 2 : 1) * rows * elem_size +
         size_t(waves) * stack_depth * rows * elem_size + size_t(waves) * size_t(max_checks) * rows * elem_size +
         (size_t(trees_per_block) * size_t(max_checks) * elem_size + 15) / 16 * 16 + size_t(code_lds) * 16;
}

// Waves per workgroup: the f32 BASIC loss kernel has 4- and 8-wave (L2) builds (SR_AMD_WAVES selects);
// every other kernel runs 4 waves.
int sr_waves_per_block(int elem_size, int mode, int tier, int rows_per_lane, int requested) {
  if (elem_size == 4 && mode == SR_MODE_LOSS && tier == SR_TIER_BASIC && rows_per_lane == 8 && requested == 8)
    return 8;
  return 4;
}

// BASIC-tier loss kernels are built per elementwise loss (the loss code folds away).
template <typename T, int R, bool GATHER, bool VSTK = false>
hipError_t sr_launch_basic_loss(const SrEvalArgs<T>& a, int n_blocks, hipStream_t s) {
  if (a.loss_kind == SR_LOSS_L1)
    return sr_launch_tile<T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, SR_LOSS_L1, VSTK>(a, n_blocks, s);
  if (a.loss_kind == SR_LOSS_L2)
    return sr_launch_tile<T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, SR_LOSS_L2, VSTK>(a, n_blocks, s);
  return sr_launch_tile<T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, -1, VSTK>(a, n_blocks, s);  // other losses
}

// Register-stack kernels (f32 BASIC loss over the full dataset, operand stack in VGPRs): rows per
// lane for a view of n rows, or 0 when the classic LDS-stack kernel should run.  Larger tiles halve
// the per-tree epilogues and dispatches per row and, with no LDS stack, keep the workgroup's LDS at
// the X tile (C2 kernel -5 %, its complete trees -12 %, arithmetic-only -18 %); below
// 2^17 rows the padding and the loss of parallelism cost more.  requested: SR_AMD_ROWS_PER_LANE
// (16 / 32 force a register-stack kernel, 4 / 8 the classic one; f64: 8 selects its register-stack
// build).
#ifndef SR_VSTK_DEFAULT_ROWS
#define SR_VSTK_DEFAULT_ROWS 16
#endif
int sr_vstk_rows(int elem_size, int64_t n_rows, int requested) {
  // f64: the 8-rows/lane register-stack build (181 VGPRs, 2 waves per SIMD) against the classic
  // 4-rows/lane build (100, 5 waves): round 2 measured it 3 % slower; with the launch order dealt over
  // tree groups it is faster (C2 in f64 13.45 -> 12.69 ms per step, arithmetic-only -19 %,
  // profiles/r03_ab_f64_vstk.txt), so it is the default for large views too
  if (elem_size == 8) {
    if (requested == 8 || requested == -4) return requested == 8 ? 8 : 4;  // (-4: the 4-row register-stack build)
    if (requested == 4 || requested == 2) return 0;
    return n_rows >= (int64_t(1) << 17) ? 8 : 0;
  }
  if (requested == 16 || requested == 32) return requested;
  if (requested == 4 || requested == 8) return 0;
  return n_rows >= (int64_t(1) << 17) ? SR_VSTK_DEFAULT_ROWS : 0;
}

template <typename T>
hipError_t sr_launch_eval(const SrEvalArgs<T>& a, int mode, bool gather, int tier, int R, int waves, bool vstk,
                          int n_blocks, hipStream_t s) {
  if constexpr (sizeof(T) == 4) {
    if (mode == SR_MODE_FOLD) {  // (the launch shapes of the loss launches a large call runs: sr_inst_f32_fold*.hip)
      const bool l2 = a.loss_kind == SR_LOSS_L2;
      if (vstk) {
        if (tier != SR_TIER_BASIC || gather || R != 16) return hipErrorInvalidValue;
        return l2 ? sr_launch_tile<T, 16, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, SR_LOSS_L2, true>(a, n_blocks, s)
                  : sr_launch_tile<T, 16, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, -1, true>(a, n_blocks, s);
      }
      if (tier == SR_TIER_BASIC) {
        if (R != 8 || waves != 4) return hipErrorInvalidValue;
        if (gather) return sr_launch_tile<T, 8, SR_MODE_FOLD, true, SR_TIER_BASIC, 4, -1>(a, n_blocks, s);
        return l2 ? sr_launch_tile<T, 8, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, SR_LOSS_L2>(a, n_blocks, s)
                  : sr_launch_tile<T, 8, SR_MODE_FOLD, false, SR_TIER_BASIC, 4, -1>(a, n_blocks, s);
      }
      if (R != 4) return hipErrorInvalidValue;
      return gather ? sr_launch_tile<T, 4, SR_MODE_FOLD, true, SR_TIER_FULL>(a, n_blocks, s)
                    : sr_launch_tile<T, 4, SR_MODE_FOLD, false, SR_TIER_FULL>(a, n_blocks, s);
    }
    if (vstk) {
      if (mode != SR_MODE_LOSS || tier != SR_TIER_BASIC || gather) return hipErrorInvalidValue;
      if (R == 32) return sr_launch_basic_loss<T, 32, false, true>(a, n_blocks, s);
      if (R == 16) return sr_launch_basic_loss<T, 16, false, true>(a, n_blocks, s);
      if (R == 8) return sr_launch_basic_loss<T, 8, false, true>(a, n_blocks, s);
      return hipErrorInvalidValue;
    }
    if (mode == SR_MODE_LOSS) {
      if (tier == SR_TIER_BASIC) {
        if (gather) return sr_launch_basic_loss<T, 8, true>(a, n_blocks, s);
        if (R == 16) return sr_launch_basic_loss<T, 16, false>(a, n_blocks, s);
        if (R == 4) return sr_launch_tile<T, 4, SR_MODE_LOSS, false, SR_TIER_BASIC>(a, n_blocks, s);
        if (waves == 8 && a.loss_kind == SR_LOSS_L2)
          return sr_launch_tile<T, 8, SR_MODE_LOSS, false, SR_TIER_BASIC, 8, SR_LOSS_L2>(a, n_blocks, s);
        return sr_launch_basic_loss<T, 8, false>(a, n_blocks, s);
      }
      return gather ? sr_launch_tile<T, 4, SR_MODE_LOSS, true, SR_TIER_FULL>(a, n_blocks, s)
                    : sr_launch_tile<T, 4, SR_MODE_LOSS, false, SR_TIER_FULL>(a, n_blocks, s);
    }
    if (mode == SR_MODE_PRED)
      return gather ? sr_launch_tile<T, 4, SR_MODE_PRED, true, SR_TIER_FULL>(a, n_blocks, s)
                    : sr_launch_tile<T, 4, SR_MODE_PRED, false, SR_TIER_FULL>(a, n_blocks, s);
    if (tier == SR_TIER_BASIC) {  // (EXACT over a BASIC operator set: the smaller dispatch)
      if (waves == 4)
        return gather ? sr_launch_tile<T, 4, SR_MODE_EXACT, true, SR_TIER_BASIC, 4>(a, n_blocks, s)
                      : sr_launch_tile<T, 4, SR_MODE_EXACT, false, SR_TIER_BASIC, 4>(a, n_blocks, s);
      return gather ? sr_launch_tile<T, 4, SR_MODE_EXACT, true, SR_TIER_BASIC, 1>(a, n_blocks, s)
                    : sr_launch_tile<T, 4, SR_MODE_EXACT, false, SR_TIER_BASIC, 1>(a, n_blocks, s);
    }
    if (waves == 4)  // (EXACT: 1 or 4 waves per workgroup, sharing the staged rows)
      return gather ? sr_launch_tile<T, 4, SR_MODE_EXACT, true, SR_TIER_FULL, 4>(a, n_blocks, s)
                    : sr_launch_tile<T, 4, SR_MODE_EXACT, false, SR_TIER_FULL, 4>(a, n_blocks, s);
    return gather ? sr_launch_tile<T, 4, SR_MODE_EXACT, true, SR_TIER_FULL, 1>(a, n_blocks, s)
                  : sr_launch_tile<T, 4, SR_MODE_EXACT, false, SR_TIER_FULL, 1>(a, n_blocks, s);
  } else {
    if (mode == SR_MODE_FOLD) return hipErrorInvalidValue;  // (Float64: small calls only, from stored losses)
    if (vstk) {
      if (mode != SR_MODE_LOSS || tier != SR_TIER_BASIC || gather) return hipErrorInvalidValue;
      if (R == 8) return sr_launch_basic_loss<T, 8, false, true>(a, n_blocks, s);
      if (R == 4) return sr_launch_basic_loss<T, 4, false, true>(a, n_blocks, s);
      return hipErrorInvalidValue;
    }
    if (mode == SR_MODE_LOSS) {
      if (tier == SR_TIER_BASIC)
        return gather ? sr_launch_basic_loss<T, 4, true>(a, n_blocks, s) : sr_launch_basic_loss<T, 4, false>(a, n_blocks, s);
      return gather ? sr_launch_tile<T, 2, SR_MODE_LOSS, true, SR_TIER_FULL>(a, n_blocks, s)
                    : sr_launch_tile<T, 2, SR_MODE_LOSS, false, SR_TIER_FULL>(a, n_blocks, s);
    }
    if (mode == SR_MODE_PRED)
      return gather ? sr_launch_tile<T, 2, SR_MODE_PRED, true, SR_TIER_FULL>(a, n_blocks, s)
                    : sr_launch_tile<T, 2, SR_MODE_PRED, false, SR_TIER_FULL>(a, n_blocks, s);
    if (tier == SR_TIER_BASIC) {
      if (waves == 4)
        return gather ? sr_launch_tile<T, 2, SR_MODE_EXACT, true, SR_TIER_BASIC, 4>(a, n_blocks, s)
                      : sr_launch_tile<T, 2, SR_MODE_EXACT, false, SR_TIER_BASIC, 4>(a, n_blocks, s);
      return gather ? sr_launch_tile<T, 2, SR_MODE_EXACT, true, SR_TIER_BASIC, 1>(a, n_blocks, s)
                    : sr_launch_tile<T, 2, SR_MODE_EXACT, false, SR_TIER_BASIC, 1>(a, n_blocks, s);
    }
    if (waves == 4)
      return gather ? sr_launch_tile<T, 2, SR_MODE_EXACT, true, SR_TIER_FULL, 4>(a, n_blocks, s)
                    : sr_launch_tile<T, 2, SR_MODE_EXACT, false, SR_TIER_FULL, 4>(a, n_blocks, s);
    return gather ? sr_launch_tile<T, 2, SR_MODE_EXACT, true, SR_TIER_FULL, 1>(a, n_blocks, s)
                  : sr_launch_tile<T, 2, SR_MODE_EXACT, false, SR_TIER_FULL, 1>(a, n_blocks, s);
  }
}
template hipError_t sr_launch_eval<float>(const SrEvalArgs<float>&, int, bool, int, int, int, bool, int, hipStream_t);
template hipError_t sr_launch_eval<double>(const SrEvalArgs<double>&, int, bool, int, int, int, bool, int, hipStream_t);
template hipError_t sr_launch_transpose<float>(const float*, int64_t, int64_t, int64_t, float*, hipStream_t);
template hipError_t sr_launch_transpose<double>(const double*, int64_t, int64_t, int64_t, double*, hipStream_t);
template hipError_t sr_launch_pad<float>(float*, int64_t, int64_t, float, int, hipStream_t);
template hipError_t sr_launch_pad<double>(double*, int64_t, int64_t, double, int, hipStream_t);
