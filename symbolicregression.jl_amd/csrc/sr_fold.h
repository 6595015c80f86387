// sr_fold.h — does the reference's loss fold overflow T?
//
// The reference aggregates elementwise losses with LossFunctions.jl (src/LossFunctions.jl:38-58):
// `mean(loss, x, y)` (Statistics.mean over a generator: v = l_1; v = v + l_i; then v / n) and
// `sum(loss, x, y, w; normalize=true)` (Base.sum over a generator, the same left fold of w_i * l_i, then
// / sum(w)).  Both folds run in T, so a complete tree whose losses are finite but whose T-precision
// running sum passes floatmax(T) scores +Inf there, while an f64 accumulation (the device's) stays
// finite.  The losses are >= 0, so the fold's prefix sums are monotone and the verdict follows from
// bounds on the fold in terms of the exact sum S of the T losses (n terms, unit roundoff u of T;
// every rounding error is at most u times the rounded prefix, which never exceeds the final fold F):
//     S / (1 + (n - 1) u)  <=  F  <=  S (1 + u)^(n - 1)
// so F certainly overflows when the lower bound reaches the overflow threshold M = floatmax + ulp/2,
// and certainly does not when the upper bound stays below it.  F is also at least the fold of any
// subsequence of the losses (p only grows, and rounding is monotone), so a loss of +Inf, or two whose
// T sum is +Inf, make F = +Inf: the interpreter flags that (SR_FLAG_ELEMINF) from the first level of
// its pairwise tile sums.  Between the bounds (and whenever the device's own sum overflowed without such
// a pair) the fold is computed exactly, in order, by sr_fold_kernel (sr_aux.hip).  Negative weights
// break the monotonicity: this rule assumes w >= 0.
#pragma once
#include <math.h>
#include <stdint.h>

#include "sr_ops.h"

enum { SR_FOLD_FINITE = 0, SR_FOLD_INF = 1, SR_FOLD_EXACT = 2 };

template <typename T>
struct SrFoldTraits;
template <>
struct SrFoldTraits<float> {
  static constexpr int mant = 23;                        // stored mantissa bits
  static constexpr int qmin = -149;                      // exponent of the subnormal spacing
  static constexpr double u = 5.9604644775390625e-08;    // 2^-24
  static constexpr double M = 3.4028235677973366e38;     // 2^128 - 2^103: the smallest sum rounding to Inf
};
template <>
struct SrFoldTraits<double> {
  static constexpr int mant = 52;
  static constexpr int qmin = -1074;
  static constexpr double u = 1.1102230246251565e-16;    // 2^-53
  static constexpr double M = 1.7976931348623157e308;    // (2^1024 - 2^970 is not a double: DBL_MAX, so
                                                         //  the Inf verdict is never taken early for f64)
};

// Relative error of the device's f64 loss sum against the exact sum of the T losses: each tile's
// sum is a T pairwise sum of <= 64 x 32 losses (<= 11 levels), the tiles and row blocks then add in f64.
template <typename T>
SR_HD inline double sr_fold_dev_eps(int64_t n_terms) {
  return 11.0 * SrFoldTraits<T>::u * 1.001 + (double(n_terms) / 64.0 + 64.0) * 1.1102230246251565e-16;
}

// Classify one complete tree from the device's loss sum S (f64 accumulation of the T losses) over
// n_terms rows: SR_FOLD_FINITE (use S), SR_FOLD_INF (the reference's fold overflows), SR_FOLD_EXACT
// (fold the losses in order).  elem_inf: some elementwise loss is +Inf (SR_FLAG_ELEMINF).
template <typename T>
SR_HD inline int sr_fold_class(double S, bool elem_inf, int64_t n_terms) {
  using Tr = SrFoldTraits<T>;
  if (elem_inf) return SR_FOLD_INF;
  if (S != S) return SR_FOLD_FINITE;  // a NaN loss: the fold is NaN too (no overflow question)
  if (S == INFINITY) return SR_FOLD_EXACT;  // the device's T tile sums overflowed: decide exactly
  if (S < 0.0) return SR_FOLD_FINITE;       // (negative weights: outside the rule)
  const double k = double(n_terms > 1 ? n_terms - 1 : 0);
  const double eps = sr_fold_dev_eps<T>(n_terms);
  // upper bound on F: S (1 + eps) (1 + u)^k, the power rounded up
  const double grow = exp(k * log1p(Tr::u)) * (1.0 + 1e-12);
  const double hi = S * (1.0 + eps) * grow;
  if (hi < Tr::M) return SR_FOLD_FINITE;
  const double lo = S * (1.0 - eps) / (1.0 + k * Tr::u);
  if (lo >= Tr::M && sizeof(T) == 4) return SR_FOLD_INF;
  return SR_FOLD_EXACT;
}
