// sr_fold_dev.h — device side of the reference's in-order loss fold (sr_fold.h), shared by the fold
// kernels (sr_aux.hip) and the interpreter's FOLD mode (sr_tile_impl.h).
//
// LossFunctions' mean / weighted sum fold the elementwise losses left to right in T
// (/root/reference/src/LossFunctions.jl:38-58).  While the running value p stays in one binade
// [2^e, 2^(e+1)) with spacing 2^q, fl(p + l) = p + 2^q (m + r), where l / 2^q = m + f (m integer) and r
// rounds f half-to-even against the parity of p / 2^q + m — so a step depends on the running value only
// through its parity, and runs of steps compose (a pair: the ulps added from an even and from an odd
// start; compose(x, y)(b) = x(b) + y((b + x(b)) & 1)).  The step that leaves the binade is the hardware
// add itself.  A step with f != 1/2 does not depend on the parity at all: it is rint(l / 2^q), so a run
// of rows without an exact half is one sum (the FOLD mode's fast path below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sr_fold.h"
#include "sr_ops.h"

// Per-(row block, position) codes of a call's fold plan (sr_fold_plan_kernel / sr_fold_stab_kernel):
//   SR_FCODE_SKIP        the tree is not folded (incomplete, NaN, overflow band, or out of slots)
//   >= SR_FCODE_SLOT0    a slow segment: its losses are stored in slot (code - SR_FCODE_SLOT0) and the
//                        walk folds them row by row (the first segment; any segment the fold may cross a
//                        binade in)
//   otherwise            the binade spacing exponent q of the segment's composed step (fold_tab)
constexpr int32_t SR_FCODE_SKIP = int32_t(0x80000000u);
constexpr int32_t SR_FCODE_SLOT0 = 0x40000000;
// per-tree status of the walk (sr_fold_walk_kernel): not folded / the fold's exact value / the plan's
// speculated binades missed (the host folds that tree through the prediction pass instead)
enum { SR_FST_NONE = 0, SR_FST_OK = 1, SR_FST_FAIL = 2 };

template <typename T>
struct SrFoldStep {
  int64_t m;
  int kind;  // 0: f < 1/2, 1: f == 1/2 (tie), 2: f > 1/2
};

template <typename T>
__device__ __forceinline__ SrFoldStep<T> sr_fold_step(T e, int q, int64_t cap) {
  SrFoldStep<T> st{cap, 0};
  const double t = ldexp(double(e), -q);  // exact: a power-of-two scaling of a T value
  if (!(t < double(cap))) return st;      // (also NaN / Inf: a crossing, taken by the hardware add)
  const double fl = floor(t);
  const double f = t - fl;
  st.m = int64_t(fl);
  st.kind = f > 0.5 ? 2 : (f == 0.5 ? 1 : 0);
  return st;
}
template <typename T>
__device__ __forceinline__ int64_t sr_fold_inc(const SrFoldStep<T>& st, int64_t b) {
  return st.m + (st.kind == 2 ? 1 : (st.kind == 1 ? ((b + st.m) & 1) : 0));
}
// (a0, a1): ulps added from an even / odd start; y := x then y (saturating at cap)
__device__ __forceinline__ void sr_fold_compose(int64_t x0, int64_t x1, int64_t& y0, int64_t& y1, int64_t cap) {
  const int64_t n0 = x0 + ((x0 & 1) ? y1 : y0);
  const int64_t n1 = x1 + (((1 + x1) & 1) ? y1 : y0);
  y0 = n0 < cap ? n0 : cap;
  y1 = n1 < cap ? n1 : cap;
}

// The step of one loss for the segment tables, in the narrowest exact arithmetic: Float32 losses in
// Float32 (e 2^-q is exact but for an underflow, which only ever hides a fraction below 1/2; the
// saturation CAP = 2^26 keeps the counts in int32), Float64 losses in Float64 / int64.
template <typename T>
struct SrFoldTab;
template <>
struct SrFoldTab<float> {
  using I = int32_t;
  using Pair = int2;
  static __device__ __forceinline__ void step(float e, int q, I& m, int& kind) {
    constexpr float CAPF = float(1 << 26);
    const float t = ldexpf(e, -q);
    if (!(t < CAPF)) {  // (also NaN / Inf)
      m = I(1) << 26;
      kind = 0;
      return;
    }
    const float fl = floorf(t);
    const float f = t - fl;
    m = I(fl);
    kind = f > 0.5f ? 2 : (f == 0.5f ? 1 : 0);
  }
  static __device__ __forceinline__ Pair pair(I a, I b) { return make_int2(a, b); }
};
template <>
struct SrFoldTab<double> {
  using I = int64_t;
  using Pair = longlong2;
  static __device__ __forceinline__ void step(double e, int q, I& m, int& kind) {
    const SrFoldStep<double> st = sr_fold_step<double>(e, q, int64_t(1) << 55);
    m = st.m;
    kind = st.kind;
  }
  static __device__ __forceinline__ Pair pair(I a, I b) { return make_longlong2(a, b); }
};
template <typename I>
__device__ __forceinline__ void sr_fold_compose_i(I x0, I x1, I& y0, I& y1, I cap) {
  const I n0 = x0 + ((x0 & 1) ? y1 : y0);
  const I n1 = x1 + (((1 + x1) & 1) ? y1 : y0);
  y0 = n0 < cap ? n0 : cap;
  y1 = n1 < cap ? n1 : cap;
}
template <typename I>
__device__ __forceinline__ void sr_fold_add_i(I m, int kind, I cap, I& a0, I& a1) {
  // (a0, a1) then the step (m, kind): from start parity b the running value's parity is b + a_b
  const I e0 = m + (kind == 2 ? 1 : (kind == 1 ? ((a0 + m) & 1) : 0));
  const I e1 = m + (kind == 2 ? 1 : (kind == 1 ? ((1 + a1 + m) & 1) : 0));
  a0 = a0 + e0 < cap ? a0 + e0 : cap;
  a1 = a1 + e1 < cap ? a1 + e1 : cap;
}

// Inclusive wave scan of nonnegative values in lane order, by DPP lane moves (pure VALU, no LDS round
// trips): row_shr 1, 2, 4, 8 within each row of 16 lanes (lanes shifted in from outside the row read
// 0), then row 0's total into rows 1 and 3 (row_bcast:15) and rows 0 + 1 into rows 2 and 3
// (row_bcast:31).  Integer-valued sums are exact below 2^(mant+1) and monotone above.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int sr_fold_dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, true);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float sr_fold_dpp_add(float v) {
  return v + __int_as_float(sr_fold_dpp<CTRL, ROW_MASK>(__float_as_int(v)));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double sr_fold_dpp_add(double v) {
  const uint64_t b = uint64_t(__double_as_longlong(v));
  const uint32_t lo = uint32_t(sr_fold_dpp<CTRL, ROW_MASK>(int(uint32_t(b))));
  const uint32_t hi = uint32_t(sr_fold_dpp<CTRL, ROW_MASK>(int(uint32_t(b >> 32))));
  return v + __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
}
template <typename T>
__device__ __forceinline__ T sr_fold_scan(T v) {
  v = sr_fold_dpp_add<0x111>(v);       // row_shr:1
  v = sr_fold_dpp_add<0x112>(v);       // row_shr:2
  v = sr_fold_dpp_add<0x114>(v);       // row_shr:4
  v = sr_fold_dpp_add<0x118>(v);       // row_shr:8
  v = sr_fold_dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v = sr_fold_dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return v;
}
// the value of lane l (wave-uniform l), by readlane (a few cycles; __shfl is an LDS permute round trip)
__device__ __forceinline__ float sr_fold_lane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double sr_fold_lane(double v, int l) {
  const uint64_t b = uint64_t(__double_as_longlong(v));
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(b)), l));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(b >> 32)), l));
  return __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
}

__device__ __forceinline__ int32_t sr_fold_lane(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int64_t sr_fold_lane(int64_t v, int l) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v))), l));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v) >> 32)), l));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// A finite running value F >= 0 as (q, P, lim): F = P 2^q with P < lim in F's binade (spacing 2^q; the
// subnormals share the lowest normal binade's spacing, lim = 2^mant), by the bits alone (no f64
// round trip: the walk's rounds are a chain of these).  And back: (P, q) with P < lim -> F, bits =
// ((q - qmin) << mant) + P for the normal and the subnormal binades alike.
template <typename T>
struct SrFoldBinade;
template <>
struct SrFoldBinade<float> {
  int q;
  int32_t P, lim;
  __device__ __forceinline__ explicit SrFoldBinade(float F) {
    const uint32_t b = __float_as_uint(F);
    const int e = int(b >> 23);
    q = e == 0 ? -149 : e - 150;
    P = e == 0 ? int32_t(b) : int32_t((b & 0x7fffffu) | 0x800000u);
    lim = e == 0 ? (1 << 23) : (1 << 24);
  }
  static __device__ __forceinline__ float value(int32_t P, int q) {
    return __uint_as_float((uint32_t(q + 149) << 23) + uint32_t(P));
  }
};
template <>
struct SrFoldBinade<double> {
  int q;
  int64_t P, lim;
  __device__ __forceinline__ explicit SrFoldBinade(double F) {
    const uint64_t b = uint64_t(__double_as_longlong(F));
    const int e = int(b >> 52);
    q = e == 0 ? -1074 : e - 1075;
    P = e == 0 ? int64_t(b) : int64_t((b & 0xfffffffffffffull) | 0x10000000000000ull);
    lim = e == 0 ? (int64_t(1) << 52) : (int64_t(1) << 53);
  }
  static __device__ __forceinline__ double value(int64_t P, int q) {
    return __longlong_as_double(int64_t((uint64_t(q + 1074) << 52) + uint64_t(P)));
  }
};

// binade spacing exponent q of a value >= 0 (subnormals and 0: the fixed subnormal spacing); values
// past the type's range get a q no finite running value has
template <typename T>
__device__ __forceinline__ int sr_fold_q(double x) {
  using Tr = SrFoldTraits<T>;
  constexpr double MIN_NORMAL = sizeof(T) == 4 ? 1.17549435e-38 : 2.2250738585072014e-308;
  if (!(x >= MIN_NORMAL)) return Tr::qmin;
  if (!(x <= double(SrM<T>::big))) return 1 << 20;
  int ex;
  (void)frexp(x, &ex);
  return ex - 1 - Tr::mant;
}

// May a complete tree's loss be folded by the plan?  Its f64 sum S is finite, >= 0, and the overflow
// rule of sr_fold.h leaves the fold finite (the band trees keep the prediction-pass fold; +Inf verdicts
// stay +Inf).  flags: the call's per-tree flags (BIG trees are folded too: the exact pass decides later).
template <typename T>
__device__ __forceinline__ bool sr_fold_eligible(double S, uint32_t flags, int64_t n_terms) {
  if (flags & (SR_FLAG_NONFINITE | SR_FLAG_STATIC | SR_FLAG_ELEMINF)) return false;
  if (!(S >= 0.0) || !(S <= 1.7976931348623157e308)) return false;
  return sr_fold_class<T>(S, false, n_terms) == SR_FOLD_FINITE;
}

// Which trees a call's fold plan folds, and where their folds start (kernel argument, by value): a
// single-GPU call reads its per-tree f64 sums and flags (sr_fold_eligible); a row-sharded call passes
// the ranks' agreed verdicts (elig: nonzero = fold) and, per tree, the f64 sum of the shards before this
// one (est); first: this view starts the fold (its first loss starts it, the first segment is slow).
struct SrFoldWho {
  const double* sums;
  const uint32_t* flags;
  int64_t n_terms;
  const uint8_t* elig;
  const double* est;
  int first;
  // (a small stored-loss call's results in pinned memory: the walk copies each tree's Σ and flags there
  //  beside its value, so the call needs no copy back; nullptr: none)
  double* msum = nullptr;
  uint32_t* mflag = nullptr;
  template <typename T>
  __device__ __forceinline__ bool eligible(uint32_t t) const {
    return elig ? elig[t] != 0 : sr_fold_eligible<T>(sums[t], flags[t], n_terms);
  }
};

// The composed step of one tree over one row tile under binade spacing 2^q: l[R] = the lane's losses
// in the tile layout (chunk c of lane l = tile rows c*64*C + l*C + j, sr_tile_impl.h SrLane), rows past
// the view already 0.  Returns the wave-uniform pair (from an even / an odd start).  Fast path: no loss
// of the tile is an exact half ulp of the binade, so every step is rint(l 2^-q) whatever the parity and
// the tile's step is their sum (partial sums of integers exact below 2^(mant+1) and monotone above, +Inf
// included, so a sum that leaves the binade still reads as one); otherwise the ordered
// composition, row by row in the lane, then over the lanes (lane order = row order in a chunk), then
// over the chunks.
template <typename T, int R, int C>
__device__ __forceinline__ void sr_fold_tile_step(const T (&l)[R], int q, int lane, typename SrFoldTab<T>::I& t0,
                                                  typename SrFoldTab<T>::I& t1) {
  using I = typename SrFoldTab<T>::I;
  constexpr I CAP = I(1) << (SrFoldTraits<T>::mant + 3);
  T tsum = T(0), dmax = T(0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const T v = sizeof(T) == 4 ? T(ldexpf(float(l[r]), -q)) : T(ldexp(double(l[r]), -q));
    const T s = sizeof(T) == 4 ? T(rintf(float(v))) : T(rint(double(v)));
    const T d = v - s;
    const T ad = d < T(0) ? -d : d;
    dmax = ad > dmax ? ad : dmax;  // (NaN — a step past the type's range, Inf - Inf — ignored)
    tsum += s;  // (no clamp: a sum past 2^(mant+1) reads as CAP below whatever it is, +Inf included)
  }
  if (__builtin_amdgcn_ballot_w64(dmax == T(0.5)) == 0) {
    // wave sum of nonnegative integer values (lane 63's inclusive scan): exact below 2^(mant+1), and any
    // sum past that fails a run the same way
    const T v = sr_fold_lane(sr_fold_scan(tsum), 63);
    const I t = v < T(CAP) ? I(v) : CAP;
    t0 = t;
    t1 = t;
    return;
  }
  I y0 = 0, y1 = 0;  // the tile so far (uniform)
#pragma unroll
  for (int c = 0; c < R / C; ++c) {
    I a0 = 0, a1 = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      I m;
      int kind;
      SrFoldTab<T>::step(l[c * C + j], q, m, kind);
      sr_fold_add_i<I>(m, kind, CAP, a0, a1);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // ordered: lane l's rows precede lane l + 1's
      I o0 = __shfl_down(a0, off, 64), o1 = __shfl_down(a1, off, 64);
      if ((lane & (2 * off - 1)) == 0) {
        sr_fold_compose_i<I>(a0, a1, o0, o1, CAP);
        a0 = o0;
        a1 = o1;
      }
    }
    I c0 = __shfl(a0, 0, 64), c1 = __shfl(a1, 0, 64);
    sr_fold_compose_i<I>(y0, y1, c0, c1, CAP);
    y0 = c0;
    y1 = c1;
  }
  t0 = y0;
  t1 = y1;
}
