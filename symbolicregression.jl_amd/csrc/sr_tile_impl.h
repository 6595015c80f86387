// sr_tile_impl.h — CDNA4 (gfx950) batched expression-tree interpreter (kernel template).
//
// What it replaces: DynamicExpressions' array-at-a-time `eval_tree_array` + SymbolicRegression's
// `_eval_loss` (reference src/LossFunctions.jl:90-117), for a whole population at once.
//
// Execution model:
//   * a workgroup = 4 wave64s owns one row block (`tiles` row tiles of 64*R rows each) and a group
//     of G trees; per tile, the X rows (all features), y and weights are staged ONCE in LDS and
//     shared by the 4 waves, which take different trees of the group (tree g -> wave g % 4);
//   * lane `l` owns R rows of the tile: chunk c (16 bytes = C values) of lane l is tile row
//     c*64*C + l*C + j, so every LDS read of a feature / stack slot is a conflict-free ds_read_b128
//     and the LDS image of a tile is a plain copy of the global rows;
//   * each wave interprets its trees' programs: the program sits in VGPRs (one 16-byte instruction
//     per lane, 64-instruction windows, the next window in flight while one runs) and each step
//     reads its opcode word with v_readlane; one flat `switch` over the opcode dispatches to
//     straight-line VALU bodies on the R-row top of stack (VGPRs); operand stack slots (assigned
//     statically by the compiler) live in a per-wave LDS area;
//   * DynamicExpressions' validity checks: BASIC tier — every operator output updates a running
//     max |v| (v_max3 with abs modifiers), decided once per tree and tile (Inf -> incomplete,
//     >= tbig -> exact-sum path, NaN reaches the root); FULL tier — per CHECK node, integer-max
//     test + ballot, early exit on a non-finite value;
//   * per-tree loss: T per lane -> DPP wave sum -> f64 accumulator in the owning lane (tiles in
//     order: deterministic) -> one partial per (row block, tree) -> fixed-order reduce kernel.
// Compile with -mllvm -structurizecfg-skip-uniform-regions=true: all branches here are
// wave-uniform, and without the flag LLVM's structurizer turns the opcode switch into a chain of
// exec-mask "flow" blocks with copies of the stack registers at every join.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sr_eval.h"
#include "sr_fold_dev.h"
#include "sr_ops.h"

// Waves per workgroup W is a template parameter (4 by default); the minimum resident waves per
// SIMD the register allocator must allow is derived from it (SrMinWaves).
template <int W>
struct SrMinWaves {
  static constexpr int value = W >= 16 ? 8 : (W >= 8 ? 6 : 1);
};
// The f32 BASIC 8-rows/lane kernels fit 96 VGPRs (5 waves per SIMD; the interpreter loop is
// latency-bound, so the fifth wave is worth it: C2 -4 %, arithmetic-only populations -10 %); the
// few spills this forces sit in the tile-staging code, not in the interpreter loop.  The other
// variants would spill inside the loop at that bound.
#ifndef SR_MIN_WAVES_W4
#define SR_MIN_WAVES_W4 5
#endif
#ifndef SR_MIN_WAVES_R16
#define SR_MIN_WAVES_R16 2
#endif
#ifndef SR_MIN_WAVES_VSTK16
#define SR_MIN_WAVES_VSTK16 4
#endif

#ifndef SR_MIN_WAVES_VSTK8
#define SR_MIN_WAVES_VSTK8 6
#endif
// f64 register stack at 8 rows per lane: 168 VGPRs = 3 waves per SIMD for the L2 / L1 builds, no
// spills (round 4's epilogue grew them to 172 — 2 waves — and the Float64 C2 step to 22.7 ms from
// 15.9; profiles/r04_ab_regress.txt); the generic-loss build keeps 2 (it would spill at 168)
#ifndef SR_MIN_WAVES_VSTK_F64
#define SR_MIN_WAVES_VSTK_F64 3
#endif
#ifndef SR_MIN_WAVES_VSTK_F64_GENERIC
#define SR_MIN_WAVES_VSTK_F64_GENERIC 2
#endif
// the f32 gather (SubDataset / several-view) build: 80 VGPRs, 6 waves per SIMD (it needed 75 before
// the row-view segments); the f64 classic generic-loss builds: 128, 4 waves
#ifndef SR_MIN_WAVES_GATHER_F32
#define SR_MIN_WAVES_GATHER_F32 6
#endif
#ifndef SR_MIN_WAVES_F64_GENERIC
#define SR_MIN_WAVES_F64_GENERIC 4
#endif
#ifndef SR_MIN_WAVES_VSTK4_F64
#define SR_MIN_WAVES_VSTK4_F64 4  // f64 register stack at 4 rows per lane: <= 128 VGPRs
#endif
#ifndef SR_MIN_WAVES_VSTK32
#define SR_MIN_WAVES_VSTK32 3
#endif
template <typename T, int R, int TIER, int W, bool VSTK = false, int LK = -1, bool GATHER = false, int MODE = 0>
struct SrMinWavesFor {
  static constexpr bool f32_basic = sizeof(T) == 4 && TIER == SR_TIER_BASIC && W == 4;
  static constexpr bool f64_basic = sizeof(T) == 8 && TIER == SR_TIER_BASIC && W == 4;
  static constexpr bool loss = MODE == 0;  // (SR_MODE_LOSS)
  static constexpr int value = (f64_basic && VSTK && R == 4)     ? SR_MIN_WAVES_VSTK4_F64
                               : (f64_basic && VSTK && LK >= 0)    ? SR_MIN_WAVES_VSTK_F64
                               : (f64_basic && VSTK)               ? SR_MIN_WAVES_VSTK_F64_GENERIC
                               : (f64_basic && loss && R == 4 && LK < 0) ? SR_MIN_WAVES_F64_GENERIC
                               : (f32_basic && loss && GATHER && R == 8 && LK >= 0) ? SR_MIN_WAVES_GATHER_F32
                               : (f32_basic && VSTK && R == 8)    ? SR_MIN_WAVES_VSTK8
                               : (f32_basic && VSTK && R == 16)   ? SR_MIN_WAVES_VSTK16
                               : (f32_basic && VSTK && R == 32) ? SR_MIN_WAVES_VSTK32
                               : (f32_basic && R == 8)          ? SR_MIN_WAVES_W4
                               : (f32_basic && R == 16)         ? SR_MIN_WAVES_R16
                                                                : SrMinWaves<W>::value;
};

// 16-byte chunks of C values.
template <typename T>
struct SrChunk;
template <>
struct SrChunk<float> {
  using V = float4;
  static constexpr int N = 4;
  static __device__ inline void get(const V& v, float* o) { o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w; }
  static __device__ inline V make(const float* o) { return make_float4(o[0], o[1], o[2], o[3]); }
};
template <>
struct SrChunk<double> {
  using V = double2;
  static constexpr int N = 2;
  static __device__ inline void get(const V& v, double* o) { o[0] = v.x; o[1] = v.y; }
  static __device__ inline V make(const double* o) { return make_double2(o[0], o[1]); }
};

// A lane's R values of one tile-shaped array (X feature row, stack slot, y, w): chunk c of lane l at
// element (c*64 + l)*C.  `p` points at element l*C of chunk 0.
template <typename T, int R>
struct SrLane {
  using Ch = SrChunk<T>;
  static constexpr int C = Ch::N;
  static constexpr int NC = R / C;
  static_assert(R % C == 0, "rows per lane must fill whole 16-byte chunks");
  static __device__ inline void load(const T* p, T (&o)[R]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) Ch::get(*reinterpret_cast<const typename Ch::V*>(p + c * 64 * C), o + c * C);
  }
  static __device__ inline void store(T* p, const T (&o)[R]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) *reinterpret_cast<typename Ch::V*>(p + c * 64 * C) = Ch::make(o + c * C);
  }
  // tile row (0-based within the tile) of value r of lane l
  static __device__ inline int row(int l, int r) { return (r / C) * 64 * C + l * C + (r % C); }
};

// Whole-wave sum with DPP lane moves (pure VALU: no LDS round trips), in a fixed order:
// pairs, quads (quad_perm), 8 (row_half_mirror), 16 (row_mirror), then rows 0+1 / 2+3
// (row_bcast:15) and the two halves (row_bcast:31).  The total is read from lane 63 (uniform).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int sr_dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float sr_dpp_add(float v) {
  return v + __int_as_float(sr_dpp<CTRL, ROW_MASK>(__float_as_int(v)));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double sr_dpp_add(double v) {
  const uint64_t b = uint64_t(__double_as_longlong(v));
  const uint32_t lo = uint32_t(sr_dpp<CTRL, ROW_MASK>(int(uint32_t(b))));
  const uint32_t hi = uint32_t(sr_dpp<CTRL, ROW_MASK>(int(uint32_t(b >> 32))));
  return v + __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
}
template <typename T>
__device__ __forceinline__ T sr_wave_sum(T v) {
  v = sr_dpp_add<0xb1>(v);        // quad_perm [1,0,3,2]
  v = sr_dpp_add<0x4e>(v);        // quad_perm [2,3,0,1]
  v = sr_dpp_add<0x141>(v);       // row_half_mirror
  v = sr_dpp_add<0x140>(v);       // row_mirror
  v = sr_dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v = sr_dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  if constexpr (sizeof(T) == 4) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
  } else {
    const uint64_t b = uint64_t(__double_as_longlong(v));
    const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(b)), 63));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(b >> 32)), 63));
    return __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
  }
}
__device__ __forceinline__ uint64_t sr_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Magnitude key for the validity checks: ordered like |v| for finite values, and above every finite
// value for Inf / NaN.  f64 uses the high word only (conservative: a few values just below tbig
// also count as suspicious, which only sends the tree through the exact-sum path).
template <typename T>
struct SrBits;
template <>
struct SrBits<float> {
  static __device__ inline uint32_t mag(float x) { return __float_as_uint(x) & 0x7fffffffu; }
};
template <>
struct SrBits<double> {
  static __device__ inline uint32_t mag(double x) {
    return uint32_t(uint64_t(__double_as_longlong(x)) >> 32) & 0x7fffffffu;
  }
};

// Running max of |checked values| (deferred validity checks, BASIC tier): m <- max(m, |a|, |b|).
// NaN operands are ignored by the IEEE max; the BASIC operators all map NaN to NaN, so a NaN at any
// checked node reaches the root, whose values are tested for NaN explicitly.
template <typename T>
struct SrMaxAbs;
template <>
struct SrMaxAbs<float> {
  static __device__ __forceinline__ float step(float m, float a, float b) {
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
  }
};
template <>
struct SrMaxAbs<double> {
  static __device__ __forceinline__ double step(double m, double a, double b) {
    double r, q;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(q) : "v"(m), "v"(a));
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(q), "v"(b));
    return r;
  }
};


// The constant of instruction k of a window (uniform): c0 (f32) or c0 | c1 << 32 (f64).
template <typename T>
__device__ __forceinline__ T sr_lane_value(uint32_t wc0, uint32_t wc1, uint32_t k) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(int(wc0), int(k)));
  } else {
    // readlane returns int: widen through uint32_t (no sign extension into the high word)
    return __builtin_bit_cast(T, uint64_t(uint32_t(__builtin_amdgcn_readlane(int(wc0), int(k)))) |
                                     (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(wc1), int(k)))) << 32));
  }
}

// Row `meta & SR_M_INDEX` of a [.][ROWS] LDS array: the byte offset is meta << log2(ROWS*sizeof(T))
// in 32 bits, which drops meta's flag bits (24..31) since the shift is >= 8.
template <int ROWS, typename P>
__device__ __forceinline__ P* sr_row_at(P* base, uint32_t meta) {
  constexpr uint32_t bytes = uint32_t(ROWS * sizeof(P));
  constexpr uint32_t sh = bytes >= 8192u ? 13u : bytes >= 4096u ? 12u : bytes >= 2048u ? 11u
                        : bytes >= 1024u ? 10u : bytes >= 512u ? 9u : 8u;
  static_assert((1u << sh) == bytes, "row stride must be a power of two >= 256 bytes");
  using B = typename std::conditional<std::is_const<P>::value, const char, char>::type;
  return reinterpret_cast<P*>(reinterpret_cast<B*>(base) + (meta << sh));
}

// The double-precision Float32 libm (log / cos / sin, sr_libm.h) over a lane's R rows, as a real
// call: its polynomial constants and f64 temporaries live in the callee's own registers instead of
// being hoisted out of the interpreter loop and spilled, and each body exists once per kernel.
// Rows per scheduling group inside the libm row callees: a sched_barrier after every group keeps
// the callee's live registers to that many rows' temporaries (1 = row by row).
#ifndef SR_LIBM_ILP
#define SR_LIBM_ILP 1
#endif
#define SR_LIBM_ROW_END(r) \
  if (((r) + 1) % SR_LIBM_ILP == 0) __builtin_amdgcn_sched_barrier(0)
template <int R>
using SrRowVec = float __attribute__((ext_vector_type(R)));
#ifdef SR_LIBM_INLINE
#define SR_LIBM_CALL __attribute__((always_inline))
#else
#define SR_LIBM_CALL __attribute__((noinline))
#endif
// every row through the full-range function (Float32 log / cos / sin)
template <uint32_t ID, int R>
__device__ __attribute__((noinline)) SrRowVec<R> sr_libm_rows(SrRowVec<R> v) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    v[r] = sr_unary<float>(ID, v[r]);
    __builtin_amdgcn_sched_barrier(0);  // row by row: few live registers
  }
  return v;
}
// Float64 transcendentals (OCML) over the rows, as a real call: inlined into the interpreter's
// switch their temporaries set the kernel's VGPR count (143 at 4 rows per lane: 3 waves per SIMD).
template <uint32_t ID, int R>
using SrRowVecD = double __attribute__((ext_vector_type(R)));
template <uint32_t ID, int R>
__device__ __attribute__((noinline)) SrRowVecD<ID, R> sr_libm_rows_f64(SrRowVecD<ID, R> v) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    v[r] = sr_unary<double>(ID, v[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
  return v;
}
// Float32 log over the rows, its coefficients in scalar registers for the whole call.  When every row
// of the wave is a positive normal finite value (unsigned bits in [2^23, 0x7f7fffff]: one max and one
// min per row, one ballot) the rows take the bare reduction + polynomial; otherwise every row takes
// the full function (same arithmetic for those values, plus zeros, subnormals, Inf, NaN, negatives).
template <int R>
__device__ SR_LIBM_CALL SrRowVec<R> sr_log_rows(SrRowVec<R> v) {
  const SrLogC c = sr_logc_sgpr();
  const double* tab = sr_log_tab();
  uint32_t hi = 0u, lo = 0xffffffffu;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t b = __float_as_uint(v[r]);
    hi = b > hi ? b : hi;
    lo = b < lo ? b : lo;
  }
  if (__builtin_amdgcn_ballot_w64(hi > 0x7f7fffffu || lo < 0x00800000u) == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[r] = float(sr_log_normal(__float_as_uint(v[r]), 0, tab, c));
      SR_LIBM_ROW_END(r);
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[r] = sr_logf_core(v[r], tab, c);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  return v;
}
// cos / sin when every row of the wave has |x| < 2^20 (a separate function: its few registers are
// all caller-saved, so the common call saves nothing)
template <uint32_t ID, int R>
__device__ SR_LIBM_CALL SrRowVec<R> sr_trig_rows_fast(SrRowVec<R> v) {
#ifdef SR_TRIG_PIPE
  // (A/B) table reads one row ahead: row r+1's reduction and (sin, cos)(k pi/128) read are issued
  // before row r's polynomial, so the LDS latency overlaps the previous row's five f64 operations
  // (same arithmetic per row: bit-identical)
  const double* tab = sr_trig_tab();
  SrTrigArg cur = sr_trig_arg(v[0], tab);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    SrTrigArg nxt = cur;
    if (r + 1 < R) nxt = sr_trig_arg(v[r + 1], tab);
    __builtin_amdgcn_sched_barrier(0);
    v[r] = sr_trig_poly<ID == SR_U_COS>(cur);
    __builtin_amdgcn_sched_barrier(0);
    cur = nxt;
  }
#else
#pragma unroll
  for (int r = 0; r < R; ++r) {
    v[r] = (ID == SR_U_COS) ? sr_cosf_fast(v[r]) : sr_sinf_fast(v[r]);
    SR_LIBM_ROW_END(r);
  }
#endif
  return v;
}

// Two rows per v_pk_* instruction (gfx950 packed fp32: v_pk_fma / v_pk_mul / v_pk_add).
using SrF2 = float __attribute__((ext_vector_type(2)));
__device__ __forceinline__ SrF2 sr_pk_fma(SrF2 a, SrF2 b, SrF2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float sr_min3_abs(float m, float a, float b) {
  float r;
  asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// Float32 exp over the rows.  When every row of the wave has |x| <= 88 (one ballot) this is the
// OCML expf sequence itself — ph = x*log2e, pl = fma(x, log2e_lo, fma(x, log2e, -ph)),
// exp2((ph - rint(ph)) + pl) * 2^rint(ph) — without its range selects, which are no-ops there (and
// without the evaluator's x > MAX_EXP test), with the rounding steps two rows per packed
// instruction and rint by the 1.5*2^23 shifter (exact for |ph| < 2^22): bit-identical results at
// about half the VALU issue.  Otherwise every row takes the full function.
template <int R>
__device__ __forceinline__ void sr_exp_rows_f32(float (&v)[R]) {
  static_assert(R % 2 == 0, "pairs of rows");
  float m = 0.0f;
#pragma unroll
  for (int r = 0; r < R; r += 2) m = SrMaxAbs<float>::step(m, v[r], v[r + 1]);
  if (__builtin_amdgcn_ballot_w64(!(m <= 88.0f)) == 0) {
    const SrF2 c = __builtin_bit_cast(float, 0x3fb8aa3bu);    // log2(e) rounded
    const SrF2 cc = __builtin_bit_cast(float, 0x32a5705fu);   // log2(e) - c
    const SrF2 sh = 0x1.8p23f;
#pragma unroll
    for (int r = 0; r < R; r += 2) {
      const SrF2 x = {v[r], v[r + 1]};
      const SrF2 ph = x * c;
      const SrF2 pl = sr_pk_fma(x, cc, sr_pk_fma(x, c, -ph));
      const SrF2 t = ph + sh;
      const SrF2 e = t - sh;
      const SrF2 f = (ph - e) + pl;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int k = int(e[q]);  // rint(ph), exact
        v[r + q] = __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f[q]), k);
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = sr_unary<float>(SR_U_EXP, v[r]);
  }
}

// Float32 a / b over the rows (IEEE, as Julia's `/`).  The library's correctly rounded division
// scales its operands (v_div_scale) and fixes up special cases (v_div_fixup) around a Newton /
// Markstein core: y = rcp(b) refined once, q = a*y corrected twice by the exact remainder
// fma(-b, q, a).  When |a| and |b| lie in [2^-40, 2^40] in every row of the wave the scaling is the
// identity and no intermediate over- or underflows (1/b and q within 2^+-80, remainders exact), so
// the bare core — its fma / mul steps two rows per packed instruction — returns the same correctly
// rounded quotient.  The range test is one max3 and one min3 per row and one ballot (a NaN operand
// is ignored by both and yields NaN through the core, as it must); a wave with any row outside it
// (zeros, infinities, huge or tiny values) takes the full division in every row.
// The full division over the rows as a real call (SR_DIV_FULL_CALL builds): the rarely taken branch
// of every division case then costs one call site instead of R inlined divisions (the 14 division
// cases of the register-stack kernel carried ~18 KB of such cold code).
template <int R>
__device__ __attribute__((noinline)) SrRowVec<R> sr_div_rows_full(SrRowVec<R> a, SrRowVec<R> b) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    a[r] = a[r] / b[r];
    __builtin_amdgcn_sched_barrier(0);
  }
  return a;
}
template <int R>
__device__ __forceinline__ void sr_div_rows_f32(float (&out)[R], const float (&a)[R], const float (&b)[R]) {
  static_assert(R % 2 == 0, "pairs of rows");
  float hi = 0.0f, lo = 0x1p40f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    hi = SrMaxAbs<float>::step(hi, a[r], b[r]);
    lo = sr_min3_abs(lo, a[r], b[r]);
  }
  if (__builtin_amdgcn_ballot_w64(!(hi <= 0x1p40f) || !(lo >= 0x1p-40f)) == 0) {
    const SrF2 one = 1.0f;
#pragma unroll
    for (int r = 0; r < R; r += 2) {
      const SrF2 A = {a[r], a[r + 1]};
      const SrF2 B = {b[r], b[r + 1]};
      SrF2 y = {__builtin_amdgcn_rcpf(b[r]), __builtin_amdgcn_rcpf(b[r + 1])};
      y = sr_pk_fma(sr_pk_fma(-B, y, one), y, y);
      SrF2 Q = A * y;
      Q = sr_pk_fma(sr_pk_fma(-B, Q, A), y, Q);
      Q = sr_pk_fma(sr_pk_fma(-B, Q, A), y, Q);
      out[r] = Q[0];
      out[r + 1] = Q[1];
    }
  } else {
#ifdef SR_DIV_FULL_CALL
    SrRowVec<R> va, vb;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      va[r] = a[r];
      vb[r] = b[r];
    }
    va = sr_div_rows_full<R>(va, vb);
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = va[r];
#else
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = a[r] / b[r];
#endif
  }
}

// A unary operator over a lane's R rows.  Float32 cos / sin take the Cody-Waite fast path for all
// rows unless some lane holds |x| >= 2^20 (one ballot: the Payne-Hanek path stays out of the
// common case).
template <typename T, uint32_t ID, int R>
__device__ __forceinline__ void sr_unary_rows(T (&v)[R]) {
  if constexpr (sizeof(T) == 4 && ID == SR_U_EXP && R % 2 == 0) {
    sr_exp_rows_f32<R>(v);
  } else if constexpr (sizeof(T) == 4 && (ID == SR_U_LOG || ID == SR_U_COS || ID == SR_U_SIN)) {
    SrRowVec<R> x;
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = v[r];
    bool slow = false;
    if constexpr (ID == SR_U_COS || ID == SR_U_SIN) {
      // max |x| over the rows (v_max3 ignores NaN, which the fast path maps to NaN itself)
      float m = 0.0f;
#pragma unroll
      for (int r = 0; r + 1 < R; r += 2) m = SrMaxAbs<float>::step(m, v[r], v[r + 1]);
      if constexpr (R % 2 != 0) m = SrMaxAbs<float>::step(m, v[R - 1], v[R - 1]);
      slow = !(m < srl::kTrigFastLimit);
    }
    if constexpr (ID == SR_U_LOG)
      x = sr_log_rows<R>(x);
    else if (__builtin_amdgcn_ballot_w64(slow) == 0)
      x = sr_trig_rows_fast<ID, R>(x);
    else
      x = sr_libm_rows<ID, R>(x);
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = x[r];
  } else if constexpr (sizeof(T) == 8 && (ID == SR_U_EXP || ID == SR_U_LOG || ID == SR_U_COS || ID == SR_U_SIN)) {
    SrRowVecD<ID, R> x;
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = v[r];
    x = sr_libm_rows_f64<ID, R>(x);
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = x[r];
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = sr_unary<T>(ID, v[r]);
  }
}

// A unary operator fused into the instruction computing its child (the POST field of the op word):
// the same row bodies as the UNARY opcodes; INF = DynamicExpressions' fused form (non-finite input ->
// +Inf), which only the per-node-check kernels distinguish (under deferred checks the input is a
// tracked operator output, so a non-finite input already decides the tree).
#define SR_POST_CASE(ID) \
  case ID:               \
    sr_unary_rows<T, ID, R>(tos); \
    break;
template <typename T, int R, int TIER, bool FAST>
__device__ __forceinline__ void sr_post_unary(uint32_t u, bool inf, T (&tos)[R]) {
  uint32_t nonfin = 0u;
  if constexpr (!FAST) {
    if (inf) {
#pragma unroll
      for (int r = 0; r < R; ++r) nonfin |= sr_isfinite(tos[r]) ? 0u : (1u << r);
    }
  }
  switch (u) {
    SR_POST_CASE(SR_U_NEG) SR_POST_CASE(SR_U_SQUARE) SR_POST_CASE(SR_U_CUBE) SR_POST_CASE(SR_U_EXP)
    SR_POST_CASE(SR_U_COS) SR_POST_CASE(SR_U_SIN) SR_POST_CASE(SR_U_LOG) SR_POST_CASE(SR_U_SQRT)
    SR_POST_CASE(SR_U_ABS)
    default:
      if constexpr (TIER == SR_TIER_FULL) {
        switch (u) {
          SR_POST_CASE(SR_U_TAN) SR_POST_CASE(SR_U_LOG2) SR_POST_CASE(SR_U_LOG10) SR_POST_CASE(SR_U_LOG1P)
          SR_POST_CASE(SR_U_SIGN) SR_POST_CASE(SR_U_TANH) SR_POST_CASE(SR_U_SINH) SR_POST_CASE(SR_U_COSH)
          SR_POST_CASE(SR_U_ATAN) SR_POST_CASE(SR_U_ASIN) SR_POST_CASE(SR_U_ACOS) SR_POST_CASE(SR_U_ACOSH)
          SR_POST_CASE(SR_U_ATANH) SR_POST_CASE(SR_U_ASINH) SR_POST_CASE(SR_U_RELU) SR_POST_CASE(SR_U_INV)
          SR_POST_CASE(SR_U_ERF) SR_POST_CASE(SR_U_ERFC) SR_POST_CASE(SR_U_GAMMA) SR_POST_CASE(SR_U_ROUND)
          SR_POST_CASE(SR_U_FLOOR) SR_POST_CASE(SR_U_CEIL) SR_POST_CASE(SR_U_EXP2) SR_POST_CASE(SR_U_EXPM1)
          default: break;
        }
      }
      break;
  }
  if constexpr (!FAST) {
    if (inf) {
#pragma unroll
      for (int r = 0; r < R; ++r) tos[r] = ((nonfin >> r) & 1u) ? sr_inf<T>() : tos[r];
    }
  }
}
#undef SR_POST_CASE

// ------------------------------------------------------------------ dispatch cases
#define SR_EACH(EXPR)                             \
  _Pragma("unroll") for (int r = 0; r < R; ++r) { \
    const T x = tos[r];                           \
    tos[r] = (EXPR);                              \
  }
#define SR_BIN_EACH(AEXPR, BEXPR, ID)                                     \
  if constexpr (sizeof(T) == 4 && (ID) == SR_B_DIV && R % 2 == 0) {       \
    T aa_[R], bb_[R];                                                     \
    _Pragma("unroll") for (int r = 0; r < R; ++r) {                       \
      aa_[r] = (AEXPR);                                                   \
      bb_[r] = (BEXPR);                                                   \
    }                                                                     \
    sr_div_rows_f32<R>(reinterpret_cast<float(&)[R]>(tos),                \
                       reinterpret_cast<const float(&)[R]>(aa_),          \
                       reinterpret_cast<const float(&)[R]>(bb_));         \
  } else {                                                                \
    _Pragma("unroll") for (int r = 0; r < R; ++r) {                       \
      const T aa = (AEXPR);                                               \
      const T bb = (BEXPR);                                               \
      tos[r] = sr_binary<T>(ID, aa, bb);                                  \
    }                                                                     \
  }
// Outputs the deferred checks need not track (SR_TRACK_LITE, round 5): bounded by 1 (cos, sin), by
// their input (neg, abs, sqrt: max(1, |x|)), or by the sum of their operands' magnitudes (+ and - of two
// stack values / features); the launch's tbig and BIG budget are divided by the largest tree's node
// count L, which bounds every untracked value by L x max(tracked max, max|x|, 1) (sr_capi.cpp
// run_batch).  Data at or above tbig / L runs the per-node-check (FULL tier) kernels instead.
#ifdef SR_TRACK_LITE
constexpr bool sr_untracked_u(uint32_t id) {
  return id == SR_U_COS || id == SR_U_SIN || id == SR_U_NEG || id == SR_U_ABS || id == SR_U_SQRT;
}
constexpr bool sr_untracked_b(uint32_t id) { return id == SR_B_ADD || id == SR_B_SUB; }
#else
constexpr bool sr_untracked_u(uint32_t) { return false; }
constexpr bool sr_untracked_b(uint32_t) { return false; }
#endif
// FAST_CHECK: every operator output joins the running max |v| of the tree
#define SR_TRACK()                                                        \
  if constexpr (FAST_CHECK && MODE == SR_MODE_LOSS) {                     \
    _Pragma("unroll") for (int r = 0; r < R; r += 4) {                    \
      mrun = SrMaxAbs<T>::step(mrun, tos[r], tos[r + 1]);                 \
      if (r + 3 < R) mrun1 = SrMaxAbs<T>::step(mrun1, tos[r + 2], tos[r + 3]); \
    }                                                                     \
  }
// The fused unary (UNARY_INF: non-finite input -> +Inf) needs its own body only where checks are
// per node: under the deferred checks (FAST_CHECK) the fused node's input is itself a tracked
// operator output, so a non-finite input already marks the tree incomplete and the fused node's
// value no longer matters — both opcodes share one body (half the transcendental code).
#define SR_UCASE_GEN(ID, ENABLED)                                   \
  case SR_OP_UNARY_INF0 + ID:                                       \
    if constexpr (!FAST_CHECK) {                                    \
      if (ENABLED) {                                                \
        SR_EACH(sr_isfinite(x) ? sr_unary<T>(ID, x) : sr_inf<T>()); \
        SR_TRACK();                                                 \
      }                                                             \
      break;                                                        \
    }                                                               \
    [[fallthrough]];                                                \
  case SR_OP_UNARY0 + ID: {                                         \
    if (ENABLED) {                                                  \
      sr_unary_rows<T, ID, R>(tos);                                 \
      if constexpr (!sr_untracked_u(ID)) SR_TRACK();                \
    }                                                               \
    break;                                                          \
  }
#define SR_UCASE(ID) SR_UCASE_GEN(ID, true)
#define SR_UCASE_FULL(ID) SR_UCASE_GEN(ID, TIER == SR_TIER_FULL)
// operand addresses: stack slot / feature row from the instruction's meta word (one shift: the
// flag bits above the index shift out of the 32-bit byte offset); constants from the c words
#define SR_OPND_STK() sr_row_at<ROWS>(stk_lane, SR_META())
#define SR_OPND_X() sr_row_at<ROWS>(x_lane, SR_META())
// stack operand: VSTK kernels keep the (at most two) operand-stack slots in VGPRs (s0, s1; the slot
// is the operand index); the others read the slot's rows from the wave's LDS stack area
// (SR_KEEP_BRANCH: an empty volatile asm in each arm keeps the wave-uniform slot choice a scalar
// branch; if-converted, LLVM selects every row of both slots with v_cndmask)
#define SR_KEEP_BRANCH() asm volatile("")
#define SR_STK_BIN(ID, LEFT)                                          \
  if constexpr (VSTK) {                                               \
    if (SR_VSTK_SLOTS == 1 || (SR_META() & SR_M_INDEX) == 0u) {       \
      SR_KEEP_BRANCH();                                               \
      SR_BIN_EACH((LEFT) ? s0[r] : tos[r], (LEFT) ? tos[r] : s0[r], ID); \
    } else {                                                          \
      SR_KEEP_BRANCH();                                               \
      SR_BIN_EACH((LEFT) ? s1[r] : tos[r], (LEFT) ? tos[r] : s1[r], ID); \
    }                                                                 \
  } else {                                                            \
    T o[R];                                                           \
    L::load(SR_OPND_STK(), o);                                        \
    SR_BIN_EACH((LEFT) ? o[r] : tos[r], (LEFT) ? tos[r] : o[r], ID);  \
  }
#define SR_BCASE_R(ID, ENABLED)        \
  case SR_BIN_OPC(ID, SR_V_SR): {      \
    if (ENABLED) {                     \
      SR_STK_BIN(ID, false);           \
      if constexpr (!sr_untracked_b(ID)) SR_TRACK(); \
    }                                  \
    break;                             \
  }                                    \
  case SR_BIN_OPC(ID, SR_V_FR): {      \
    if (ENABLED) {                     \
      T o[R];                          \
      L::load(SR_OPND_X(), o);         \
      SR_BIN_EACH(tos[r], o[r], ID);   \
      if constexpr (!sr_untracked_b(ID)) SR_TRACK(); \
    }                                  \
    break;                             \
  }                                    \
  case SR_BIN_OPC(ID, SR_V_CR): {      \
    if (ENABLED) {                     \
      const T cv = SR_CVAL();          \
      SR_BIN_EACH(tos[r], cv, ID);     \
      SR_TRACK();                      \
    }                                  \
    break;                             \
  }
#define SR_BCASE_L(ID, ENABLED)        \
  case SR_BIN_OPC(ID, SR_V_SL): {      \
    if (ENABLED) {                     \
      SR_STK_BIN(ID, true);            \
      if constexpr (!sr_untracked_b(ID)) SR_TRACK(); \
    }                                  \
    break;                             \
  }                                    \
  case SR_BIN_OPC(ID, SR_V_FL): {      \
    if (ENABLED) {                     \
      T o[R];                          \
      L::load(SR_OPND_X(), o);         \
      SR_BIN_EACH(o[r], tos[r], ID);   \
      if constexpr (!sr_untracked_b(ID)) SR_TRACK(); \
    }                                  \
    break;                             \
  }                                    \
  case SR_BIN_OPC(ID, SR_V_CL): {      \
    if (ENABLED) {                     \
      const T cv = SR_CVAL();          \
      SR_BIN_EACH(cv, tos[r], ID);     \
      SR_TRACK();                      \
    }                                  \
    break;                             \
  }
// PAIR instructions: op(leaf, leaf) with the first feature in meta, the second feature in c0 (FF)
// or the constant in the c words (FC / CF); the PUSH forms first store the old tos
#define SR_PCASE(ID, ENABLED, PV, BODY)                          \
  case SR_PAIR_OPC(ID, PV): {                                    \
    if (ENABLED) {                                               \
      BODY;                                                      \
      if constexpr (!(PV == SR_P_FF && sr_untracked_b(ID))) SR_TRACK(); \
    }                                                            \
    break;                                                       \
  }                                                              \
  case SR_PAIR_OPC(ID, PV + SR_P_PUSH): {                        \
    if (ENABLED) {                                               \
      SR_PUSH_TOS();                                             \
      BODY;                                                      \
      if constexpr (!(PV == SR_P_FF && sr_untracked_b(ID))) SR_TRACK(); \
    }                                                            \
    break;                                                       \
  }
#define SR_PAIR_FF(ID)                                                                   \
  T o[R];                                                                                \
  L::load(SR_OPND_X(), tos);                                                             \
  L::load(sr_row_at<ROWS>(x_lane, uint32_t(__builtin_amdgcn_readlane(int(wc0), int(k)))), o); \
  SR_BIN_EACH(tos[r], o[r], ID)
#define SR_PAIR_FC(ID)       \
  L::load(SR_OPND_X(), tos); \
  const T cv = SR_CVAL();    \
  SR_BIN_EACH(tos[r], cv, ID)
#define SR_PAIR_CF(ID)       \
  L::load(SR_OPND_X(), tos); \
  const T cv = SR_CVAL();    \
  SR_BIN_EACH(cv, tos[r], ID)
#define SR_PCASES_R(ID, ENABLED) \
  SR_PCASE(ID, ENABLED, SR_P_FF, SR_PAIR_FF(ID)) SR_PCASE(ID, ENABLED, SR_P_FC, SR_PAIR_FC(ID))
#define SR_PCASES(ID, ENABLED) SR_PCASES_R(ID, ENABLED) SR_PCASE(ID, ENABLED, SR_P_CF, SR_PAIR_CF(ID))

// + and * commute: the compiler emits only their R variants (and no CF pairs)
#define SR_BCASE_COMM(ID) SR_BCASE_R(ID, true) SR_PCASES_R(ID, true)
#define SR_BCASE(ID) SR_BCASE_R(ID, true) SR_BCASE_L(ID, true) SR_PCASES(ID, true)
#define SR_BCASE_FULL(ID) \
  SR_BCASE_R(ID, TIER == SR_TIER_FULL) SR_BCASE_L(ID, TIER == SR_TIER_FULL) SR_PCASES(ID, TIER == SR_TIER_FULL)

// LDS carve, in bytes, 16-aligned: X tile [nf][ROWS] T | y [ROWS] | w [ROWS] (weighted) | stack
// [W][depth][ROWS] T | EXACT mode: checked values [W][max_checks][ROWS] T and the running Julia-order
// sums [G][max_checks] T | program cache [code_lds] 16-byte instructions (LOSS)
template <typename T>
struct SrLdsPlan {
  size_t x, y, w, stk, chk, jst, code, total;
  __host__ __device__ SrLdsPlan(int nf, int rows, int depth, int G, int max_checks, int waves, bool weighted,
                                int code_lds = 0) {
    size_t o = 0;
    x = o;
    o += size_t(nf) * rows * sizeof(T);
    y = o;
    o += size_t(rows) * sizeof(T);
    w = o;
    if (weighted) o += size_t(rows) * sizeof(T);
    stk = o;
    o += size_t(waves) * size_t(depth) * rows * sizeof(T);
    chk = o;
    o += size_t(waves) * size_t(max_checks) * rows * sizeof(T);
    jst = o;
    o += (size_t(G) * size_t(max_checks) * sizeof(T) + 15) / 16 * 16;
    code = o;
    o += size_t(code_lds) * 16;
    total = o;
  }
};

__device__ __forceinline__ uint4 sr_load_window(const void* code, uint32_t at) {
  return *reinterpret_cast<const uint4*>(static_cast<const unsigned char*>(code) + size_t(at) * 16u);
}

// The tile interpreter's program window: instructions base .. base+SR_WIN-1 (those before `end`),
// one per lane.  f32 programs load only the words they use (op, meta, c0): a loaded-but-dead c1
// register would be reused as a temporary while the prefetch is in flight, which makes the
// interpreter wait for the prefetch (vmcnt) at its first use of that register.
// (An end-of-window opcode handled inside the switch would give the interpreter loop a second exit,
// which the AMDGPU structurizer turns into per-iteration register copies: the trip count stays.)
constexpr uint32_t SR_WIN = 64u;
template <typename T>
struct SrWindow {
  using type = uint4;
  __device__ static __forceinline__ type load(const void* code, uint32_t at) { return sr_load_window(code, at); }
  __device__ static __forceinline__ uint32_t c1(const type& w) { return w.w; }
};
template <>
struct SrWindow<float> {
  using type = uint3;
  __device__ static __forceinline__ type load(const void* code, uint32_t at) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(static_cast<const unsigned char*>(code) + size_t(at) * 16u);
    return make_uint3(p[0], p[1], p[2]);
  }
  __device__ static __forceinline__ uint32_t c1(const type&) { return 0u; }
};
template <typename T>
__device__ __forceinline__ typename SrWindow<T>::type sr_window(const void* code, uint32_t base, uint32_t end,
                                                                int lane) {
  typename SrWindow<T>::type w{};
  if (base + uint32_t(lane) < end) w = SrWindow<T>::load(code, base + uint32_t(lane));
  return w;
}
// the same window from the workgroup's LDS program cache (ds_read instead of a global load: the next
// tree's window arrives within the current short tree's run)
template <typename T>
__device__ __forceinline__ typename SrWindow<T>::type sr_window_lds(const uint4* lcode, uint32_t base, uint32_t end,
                                                                    int lane) {
  typename SrWindow<T>::type w{};
  if (base + uint32_t(lane) < end) {
    const uint4 v = lcode[base + uint32_t(lane)];
    if constexpr (sizeof(T) == 4) w = make_uint3(v.x, v.y, v.z);
    else w = v;
  }
  return w;
}

// ------------------------------------------------------------------ the interpreter kernel
// SR_STAMP(k): latency-analysis builds only (-DSR_STAMPS, tools/stamps.py): lane 0 of each wave
// records the wall clock at point k (0 entry, 1 prologue issued, 2 first tile staged, 3 first window
// consumed, 4 first tile's trees done, 5 all tiles done, 6 results written)
#ifdef SR_STAMPS
#define SR_STAMP(k)                                                                              \
  do {                                                                                           \
    if (a.stamps && lane == 0)                                                                   \
      a.stamps[(size_t(blockIdx.x) * size_t(W) + size_t(wave)) * SR_NSTAMPS + (k)] = wall_clock64(); \
  } while (0)
#else
#define SR_STAMP(k) ((void)0)
#endif
// MODE: SR_MODE_LOSS (partials), SR_MODE_PRED (write predictions), SR_MODE_EXACT (Julia-order sums of
// the checked arrays over row ranges: DynamicExpressions' isfinite(sum(x)) decided exactly as Base's
// pairwise `sum` computes it in T; a "row block" is one range of a.range_lo/range_hi).
//
// Tree ownership: the block's G trees are positions tree0 .. tree0+G-1 of the launch order
// (a.perm maps a position to the caller's tree index: the host orders trees by estimated cost so
// the waves of a block get equal work).  Wave w owns positions tree0 + w + W*j ("slot" j, j < 64);
// everything per tree lives in that wave: program bounds in lane j's VGPRs, the loss accumulator in
// lane j, the non-finite / suspicious bits in scalar masks.
// LK: elementwise loss fixed at compile time (SR_LOSS_L2 / SR_LOSS_L1), or -1 = a.loss_kind.
// VSTK: the operand stack (<= 2 slots: every tree of <= 30 nodes) lives in VGPRs.
template <typename T, int R, int MODE, bool GATHER, int TIER, int W, int LK, bool VSTK>
__global__ void __launch_bounds__(W * 64, (SrMinWavesFor<T, R, TIER, W, VSTK, LK, GATHER, MODE>::value)) sr_tile_kernel(const SrEvalArgs<T> a) {
  constexpr int SR_WAVES = W;
  constexpr int SR_BLOCK = W * 64;
  using L = SrLane<T, R>;
  constexpr int C = L::C;
  constexpr int ROWS = 64 * R;
  // Deferred validity checks (BASIC tier loss kernels): no per-node branch, ballot or
  // early exit; the tree's running max |v| and the root's NaN test decide at the end of the program.
  // FOLD mode runs complete trees only: the deferred-check kernels' operator bodies (FAST_CHECK), no
  // tracking (SR_TRACK), no per-node checks
  constexpr bool FAST_CHECK = (TIER == SR_TIER_BASIC) && (MODE == SR_MODE_LOSS || MODE == SR_MODE_FOLD);
  constexpr bool NODE_CHECKS = !FAST_CHECK && MODE != SR_MODE_FOLD;
  static_assert(R % 4 == 0 || R == 2, "rows per lane: 2 or a multiple of 4");
  extern __shared__ __attribute__((aligned(16))) unsigned char sr_smem[];
  const int tid = threadIdx.x;
#ifndef SR_WAVE_VGPR
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform: per-wave values in SGPRs)
#else
  const int wave = tid >> 6;
#endif
  const int lane = tid & 63;
  SR_STAMP(0);
  const int G = a.trees_per_block;
  const int MC = (MODE == SR_MODE_EXACT) ? a.max_checks : 0;
  const SrLdsPlan<T> plan(a.nf, ROWS, VSTK ? 0 : a.stack_depth, G, MC, W, a.w != nullptr,
                          (MODE == SR_MODE_LOSS || MODE == SR_MODE_FOLD) ? a.code_lds : 0);
  T* xs = reinterpret_cast<T*>(sr_smem + plan.x);
  T* ys = reinterpret_cast<T*>(sr_smem + plan.y);
  T* wsv = reinterpret_cast<T*>(sr_smem + plan.w);
  T* chk = reinterpret_cast<T*>(sr_smem + plan.chk);  // EXACT: [W][MC][ROWS] checked values of a tile
  T* jst = reinterpret_cast<T*>(sr_smem + plan.jst);  // EXACT: [G][MC] running sums
  const T* x_lane = xs + lane * C;
  const T* y_lane = ys + lane * C;
  const T* w_lane = wsv + lane * C;
  T* stk_lane = reinterpret_cast<T*>(sr_smem + plan.stk) + size_t(wave) * a.stack_depth * ROWS + lane * C;

  // tree group fastest: the blocks resident at one time share few row blocks (X stays in L2)
  int tg, rb, tree0, gcount;
  const int64_t* ridx = a.row_idx;  // GATHER: this block's row view
  if (a.segs == nullptr) {
    tg = int(blockIdx.x) % a.n_groups;
    rb = int(blockIdx.x) / a.n_groups;
    tree0 = tg * G;
    gcount = a.n_trees - tree0;
  } else {
    // several row views in one launch (sr_eval_loss_batch_views): segment s = the launch positions
    // of view s's trees, its own tree groups; its blocks follow the previous segments' (block0)
    int lo = 0, hi = a.n_segs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.segs[mid].block0 <= int(blockIdx.x)) lo = mid;
      else hi = mid - 1;
    }
    const SrSegment sg = a.segs[lo];
    const int local = int(blockIdx.x) - sg.block0;
    tg = local % sg.groups;
    rb = local / sg.groups;
    tree0 = sg.pos0 + tg * G;
    gcount = sg.pos0 + sg.n_pos - tree0;
    ridx += sg.row_off;
  }
  if (gcount > G) gcount = G;
  const bool weighted = a.w != nullptr;
  const uint32_t thr = SrBits<T>::mag(a.tbig);
  // tbig held in a register for the whole kernel: left as a kernel argument, the per-tree epilogue
  // re-reads it with a scalar load and a full lgkmcnt wait under the kernel's SGPR pressure
  T tbig = a.tbig;
  asm volatile("" : "+v"(tbig));
  const int lk = LK >= 0 ? LK : a.loss_kind;

  // this wave's slots
  const int S = gcount > wave ? (gcount - wave + SR_WAVES - 1) / SR_WAVES : 0;
  const int my_pos = tree0 + wave + SR_WAVES * lane;
  uint32_t my_pb = 0u, my_pe = 0u;
  if (lane < S) {
    const uint32_t t = a.perm ? a.perm[my_pos] : uint32_t(my_pos);
    my_pb = a.offsets[t];
    my_pe = a.ends ? a.ends[t] : a.offsets[t + 1];
  }
  // LDS program cache (LOSS): the group's programs are one contiguous span of the launch-ordered code
  // (first position's start .. last position's end); copied once, read by every tile's windows
  const uint4* lcode = reinterpret_cast<const uint4*>(sr_smem + plan.code);
  bool lds_code = false;
  if ((MODE == SR_MODE_LOSS || MODE == SR_MODE_FOLD) && a.code_lds > 0 && a.ends != nullptr && gcount > 0) {
    const uint32_t t_first = a.perm ? a.perm[tree0] : uint32_t(tree0);
    const uint32_t t_last = a.perm ? a.perm[tree0 + gcount - 1] : uint32_t(tree0 + gcount - 1);
    const uint32_t gbase = __builtin_amdgcn_readfirstlane(a.offsets[t_first]);
    const uint32_t gend = __builtin_amdgcn_readfirstlane(a.ends[t_last]);
    if (gend >= gbase && gend - gbase <= uint32_t(a.code_lds)) {
      lds_code = true;
      const uint4* src = reinterpret_cast<const uint4*>(a.code) + gbase;
      uint4* dst = reinterpret_cast<uint4*>(sr_smem + plan.code);
      for (uint32_t i = uint32_t(tid); i < gend - gbase; i += uint32_t(SR_BLOCK)) dst[i] = src[i];
      if (lane < S) {
        my_pb -= gbase;
        my_pe -= gbase;
      }
    }
  }
  // FOLD: this row block's plan code of each of the wave's trees (lane j: tree j); SKIP trees are not run
  int32_t my_code = SR_FCODE_SKIP, my_sq = SR_FCODE_SKIP;  // (my_sq: a slow segment's lower window binade)
  if (MODE == SR_MODE_FOLD && lane < S) {
    my_code = a.fold_code[size_t(rb) * size_t(a.n_trees) + size_t(my_pos)];
    if (my_code >= SR_FCODE_SLOT0 && a.fold_sq) my_sq = a.fold_sq[size_t(rb) * size_t(a.n_trees) + size_t(my_pos)];
  }
  const uint64_t live = sr_ballot(lane < S && my_pe > my_pb &&  // empty program: statically incomplete
                                  (MODE != SR_MODE_FOLD || my_code != SR_FCODE_SKIP));
  // FOLD: lane j's tree's composed steps over this row block (a slow segment's: under my_sq, and under
  // my_sq + 1 in facc2 / facc3)
  typename SrFoldTab<T>::I facc0 = 0, facc1 = 0, facc2 = 0, facc3 = 0;
  uint64_t dmask = 0u, bmask = 0u, emask = 0u;
  double accv = 0.0;
  // dead-tree hints shared across row blocks (LOSS mode): a tree found non-finite by any block is
  // skipped by blocks that start it later.  Loaded one tile ahead; only ever a hint (a skipped
  // tree is reported non-finite, which the discovering block reports anyway).
  const bool use_hint = (MODE == SR_MODE_LOSS) && a.hint != nullptr;
  uint32_t hintv = 0u;
  if (use_hint && lane < S) hintv = __hip_atomic_load(a.hint + my_pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  for (int i = tid; i < G * MC; i += SR_BLOCK) jst[i] = T(0);
  sr_libm_lds_fill(tid, SR_BLOCK);  // (visible after the first tile's barrier)
  // EXACT: this block's row range [rlo, rhi] of the view (one leaf block of Julia's pairwise sum)
  const int64_t rlo = (MODE == SR_MODE_EXACT) ? a.range_lo[rb] : 0;
  const int64_t rhi = (MODE == SR_MODE_EXACT) ? a.range_hi[rb] : 0;
  SR_STAMP(1);

  for (int tile = 0; tile < a.tiles_per_block; ++tile) {
    const int64_t row0 = (MODE == SR_MODE_EXACT) ? rlo + int64_t(tile) * ROWS
                                                 : (int64_t(rb) * a.tiles_per_block + tile) * ROWS;
    if (MODE == SR_MODE_EXACT ? row0 > rhi : row0 >= a.n_rows) break;  // uniform over the block
    const bool full_tile = row0 + ROWS <= a.n_rows;
    const int n_valid = (MODE == SR_MODE_EXACT) ? int(rhi - row0 + 1 < ROWS ? rhi - row0 + 1 : ROWS) : ROWS;
    __syncthreads();              // previous tile's readers are done with the LDS image
    // ---- stage the tile: X rows of every feature, y, w (a plain copy; padded rows replicate
    // row 0 of the view, so every program sees finite, in-range data there)
    if (MODE == SR_MODE_EXACT) {
      // a range starts anywhere: element-wise loads; rows past the range replicate its first row.
      // The thread's rows' sources first, then the loads of up to 4 features at a time, all in
      // flight before the LDS stores (one memory latency per 4 features, not one per element)
      constexpr int PER = (ROWS + SR_BLOCK - 1) / SR_BLOCK;
      int64_t src[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int i = tid + q * SR_BLOCK;
        const int64_t v = (i < n_valid) ? row0 + i : rlo;
        src[q] = (i < ROWS) ? (GATHER ? ridx[v] : v) : rlo;
      }
      for (int f0 = 0; f0 < a.nf; f0 += 4) {
        T v[4][PER];
#pragma unroll
        for (int df = 0; df < 4; ++df) {
          const int f = f0 + df < a.nf ? f0 + df : f0;
#pragma unroll
          for (int q = 0; q < PER; ++q) v[df][q] = a.X[int64_t(f) * a.ld + src[q]];
        }
#pragma unroll
        for (int df = 0; df < 4; ++df) {
#pragma unroll
          for (int q = 0; q < PER; ++q) {
            const int i = tid + q * SR_BLOCK;
            if (f0 + df < a.nf && i < ROWS) xs[(f0 + df) * ROWS + i] = v[df][q];
          }
        }
      }
    } else if (!GATHER) {
      constexpr int CPR = ROWS / C;  // 16-byte chunks per feature row
      using V = typename SrChunk<T>::V;
      const int n_chunks = a.nf * CPR;
      for (int i = tid; i < n_chunks; i += SR_BLOCK) {
        const int f = i / CPR, q = i - f * CPR;
        reinterpret_cast<V*>(xs)[i] = *reinterpret_cast<const V*>(a.X + int64_t(f) * a.ld + row0 + q * C);
      }
      if (MODE != SR_MODE_EXACT && a.y) {
        for (int i = tid; i < CPR; i += SR_BLOCK) {
          reinterpret_cast<V*>(ys)[i] = *reinterpret_cast<const V*>(a.y + row0 + i * C);
          if (weighted) reinterpret_cast<V*>(wsv)[i] = *reinterpret_cast<const V*>(a.w + row0 + i * C);
        }
      }
    } else {
      for (int i = tid; i < ROWS; i += SR_BLOCK) {
        const int64_t v = row0 + i;
        const int64_t src = ridx[v < a.n_rows ? v : 0];
        for (int f = 0; f < a.nf; ++f) xs[f * ROWS + i] = a.X[int64_t(f) * a.ld + src];
        if (MODE != SR_MODE_EXACT && a.y) {
          ys[i] = a.y[src];
          if (weighted) wsv[i] = a.w[src];
        }
      }
    }
    __syncthreads();
    if (tile == 0) SR_STAMP(2);

    if (use_hint) {
      dmask |= sr_ballot(hintv == a.hint_epoch) & live;
      if (lane < S) hintv = __hip_atomic_load(a.hint + my_pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t todo = (MODE == SR_MODE_LOSS) ? (live & ~dmask) : live;
    if (!todo) continue;
    // Window stream: the 64-instruction program windows of this tile's trees, in order.  The next
    // window (of this tree, or the first one of the next tree) is in flight while the current one
    // runs; the running window is a register copy, so the interpreter loop never waits on it.
    int nj = __builtin_ctzll(todo);
    todo &= todo - 1u;
    uint32_t nb = uint32_t(__builtin_amdgcn_readlane(int(my_pb), nj));
    uint32_t ne = uint32_t(__builtin_amdgcn_readlane(int(my_pe), nj));
    typename SrWindow<T>::type nx = lds_code ? sr_window_lds<T>(lcode, nb, ne, lane) : sr_window<T>(a.code, nb, ne, lane);
    int j = -1;
    uint32_t tpe = 0u;
#ifdef SR_STAMPS
    const uint32_t nb0 = nb;
#endif
    T tos[R];
    T s0[R];  // VSTK operand-stack slots
#if SR_VSTK_SLOTS > 1
    T s1[R];
#else
    T* const s1 = s0;  // (never selected: one-slot kernels take no second-slot programs)
#endif
#pragma unroll
    for (int r = 0; r < R; ++r) tos[r] = s0[r] = T(0);
#if SR_VSTK_SLOTS > 1
#pragma unroll
    for (int r = 0; r < R; ++r) s1[r] = T(0);
#endif
    bool dead = false;
    bool susp_any = false;
    int check_k = 0;
    T mrun = T(0), mrun1 = T(0);  // FAST_CHECK: running max |v| over this lane's rows (2 chains)
    bool more = true;
    while (more) {
      const typename SrWindow<T>::type cw = nx;
      const uint32_t base = nb;
      if (nj != j) {  // a new tree starts (its first instruction is a LOAD: tos needs no reset)
        j = nj;
        tpe = ne;
        dead = false;
        susp_any = false;
        check_k = 0;
        mrun = T(0);
        mrun1 = T(0);
      }
      if (base + SR_WIN < tpe) {
        nb = base + SR_WIN;
      } else if (todo) {
        nj = __builtin_ctzll(todo);
        todo &= todo - 1u;
        nb = uint32_t(__builtin_amdgcn_readlane(int(my_pb), nj));
        ne = uint32_t(__builtin_amdgcn_readlane(int(my_pe), nj));
      } else {
        more = false;
      }
      if (more) nx = lds_code ? sr_window_lds<T>(lcode, nb, ne, lane) : sr_window<T>(a.code, nb, ne, lane);
      const int g = wave + SR_WAVES * j;

      if (!dead) {
        const uint32_t wop = cw.x, wmeta = cw.y, wc0 = cw.z, wc1 = SrWindow<T>::c1(cw);
        const uint32_t n_here = __builtin_amdgcn_readfirstlane((tpe - base < SR_WIN) ? tpe - base : SR_WIN);
        // single-exit loop (a dead tree sets k past the window): a second loop exit would make
        // LLVM add an exit-selector block to every iteration
#ifdef SR_STAMPS
        if (tile == 0 && base == nb0) SR_STAMP(3);
#endif
#ifdef SR_OP_PREFETCH
        // the next instruction's op word read one iteration ahead (lane k + 1 of the window; the
        // read of lane 64 wraps to lane 0 and is never used): the scalar dispatch chain starts
        // without waiting on the VALU -> SGPR read of its own op
        uint32_t op_next = uint32_t(__builtin_amdgcn_readlane(int(wop), 0));
#endif
        for (uint32_t k = 0; k < n_here; ++k) {
#ifdef SR_OP_PREFETCH
          const uint32_t op = op_next;
          op_next = uint32_t(__builtin_amdgcn_readlane(int(wop), int((k + 1u) & 63u)));
#else
          const uint32_t op = uint32_t(__builtin_amdgcn_readlane(int(wop), int(k)));
#endif
#define SR_CVAL() sr_lane_value<T>(wc0, wc1, k)
#define SR_META() uint32_t(__builtin_amdgcn_readlane(int(wmeta), int(k)))
#define SR_PUSH_TOS()                                                                        \
  if constexpr (VSTK) {                                                                      \
    if (SR_VSTK_SLOTS == 1 || ((SR_META() >> SR_M_PUSH_SHIFT) & 0x3fu) == 1u) {              \
      SR_KEEP_BRANCH();                                                                      \
      _Pragma("unroll") for (int r = 0; r < R; ++r) s0[r] = tos[r];                          \
    } else {                                                                                 \
      SR_KEEP_BRANCH();                                                                      \
      _Pragma("unroll") for (int r = 0; r < R; ++r) s1[r] = tos[r];                          \
    }                                                                                        \
  } else {                                                                                   \
    L::store(sr_row_at<ROWS>(stk_lane, ((SR_META() >> SR_M_PUSH_SHIFT) & 0x3fu) - 1u), tos); \
  }
          switch (op & SR_OP_MASK) {
            case SR_OP_LOAD_FEAT_PUSH:
              SR_PUSH_TOS();
              [[fallthrough]];
            case SR_OP_LOAD_FEAT: {
              L::load(SR_OPND_X(), tos);
              // a checked feature array (the child of a general unary node) joins the deferred checks
              // when the data itself can be non-finite or huge (uniform: a dataset property)
              if (FAST_CHECK && a.track_x && (SR_META() & SR_M_CHECK)) {
                SR_TRACK();
              }
              break;
            }
            case SR_OP_LOAD_DERIVED_PUSH:
              SR_PUSH_TOS();
              [[fallthrough]];
            case SR_OP_LOAD_DERIVED: {
              // unary(feature) from the call's derived columns (same chunk layout as the LDS tile,
              // read straight from global memory); the node is an operator output: tracked
              if constexpr (FAST_CHECK) {
                L::load(a.derived + size_t(SR_META() & SR_M_INDEX) * size_t(a.dld) + size_t(row0) + size_t(lane * C), tos);
                SR_TRACK();
              } else {
                // other kernels running a LOSS program (the exact-sum pass): the node in place,
                // op_u(X[f]) with (u, f) from c0, exactly as the column was computed
                const uint32_t uf = uint32_t(__builtin_amdgcn_readlane(int(wc0), int(k)));
                L::load(sr_row_at<ROWS>(x_lane, uf & 0xffffu), tos);
                switch (uf >> 16) {
                  case SR_U_EXP: sr_unary_rows<T, SR_U_EXP, R>(tos); break;
                  case SR_U_COS: sr_unary_rows<T, SR_U_COS, R>(tos); break;
                  case SR_U_SIN: sr_unary_rows<T, SR_U_SIN, R>(tos); break;
                  case SR_U_LOG: sr_unary_rows<T, SR_U_LOG, R>(tos); break;
                  case SR_U_SQRT: sr_unary_rows<T, SR_U_SQRT, R>(tos); break;
                  default: break;
                }
              }
              break;
            }
            case SR_OP_LOAD_CONST_PUSH:
              SR_PUSH_TOS();
              [[fallthrough]];
            case SR_OP_LOAD_CONST: {
              const T cv = SR_CVAL();
#pragma unroll
              for (int r = 0; r < R; ++r) tos[r] = cv;
              // (a constant leaf is an operand of its parent: LOAD_CONST is only ever a constant
              // tree's root, which the deferred checks must see like every other root)
              SR_TRACK();
              break;
            }
            // BASIC tier
            SR_UCASE(SR_U_NEG) SR_UCASE(SR_U_SQUARE) SR_UCASE(SR_U_CUBE) SR_UCASE(SR_U_EXP)
            SR_UCASE(SR_U_COS) SR_UCASE(SR_U_SIN) SR_UCASE(SR_U_LOG) SR_UCASE(SR_U_SQRT)
            SR_UCASE(SR_U_ABS)
            SR_BCASE_COMM(SR_B_ADD) SR_BCASE_COMM(SR_B_MUL) SR_BCASE(SR_B_SUB) SR_BCASE(SR_B_DIV)
            // FULL tier
            SR_UCASE_FULL(SR_U_TAN) SR_UCASE_FULL(SR_U_LOG2) SR_UCASE_FULL(SR_U_LOG10)
            SR_UCASE_FULL(SR_U_LOG1P) SR_UCASE_FULL(SR_U_SIGN) SR_UCASE_FULL(SR_U_TANH)
            SR_UCASE_FULL(SR_U_SINH) SR_UCASE_FULL(SR_U_COSH) SR_UCASE_FULL(SR_U_ATAN)
            SR_UCASE_FULL(SR_U_ASIN) SR_UCASE_FULL(SR_U_ACOS) SR_UCASE_FULL(SR_U_ACOSH)
            SR_UCASE_FULL(SR_U_ATANH) SR_UCASE_FULL(SR_U_ASINH) SR_UCASE_FULL(SR_U_RELU)
            SR_UCASE_FULL(SR_U_INV) SR_UCASE_FULL(SR_U_ERF) SR_UCASE_FULL(SR_U_ERFC)
            SR_UCASE_FULL(SR_U_GAMMA) SR_UCASE_FULL(SR_U_ROUND) SR_UCASE_FULL(SR_U_FLOOR)
            SR_UCASE_FULL(SR_U_CEIL) SR_UCASE_FULL(SR_U_EXP2) SR_UCASE_FULL(SR_U_EXPM1)
            SR_BCASE_FULL(SR_B_POW) SR_BCASE_FULL(SR_B_MAX) SR_BCASE_FULL(SR_B_MIN)
            SR_BCASE_FULL(SR_B_MOD) SR_BCASE_FULL(SR_B_GREATER) SR_BCASE_FULL(SR_B_LESS)
            SR_BCASE_FULL(SR_B_GREATER_EQUAL) SR_BCASE_FULL(SR_B_LESS_EQUAL) SR_BCASE_FULL(SR_B_COND)
            SR_BCASE_FULL(SR_B_LOGICAL_OR) SR_BCASE_FULL(SR_B_LOGICAL_AND) SR_BCASE_FULL(SR_B_ATAN2)
            default:
              break;
          }
#undef SR_PUSH_TOS
          // DynamicExpressions' check of a node's output array (per node: FULL tier, PRED, EXACT)
#define SR_CHECK_NODE()                                                                                      \
  if (MODE == SR_MODE_EXACT) {                                                                               \
    /* the checked array's rows of this tile, in row order, for the Julia-order fold below */                \
    if (check_k < MC) L::store(chk + (size_t(wave) * MC + check_k) * ROWS + lane * C, tos);                  \
    ++check_k;                                                                                               \
  } else {                                                                                                   \
    /* |v| >= tbig (or NaN / Inf) in any row: one integer max per lane + one ballot; padded rows */          \
    /* replicate row 0 of the view, so no row mask is needed here */                                         \
    uint32_t m = SrBits<T>::mag(tos[0]);                                                                     \
    _Pragma("unroll") for (int r = 1; r < R; ++r) m = max(m, SrBits<T>::mag(tos[r]));                       \
    if (sr_ballot(m >= thr)) {                                                                               \
      susp_any = true;                                                                                       \
      bool nonfin = false;                                                                                   \
      _Pragma("unroll") for (int r = 0; r < R; ++r) nonfin |= !sr_isfinite(tos[r]);                         \
      if (sr_ballot(nonfin)) {                                                                               \
        dead = true;                                                                                         \
        k = SR_WIN;                                                                                          \
      }                                                                                                      \
    }                                                                                                        \
  }
          if (NODE_CHECKS && (SR_META() & SR_M_CHECK)) {
            SR_CHECK_NODE();
          }
          // the POST unary and the post binary with a constant (PBC) fused into this instruction (the
          // node whose child it computed, then that node's parent): ONE test of the op word's upper
          // half on the common path (most instructions carry neither)
          if ((op >> SR_OP_POST_SHIFT) != 0u && !dead) {
            const uint32_t post = (op >> SR_OP_POST_SHIFT) & 0x3fu;
            if (post != 0u) {
              // (an opaque copy: LLVM would otherwise fold the test above into the post switch's
              //  balanced compare tree)
              uint32_t pu = post;
#ifndef SR_POST_FOLDED
              asm volatile("" : "+s"(pu));
#endif
              sr_post_unary<T, R, TIER, FAST_CHECK>(pu, (op & SR_OP_POST_INF) != 0u, tos);
#ifdef SR_TRACK_LITE
              if (!sr_untracked_u(pu))
#endif
              SR_TRACK();
              if (NODE_CHECKS && (op & SR_OP_POST_CHECK)) {
                SR_CHECK_NODE();
              }
            }
            const uint32_t pbc = (op >> SR_OP_PBC_SHIFT) & 7u;
            if (pbc != 0u && !dead) {
              // the same row bodies as the CR / CL instructions (a constant operand: always tracked)
              const T cv = SR_CVAL();
              switch (pbc) {
                case SR_PBC_ADD: { SR_BIN_EACH(tos[r], cv, SR_B_ADD); break; }
                case SR_PBC_SUB_R: { SR_BIN_EACH(tos[r], cv, SR_B_SUB); break; }
                case SR_PBC_SUB_L: { SR_BIN_EACH(cv, tos[r], SR_B_SUB); break; }
                case SR_PBC_MUL: { SR_BIN_EACH(tos[r], cv, SR_B_MUL); break; }
                case SR_PBC_DIV_R: { SR_BIN_EACH(tos[r], cv, SR_B_DIV); break; }
                default: { SR_BIN_EACH(cv, tos[r], SR_B_DIV); break; }
              }
              SR_TRACK();
              if (NODE_CHECKS && (op & SR_OP_PBC_CHECK)) {
                SR_CHECK_NODE();
              }
            }
          }
#undef SR_CHECK_NODE
#undef SR_CVAL
        }
      }

      if (base + SR_WIN >= tpe) {  // tree j is done on this tile
        const uint64_t bit = uint64_t(1) << j;
        if (MODE == SR_MODE_EXACT) {
          // Base.mapreduce_impl's sequential leaf loop, v = v + a[i] in T, continued across the
          // range's tiles (lane k folds check k; the first row of the range starts the fold)
          __builtin_amdgcn_wave_barrier();
#ifdef SR_EXACT_NOFOLD
          const int nk = 0;  // (timing experiment only: the exact pass without its sequential folds)
#else
          const int nk = check_k < MC ? check_k : MC;
#endif
          for (int k = lane; k < nk; k += 64) {
            const T* cb = chk + (size_t(wave) * MC + k) * ROWS;
            T v = (tile == 0) ? cb[0] : jst[g * MC + k];
            int i = (tile == 0) ? 1 : 0;
            // the adds stay sequential in row order; the LDS reads go 16 rows at a time (16-byte
            // reads all in flight before the adds) instead of one latency per row
            for (; i < n_valid && (i & 3); ++i) v = v + cb[i];
            for (; i + 16 <= n_valid; i += 16) {
              using V = typename SrChunk<T>::V;
              constexpr int CH = SrChunk<T>::N;
              T blk[16];
#pragma unroll
              for (int q = 0; q < 16; q += CH) SrChunk<T>::get(*reinterpret_cast<const V*>(cb + i + q), blk + q);
#pragma unroll
              for (int q = 0; q < 16; ++q) v = v + blk[q];
            }
            for (; i < n_valid; ++i) v = v + cb[i];
            jst[g * MC + k] = v;
          }
          __builtin_amdgcn_wave_barrier();
        } else if (MODE == SR_MODE_LOSS) {
          if (!dead) {
            T l[R];
            T yv[R];
            L::load(y_lane, yv);
            if (weighted) {
              T wv[R];
              L::load(w_lane, wv);
#pragma unroll
              for (int r = 0; r < R; ++r) l[r] = sr_elem_loss<T>(lk, tos[r], yv[r], a.loss_param) * wv[r];
            } else {
#pragma unroll
              for (int r = 0; r < R; ++r) l[r] = sr_elem_loss<T>(lk, tos[r], yv[r], a.loss_param);
            }
            if (!full_tile) {  // rows past the end of the view (padding) do not count
#pragma unroll
              for (int r = 0; r < R; ++r) l[r] = (row0 + L::row(lane, r) < a.n_rows) ? l[r] : T(0);
            }
            // (small calls under the in-order fold: every live tree's losses, the fold's tables are
            //  composed from them; a tree found dead later leaves garbage the fold never reads)
            if (a.fold_loss) L::store(a.fold_loss + size_t(tree0 + g) * size_t(a.fold_pos_stride) + size_t(row0) + lane * C, l);
            // pairwise over the lane's rows by halves (rows r and r + h: adjacent pairs of rows add as
            // one packed instruction, R - 1 adds in R / 2 instructions); the wave sum follows.  The
            // first level's sums are sums of TWO losses: one of them +Inf means an elementwise loss,
            // or the T sum of two, is +Inf, and the reference's sequential fold of all the losses
            // (each >= 0) is then +Inf too (it is at least the fold of those two).  Their max (one
            // VGPR) decides that below, only when the tile's sum overflowed.
#pragma unroll
            for (int r = 0; r < R / 2; ++r) l[r] += l[r + R / 2];
            T pair_max = l[0];
#pragma unroll
            for (int r = 1; r < R / 2; ++r) pair_max = pair_max > l[r] ? pair_max : l[r];
#pragma unroll
            for (int h = R / 4; h >= 1; h /= 2) {
#pragma unroll
              for (int r = 0; r < h; ++r) l[r] += l[r + h];
            }
            if (FAST_CHECK) {
              // the root is always checked, and already in the running max: every operator output and
              // constant root joins it, a feature root when the data needs it (track_x: otherwise
              // the data is finite and below tbig); a checked value was +-Inf -> incomplete; NaN
              // anywhere reaches the root (BASIC operators propagate NaN) and shows in the lane's
              // loss sum (padded rows replicate a real row: masking them hides no NaN), or, with
              // weights or a loss that can map NaN to a number (margin losses), in the root values;
              // a large finite one: the array-sum check may overflow
              mrun = SrMaxAbs<T>::step(mrun, mrun1, T(0));
              bool nan_root = false;
              if (weighted || !sr_loss_propagates_nan(lk)) {
#pragma unroll
                for (int r = 0; r < R; ++r) nan_root |= sr_isnan(tos[r]);
              } else {
                nan_root = sr_isnan(l[0]);
              }
              if (sr_ballot(nan_root || !(mrun <= SrM<T>::big))) {
                dead = true;
              } else if (sr_ballot(!(mrun < tbig))) {
                // (rare) a value >= tbig: DynamicExpressions' isfinite(sum(x)) of some checked array may
                // fail.  Every tracked array x has Σ_rows |x_i| <= Σ over tiles of R Σ_lanes mrun, and a
                // Julia-order sum of it stays below Σ|x_i| (1 + u)^1044 (leaf folds of < 1024, <= 20
                // pairwise levels); a tile within its share of floatmax — R Σ_lanes mrun <= 64 R x
                // floatmax / (1.01 x padded rows), i.e. Σ_lanes mrun <= big_budget — cannot make any
                // sum reach it, so only a tile past its share sends the tree to the exact pass (round 5:
                // C2's typical BIG tree, one huge row per tile, no longer pays that pass).  Untracked
                // feature rows are < tbig, their sums < floatmax / 2 on their own.
                const double msum = sr_wave_sum<double>(double(mrun));
                if (!(msum <= a.big_budget)) susp_any = true;
              }
            }
            if (!dead) {
              const T s = sr_wave_sum<T>(l[0]);
              accv += (lane == j) ? double(s) : 0.0;
              if (susp_any) bmask |= bit;
              // The tile's T sum of the losses is +Inf (rare; s is wave-uniform): SR_FLAG_ELEMINF when
              // a loss or a pair sum is +Inf (the reference's fold is then +Inf); otherwise only the
              // longer sums overflowed and the host decides the fold (sr_fold.h)
              if (!(s <= SrM<T>::big) && sr_ballot(pair_max == T(INFINITY))) emask |= bit;
            }
          }
          if (dead) {
            dmask |= bit;
            if (use_hint && lane == 0)
              __hip_atomic_fetch_max(a.hint + tree0 + g, a.hint_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        } else if (MODE == SR_MODE_FOLD) {
          // the same losses as the LOSS epilogue (rows past the view: 0, which the fold skips)
          T l[R];
          T yv[R];
          L::load(y_lane, yv);
          if (weighted) {
            T wv[R];
            L::load(w_lane, wv);
#pragma unroll
            for (int r = 0; r < R; ++r) l[r] = sr_elem_loss<T>(lk, tos[r], yv[r], a.loss_param) * wv[r];
          } else {
#pragma unroll
            for (int r = 0; r < R; ++r) l[r] = sr_elem_loss<T>(lk, tos[r], yv[r], a.loss_param);
          }
          if (!full_tile) {
#pragma unroll
            for (int r = 0; r < R; ++r) l[r] = (row0 + L::row(lane, r) < a.n_rows) ? l[r] : T(0);
          }
          using I = typename SrFoldTab<T>::I;
          // this tile's composed step under binade q, then the block's so far (lane j's pair)
          auto accumulate = [&](int q, I& acc0, I& acc1) {
            I y0, y1;
            sr_fold_tile_step<T, R, C>(l, q, lane, y0, y1);
            I x0 = I(0), x1 = I(0);
            if constexpr (sizeof(I) == 4) {
              x0 = __builtin_amdgcn_readlane(int(acc0), j);
              x1 = __builtin_amdgcn_readlane(int(acc1), j);
            } else {
              x0 = __shfl(acc0, j, 64);
              x1 = __shfl(acc1, j, 64);
            }
            sr_fold_compose_i<I>(x0, x1, y0, y1, I(1) << (SrFoldTraits<T>::mant + 3));
            if (lane == j) {
              acc0 = y0;
              acc1 = y1;
            }
          };
          const int32_t code = __builtin_amdgcn_readlane(my_code, j);
          if (code >= SR_FCODE_SLOT0) {  // a slow segment: keep its losses for the walk (row order)
            L::store(a.fold_loss + size_t(code - SR_FCODE_SLOT0) * size_t(a.fold_slot_rows) + size_t(tile) * ROWS +
                         lane * C,
                     l);
            const int32_t sq = __builtin_amdgcn_readlane(my_sq, j);
            if (sq != SR_FCODE_SKIP) {
              accumulate(sq, facc0, facc1);
              accumulate(sq + 1, facc2, facc3);
            }
          } else {
            accumulate(code, facc0, facc1);
          }
        } else if (MODE == SR_MODE_PRED) {
          const uint32_t tree = a.perm ? a.perm[tree0 + g] : uint32_t(tree0 + g);
          T* out = a.pred + int64_t(tree) * a.pred_ld + row0;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int i = L::row(lane, r);
            if (row0 + i < a.n_rows) out[i] = dead ? sr_qnan<T>() : tos[r];
          }
          if (dead) dmask |= bit;
          else if (susp_any) bmask |= bit;
        }
      }
    }
    if (tile == 0) SR_STAMP(4);
  }
  SR_STAMP(5);

  if (MODE == SR_MODE_FOLD) {  // the steps segments' pairs, [row block][position] (and the slow ones')
    const size_t o = size_t(rb) * size_t(a.n_trees) + size_t(my_pos);
    if (lane < S && my_code != SR_FCODE_SKIP && my_code < SR_FCODE_SLOT0)
      static_cast<typename SrFoldTab<T>::Pair*>(a.fold_tab)[o] = SrFoldTab<T>::pair(facc0, facc1);
    if (lane < S && my_sq != SR_FCODE_SKIP) {
      static_cast<typename SrFoldTab<T>::Pair*>(a.fold_tab)[o] = SrFoldTab<T>::pair(facc0, facc1);
      static_cast<typename SrFoldTab<T>::Pair*>(a.fold_tab2)[o] = SrFoldTab<T>::pair(facc2, facc3);
    }
    return;
  }
  if (MODE == SR_MODE_EXACT) {
    __syncthreads();
    // this range's sum of every checked array: [list position][check][range]
    T* out = static_cast<T*>(a.range_sums);
    for (int i = tid; i < gcount * MC; i += SR_BLOCK) out[(size_t(tree0) * MC + i) * size_t(a.n_row_blocks) + rb] = jst[i];
    return;
  }
  if (lane < S) {
    uint32_t f = (((dmask >> lane) & 1u) ? SR_FLAG_NONFINITE : 0u) | (((bmask >> lane) & 1u) ? SR_FLAG_BIG : 0u) |
                 (((emask >> lane) & 1u) ? SR_FLAG_ELEMINF : 0u);
    if (MODE == SR_MODE_LOSS && a.out_sum) {  // one row block: final per-tree values, tree order
      const uint32_t tree = a.perm ? a.perm[my_pos] : uint32_t(my_pos);
      if (a.static_bad[tree]) f |= SR_FLAG_STATIC | SR_FLAG_NONFINITE;
      a.out_sum[tree] = accv;
      a.out_flag[tree] = f;
    } else if (MODE == SR_MODE_LOSS && a.group_cnt) {  // write-through (sc1): read by another workgroup
      const size_t o = size_t(rb) * a.n_trees + my_pos;
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.part_sum + o),
                         static_cast<unsigned long long>(__double_as_longlong(accv)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.part_flag + o, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const size_t o = size_t(rb) * a.n_trees + my_pos;  // [row block][position]: a block writes one run
      a.part_sum[o] = accv;
      a.part_flag[o] = f;
    }
  }
  if (MODE == SR_MODE_LOSS && a.group_cnt && a.out_sum == nullptr) {
    // In-launch reduction (the hand-off of MI355X_MICROARCH.md's visibility table, first row): every
    // wave drains its sc1 stores, the workgroup barrier orders them before ONE agent-scope add per
    // workgroup on the group's counter; the block whose add comes last reduces the group (sc1 loads)
    // and resets the counter.  Each wave reduces its own positions, K at a time.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last_word = reinterpret_cast<int*>(sr_smem + plan.x);  // (the tiles are done with the LDS)
    if (tid == 0) {
      const uint32_t prev = __hip_atomic_fetch_add(a.group_cnt + tree0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = prev == uint32_t(a.n_row_blocks - 1);
      if (last) __hip_atomic_store(a.group_cnt + tree0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_word = last ? 1 : 0;
    }
    __syncthreads();
    if (*last_word)
      sr_reduce_positions<8, true>(a.part_sum, a.part_flag, a.n_trees, a.n_row_blocks, tree0 + wave, SR_WAVES, S,
                                   a.perm, a.static_bad, a.fused_sum, a.fused_flag, lane);
  }
  SR_STAMP(6);
}

// ------------------------------------------------------------------ launch helpers
template <typename T, int R, int MODE, bool GATHER, int TIER, int W, int LK, bool VSTK>
hipError_t sr_launch_tile(const SrEvalArgs<T>& a, int n_blocks, hipStream_t s) {
  if (VSTK && a.stack_depth > SR_VSTK_SLOTS) return hipErrorInvalidValue;  // host routes deeper programs elsewhere
  const SrLdsPlan<T> plan(a.nf, 64 * R, VSTK ? 0 : a.stack_depth, a.trees_per_block,
                          MODE == SR_MODE_EXACT ? a.max_checks : 0, W, a.w != nullptr,
                          (MODE == SR_MODE_LOSS || MODE == SR_MODE_FOLD) ? a.code_lds : 0);
  const void* fn = reinterpret_cast<const void*>(&sr_tile_kernel<T, R, MODE, GATHER, TIER, W, LK, VSTK>);
  if (plan.total > 65536) {  // many features / a deep stack: opt in to the full 160 KiB of LDS
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(plan.total));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((sr_tile_kernel<T, R, MODE, GATHER, TIER, W, LK, VSTK>), dim3(n_blocks), dim3(W * 64), plan.total, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------ derived columns
// Column k = op_k(X[f_k]) over rows [0, n_pad) of the view (gathered rows through row_idx; rows past
// the view replicate its first row, as the tile staging does), computed with the interpreter's own
// unary bodies, so a LOAD_DERIVED reads exactly the values UNARY0 + op_k would produce in place.
template <typename T, int R>
__global__ void __launch_bounds__(256) sr_derived_kernel(const T* __restrict__ X, int64_t ld, const int64_t* row_idx,
                                                         int64_t n_view, int64_t n_pad, SrDerivedSpec spec,
                                                         T* __restrict__ out, int64_t dld) {
  sr_libm_lds_fill(int(threadIdx.x), 256);
  __syncthreads();
  const int k = int(blockIdx.y);
  const int64_t v0 = (int64_t(blockIdx.x) * 256 + threadIdx.x) * R;
  if (v0 >= n_pad) return;
  const T* xf = X + int64_t(spec.feat[k]) * ld;
  T v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t q = v0 + r;
    v[r] = xf[row_idx ? row_idx[q < n_view ? q : 0] : q];
  }
  switch (spec.op[k]) {
    case SR_U_EXP: sr_unary_rows<T, SR_U_EXP, R>(v); break;
    case SR_U_COS: sr_unary_rows<T, SR_U_COS, R>(v); break;
    case SR_U_SIN: sr_unary_rows<T, SR_U_SIN, R>(v); break;
    case SR_U_LOG: sr_unary_rows<T, SR_U_LOG, R>(v); break;
    case SR_U_SQRT: sr_unary_rows<T, SR_U_SQRT, R>(v); break;
    default: break;
  }
  T* o = out + size_t(k) * size_t(dld) + size_t(v0);
#pragma unroll
  for (int r = 0; r < R; ++r) o[r] = v[r];
}

template <typename T>
hipError_t sr_launch_derived(const T* X, int64_t ld, const int64_t* row_idx, int64_t n_view, int64_t n_pad,
                             const SrDerivedSpec& spec, T* out, int64_t dld, hipStream_t s) {
  constexpr int R = 8;
  if (spec.n <= 0) return hipSuccess;
  const int64_t per_block = 256 * R;
  const dim3 grid(unsigned((n_pad + per_block - 1) / per_block), unsigned(spec.n));
  hipLaunchKernelGGL((sr_derived_kernel<T, R>), grid, dim3(256), 0, s, X, ld, row_idx, n_view, n_pad, spec, out, dld);
  return hipGetLastError();
}
#define SR_INSTANTIATE_DERIVED(T)                                                                            \
  template hipError_t sr_launch_derived<T>(const T*, int64_t, const int64_t*, int64_t, int64_t, const SrDerivedSpec&, \
                                           T*, int64_t, hipStream_t);

// Explicit instantiations are spread over several translation units (sr_inst_*.hip, one per
// element type / mode) so the build compiles them in parallel; see the Makefile.
#define SR_INSTANTIATE_WLV(T, R, MODE, GATHER, TIER, W, LK, VSTK) \
  template hipError_t sr_launch_tile<T, R, MODE, GATHER, TIER, W, LK, VSTK>(const SrEvalArgs<T>&, int, hipStream_t);
#define SR_INSTANTIATE_WL(T, R, MODE, GATHER, TIER, W, LK) SR_INSTANTIATE_WLV(T, R, MODE, GATHER, TIER, W, LK, false)
#define SR_INSTANTIATE_W(T, R, MODE, GATHER, TIER, W) SR_INSTANTIATE_WL(T, R, MODE, GATHER, TIER, W, -1)
#define SR_INSTANTIATE(T, R, MODE, GATHER, TIER) SR_INSTANTIATE_WL(T, R, MODE, GATHER, TIER, 4, -1)
// BASIC-tier loss kernels: one instantiation per elementwise loss
#define SR_INSTANTIATE_LOSS(T, R, GATHER)                                   \
  SR_INSTANTIATE_WL(T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, SR_LOSS_L2) \
  SR_INSTANTIATE_WL(T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, SR_LOSS_L1) \
  SR_INSTANTIATE_WL(T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, -1)
// register-stack BASIC-tier loss kernels (f32, 16 / 32 rows per lane)
#define SR_INSTANTIATE_LOSS_VSTK(T, R, GATHER)                                     \
  SR_INSTANTIATE_WLV(T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, SR_LOSS_L2, true) \
  SR_INSTANTIATE_WLV(T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, SR_LOSS_L1, true) \
  SR_INSTANTIATE_WLV(T, R, SR_MODE_LOSS, GATHER, SR_TIER_BASIC, 4, -1, true)
