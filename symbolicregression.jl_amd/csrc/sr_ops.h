// sr_ops.h — operator catalog for the MI355X evaluator (host + device).
//
// Every operator the device interpreter understands, with the exact semantics the
// reference attaches to it:
//   * arithmetic `+ - * /` are plain IEEE ops (Options.jl OP_MAP keeps `/` as IEEE `/`,
//     src/Options.jl:182-202);
//   * the "safe" operators return NaN outside their domain (src/Operators.jl:35-76);
//   * `square/cube/neg/relu/greater/less/cond/logical_*` follow src/Operators.jl:81-124,
//     including Julia's Bool*Float "strong zero" (`false * x == copysign(0, x)`);
//   * `max/min/mod/sign/round` follow Julia Base float semantics.
// The same functions are used by the host-side program compiler for constant folding
// (DynamicExpressions' constant-subtree fast path) and by the HIP kernel.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SR_HD __host__ __device__
#else
#define SR_HD
#endif

#include "sr_libm.h"

// ---------------------------------------------------------------------------------------
// Operator ids (semantic; independent of the position inside options.operators).
// ---------------------------------------------------------------------------------------
enum SrUnaryOp : uint32_t {
  SR_U_NONE = 0,
  SR_U_NEG, SR_U_SQUARE, SR_U_CUBE, SR_U_EXP, SR_U_COS, SR_U_SIN, SR_U_TAN,
  SR_U_LOG, SR_U_LOG2, SR_U_LOG10, SR_U_LOG1P, SR_U_SQRT, SR_U_ABS, SR_U_SIGN,
  SR_U_TANH, SR_U_SINH, SR_U_COSH, SR_U_ATAN, SR_U_ASIN, SR_U_ACOS, SR_U_ACOSH,
  SR_U_ATANH, SR_U_ASINH, SR_U_RELU, SR_U_INV, SR_U_ERF, SR_U_ERFC, SR_U_GAMMA,
  SR_U_ROUND, SR_U_FLOOR, SR_U_CEIL, SR_U_EXP2, SR_U_EXPM1,
  SR_U_COUNT
};

enum SrBinaryOp : uint32_t {
  SR_B_NONE = 0,
  SR_B_ADD, SR_B_SUB, SR_B_MUL, SR_B_DIV, SR_B_POW, SR_B_MAX, SR_B_MIN, SR_B_MOD,
  SR_B_GREATER, SR_B_LESS, SR_B_GREATER_EQUAL, SR_B_LESS_EQUAL, SR_B_COND,
  SR_B_LOGICAL_OR, SR_B_LOGICAL_AND, SR_B_ATAN2,
  SR_B_COUNT
};

// Elementwise losses: the SupervisedLoss catalog src/Options.jl:301-328 lists (LossFunctions.jl 0.11,
// not vendored: the published definitions are restated in sr_elem_loss below; d = output - target,
// a = target * output).  Parametric ones take one parameter (P, d, eps, circ, tau, gamma, q).
enum SrLossKind : int32_t {
  SR_LOSS_L2 = 0,              // L2DistLoss: abs2(d)   (default, src/Options.jl:772)
  SR_LOSS_L1 = 1,              // L1DistLoss: abs(d)
  SR_LOSS_LP = 2,              // LPDistLoss{P}: abs(d)^P
  SR_LOSS_LOGIT = 3,           // LogitDistLoss: -log(4) - d + 2 log(1 + exp(d))
  SR_LOSS_HUBER = 4,           // HuberLoss(delta): abs(d) <= delta ? d^2/2 : delta (abs(d) - delta/2)
  SR_LOSS_L1_EPS_INS = 5,      // L1EpsilonInsLoss(eps): max(0, abs(d) - eps)
  SR_LOSS_L2_EPS_INS = 6,      // L2EpsilonInsLoss(eps): max(0, abs(d) - eps)^2
  SR_LOSS_PERIODIC = 7,        // PeriodicLoss(circ): 1 - cos(d * 2pi/circ)
  SR_LOSS_QUANTILE = 8,        // QuantileLoss(tau): d * ((d > 0) - tau)
  SR_LOSS_ZERO_ONE = 9,        // ZeroOneLoss: sign(a) < 0 ? 1 : 0
  SR_LOSS_PERCEPTRON = 10,     // PerceptronLoss: max(0, -a)
  SR_LOSS_L1_HINGE = 11,       // L1HingeLoss: max(0, 1 - a)
  SR_LOSS_L2_HINGE = 12,       // L2HingeLoss: max(0, 1 - a)^2
  SR_LOSS_SMOOTH_L1_HINGE = 13,  // SmoothedL1HingeLoss(gamma): a >= 1 - gamma ? max(0, 1-a)^2/(2 gamma) : 1 - gamma/2 - a
  SR_LOSS_MODIFIED_HUBER = 14,   // ModifiedHuberLoss: a >= -1 ? max(0, 1 - a)^2 : -4a
  SR_LOSS_L2_MARGIN = 15,      // L2MarginLoss: (1 - a)^2
  SR_LOSS_EXP = 16,            // ExpLoss: exp(-a)
  SR_LOSS_SIGMOID = 17,        // SigmoidLoss: 1 - tanh(a)
  SR_LOSS_DWD_MARGIN = 18,     // DWDMarginLoss(q): a <= q/(q+1) ? 1 - a : (q^q/(q+1)^(q+1)) / a^q
  SR_LOSS_COUNT
};
// Losses whose value is NaN whenever the prediction is (the deferred NaN test may read the loss sum)
SR_HD inline bool sr_loss_propagates_nan(int32_t kind) {
  return kind == SR_LOSS_L2 || kind == SR_LOSS_L1 || kind == SR_LOSS_LP || kind == SR_LOSS_LOGIT ||
         kind == SR_LOSS_HUBER || kind == SR_LOSS_L2_MARGIN || kind == SR_LOSS_EXP || kind == SR_LOSS_SIGMOID;
}

// ---------------------------------------------------------------------------------------
// Program instruction: one per evaluated node (a leaf that is a binary node's operand is folded into
// that node's instruction), 16 bytes for f32 and f64 alike.  The interpreter dispatches on `op`
// as read (no decoding): every variant is its own opcode.
//   op   : opcode
//       SR_OP_LOAD_FEAT  tos <- X[f]          SR_OP_LOAD_CONST  tos <- c
//       SR_OP_LOAD_FEAT_PUSH / _CONST_PUSH: the old tos is first stored to stack slot `push`
//       SR_OP_UNARY0 + u      tos <- op_u(tos)
//       SR_OP_UNARY_INF0 + u  tos <- isfinite(tos) ? op_u(tos) : +Inf — DynamicExpressions' fused
//                             unary kernels (deg1_l2_ll0_lr0 / deg1_l1_ll0)
//       SR_OP_BINARY0 + 6*(b-1) + variant              tos <- op_b(.,.) with operand variant:
//           SR_V_SL: op(S[k], tos)  SR_V_SR: op(tos, S[k])   (S[k] = stack slot k, popped)
//           SR_V_FL: op(X[f], tos)  SR_V_FR: op(tos, X[f])
//           SR_V_CL: op(c, tos)     SR_V_CR: op(tos, c)
//         + and * only ever use the R variants (the compiler canonicalises: IEEE + and * commute)
//       SR_OP_PAIR0 + 6*(b-1) + pair variant   tos <- op_b(leaf, leaf) (a binary node whose children
//           are both leaves — DE's deg2_l0_r0 — in one instruction):
//           SR_P_FF: op(X[f], X[g])  SR_P_FC: op(X[f], c)  SR_P_CF: op(c, X[f])   (f in meta, g in c0)
//           + SR_P_PUSH: the old tos is first stored to stack slot `push` (a subtree's first instruction)
//         + and * never use CF (commuted to FC)
//       SR_OP_LOAD_DERIVED (_PUSH)  tos <- D[k]: a derived column op_u(X[f]) computed once per call
//                             for the whole batch (LOSS programs of BASIC-tier kernels only: the
//                             node unary(feature), shared by many trees of a population)
//   c0 (, c1) : constant bits (C variants, LOAD_CONST*): f32 in c0, f64 in c0 | c1 << 32
//   (word order in memory: op, meta, c0, c1)
//   op bits  0-8    : the opcode (below 512)
//   op bits 16-21   : POST  unary operator applied to tos after the opcode (0 = none): a unary node
//                     fused into the instruction computing its child (one dispatch for both)
//   op bit  22      : POST_INF  the post unary is DynamicExpressions' fused form (non-finite -> +Inf)
//   op bit  23      : POST_CHECK  the post unary's output array is validity-checked
//   op bits 24-26   : PBC  a binary node with a constant operand fused into the instruction computing
//                     its other operand (round 5: one dispatch for both), applied after the POST unary:
//                     1 tos + c, 2 tos - c, 3 c - tos, 4 tos * c, 5 tos / c, 6 c / tos (c in c0 / c1:
//                     only instructions that use no constant carry it: LOAD_FEAT, unary, S / F binaries)
//   op bit  27      : PBC_CHECK  the post binary's output array is validity-checked
//   meta bits  0-15 : operand index: feature f (F variants, LOAD_FEAT*), stack slot k (S variants),
//                     pre-order constant slot of a constant leaf (gradient programs; else 0)
//   meta bits 24-29 : push slot + 1 (LOAD_*_PUSH)
//   meta bit  31    : CHECK   this node's output array is validity-checked (DE early exit)
//   (bits 16-23 stay 0, so `meta << s` with s >= 8 is the operand's byte offset for a row stride
//    of 2^s bytes: the flag bits shift out)
// ---------------------------------------------------------------------------------------
enum : uint32_t {
  SR_OP_LOAD_FEAT = 0u, SR_OP_LOAD_CONST = 1u, SR_OP_LOAD_FEAT_PUSH = 2u, SR_OP_LOAD_CONST_PUSH = 3u,
  SR_OP_UNARY0 = 4u,       // opcode = SR_OP_UNARY0 + SrUnaryOp (1..)
  SR_OP_UNARY_INF0 = 40u,  // opcode = SR_OP_UNARY_INF0 + SrUnaryOp (fused: non-finite input -> +Inf)
  SR_OP_BINARY0 = 80u,     // opcode = SR_OP_BINARY0 + 6*(SrBinaryOp-1) + variant
  SR_OP_LOAD_DERIVED = 78u, SR_OP_LOAD_DERIVED_PUSH = 79u,  // (between the unary-inf and binary ranges)
  SR_OP_PAIR0 = 256u,      // opcode = SR_OP_PAIR0 + 6*(SrBinaryOp-1) + pair variant
  SR_V_SL = 0u, SR_V_SR = 1u, SR_V_FL = 2u, SR_V_FR = 3u, SR_V_CL = 4u, SR_V_CR = 5u,
  SR_P_FF = 0u, SR_P_FC = 1u, SR_P_CF = 2u, SR_P_PUSH = 3u,
  SR_OP_MASK = 0x1ffu, SR_OP_POST_SHIFT = 16u, SR_OP_POST_INF = 1u << 22, SR_OP_POST_CHECK = 1u << 23,
  SR_OP_PBC_SHIFT = 24u, SR_OP_PBC_CHECK = 1u << 27,
  SR_PBC_ADD = 1u, SR_PBC_SUB_R = 2u, SR_PBC_SUB_L = 3u, SR_PBC_MUL = 4u, SR_PBC_DIV_R = 5u, SR_PBC_DIV_L = 6u,
  SR_M_INDEX = 0xffffu, SR_M_PUSH_SHIFT = 24u, SR_M_PUSH_MASK = 0x3fu << 24, SR_M_CHECK = 1u << 31,
  SR_MAX_STACK_SLOTS = 62u,
};
static_assert(SR_OP_UNARY0 + SR_U_COUNT <= SR_OP_UNARY_INF0, "unary opcode ranges overlap");
static_assert(SR_OP_UNARY_INF0 + SR_U_COUNT <= SR_OP_LOAD_DERIVED, "unary opcode range overlaps LOAD_DERIVED");
static_assert(SR_OP_LOAD_DERIVED_PUSH < SR_OP_BINARY0, "LOAD_DERIVED overlaps the binary range");
static_assert(SR_OP_BINARY0 + 6 * SR_B_COUNT <= SR_OP_PAIR0, "binary opcode range overlaps the pair range");
static_assert(SR_OP_PAIR0 + 6 * SR_B_COUNT <= SR_OP_MASK + 1, "opcodes must fit the op word's low 9 bits");
static_assert(SR_U_COUNT <= 64, "post-unary ids must fit 6 bits");
#define SR_BIN_OPC(b, v) (SR_OP_BINARY0 + 6u * ((b) - 1u) + (v))
#define SR_PAIR_OPC(b, v) (SR_OP_PAIR0 + 6u * ((b) - 1u) + (v))

template <typename T>
struct alignas(16) SrIns {
  uint32_t op;
  uint32_t meta;
  uint32_t c0, c1;  // (f32 programs use c0 only: the interpreter loads 12 of the 16 bytes)
  SR_HD inline uint32_t operand() const { return meta & SR_M_INDEX; }
  SR_HD inline int push_slot() const { return int((meta >> SR_M_PUSH_SHIFT) & 0x3fu) - 1; }
  SR_HD inline T value() const {
    if constexpr (sizeof(T) == 4) {
      return __builtin_bit_cast(T, c0);
    } else {
      return __builtin_bit_cast(T, uint64_t(c0) | (uint64_t(c1) << 32));
    }
  }
  SR_HD inline void set_value(T v) {
    if constexpr (sizeof(T) == 4) {
      c0 = __builtin_bit_cast(uint32_t, v);
      c1 = 0u;
    } else {
      const uint64_t b = __builtin_bit_cast(uint64_t, v);
      c0 = uint32_t(b);
      c1 = uint32_t(b >> 32);
    }
  }
};
static_assert(sizeof(SrIns<float>) == 16, "f32 instruction must be 16 bytes");
static_assert(sizeof(SrIns<double>) == 16, "f64 instruction must be 16 bytes");

// ---------------------------------------------------------------------------------------
// Type-dispatched libm (host: libm; device: ROCm OCML through the HIP math headers).
// ---------------------------------------------------------------------------------------
template <typename T> struct SrM;
template <> struct SrM<float> {
  // cos / sin / log: computed in double and rounded once (sr_libm.h); exp: OCML on the device
  // (0.675 ulp measured), the correctly rounded double version on the host (constant folding)
#if defined(__HIP_DEVICE_COMPILE__)
  static SR_HD inline float exp(float x) { return ::expf(x); }
#else
  static SR_HD inline float exp(float x) { return sr_expf(x); }
#endif
  static SR_HD inline float cos(float x) { return sr_cosf(x); }
  static SR_HD inline float sin(float x) { return sr_sinf(x); }
  static SR_HD inline float tan(float x) { return ::tanf(x); }
  static SR_HD inline float log(float x) { return sr_logf(x); }
  static SR_HD inline float log2(float x) { return ::log2f(x); }
  static SR_HD inline float log10(float x) { return ::log10f(x); }
  static SR_HD inline float log1p(float x) { return ::log1pf(x); }
  static SR_HD inline float sqrt(float x) { return ::sqrtf(x); }
  static SR_HD inline float tanh(float x) { return ::tanhf(x); }
  static SR_HD inline float sinh(float x) { return ::sinhf(x); }
  static SR_HD inline float cosh(float x) { return ::coshf(x); }
  static SR_HD inline float atan(float x) { return ::atanf(x); }
  static SR_HD inline float asin(float x) { return ::asinf(x); }
  static SR_HD inline float acos(float x) { return ::acosf(x); }
  static SR_HD inline float acosh(float x) { return ::acoshf(x); }
  static SR_HD inline float atanh(float x) { return ::atanhf(x); }
  static SR_HD inline float asinh(float x) { return ::asinhf(x); }
  static SR_HD inline float erf(float x) { return ::erff(x); }
  static SR_HD inline float erfc(float x) { return ::erfcf(x); }
  static SR_HD inline float tgamma(float x) { return ::tgammaf(x); }
  static SR_HD inline float rint(float x) { return ::rintf(x); }
  static SR_HD inline float floor(float x) { return ::floorf(x); }
  static SR_HD inline float ceil(float x) { return ::ceilf(x); }
  static SR_HD inline float exp2(float x) { return ::exp2f(x); }
  static SR_HD inline float expm1(float x) { return ::expm1f(x); }
  static SR_HD inline float pow(float x, float y) { return ::powf(x, y); }
  static SR_HD inline float fmod(float x, float y) { return ::fmodf(x, y); }
  static SR_HD inline float atan2(float y, float x) { return ::atan2f(y, x); }
  static SR_HD inline float trunc(float x) { return ::truncf(x); }
  static SR_HD inline float copysign(float x, float y) { return ::copysignf(x, y); }
  static SR_HD inline float fabs(float x) { return ::fabsf(x); }
  // Julia exp(::Float32) returns Inf above MAX_EXP = 88.72284f0 (base/special/exp.jl).
  static constexpr float max_exp = 88.72284f;
  static constexpr float big = 3.40282347e38f;
};
template <> struct SrM<double> {
  static SR_HD inline double exp(double x) { return ::exp(x); }
  static SR_HD inline double cos(double x) { return ::cos(x); }
  static SR_HD inline double sin(double x) { return ::sin(x); }
  static SR_HD inline double tan(double x) { return ::tan(x); }
  static SR_HD inline double log(double x) { return ::log(x); }
  static SR_HD inline double log2(double x) { return ::log2(x); }
  static SR_HD inline double log10(double x) { return ::log10(x); }
  static SR_HD inline double log1p(double x) { return ::log1p(x); }
  static SR_HD inline double sqrt(double x) { return ::sqrt(x); }
  static SR_HD inline double tanh(double x) { return ::tanh(x); }
  static SR_HD inline double sinh(double x) { return ::sinh(x); }
  static SR_HD inline double cosh(double x) { return ::cosh(x); }
  static SR_HD inline double atan(double x) { return ::atan(x); }
  static SR_HD inline double asin(double x) { return ::asin(x); }
  static SR_HD inline double acos(double x) { return ::acos(x); }
  static SR_HD inline double acosh(double x) { return ::acosh(x); }
  static SR_HD inline double atanh(double x) { return ::atanh(x); }
  static SR_HD inline double asinh(double x) { return ::asinh(x); }
  static SR_HD inline double erf(double x) { return ::erf(x); }
  static SR_HD inline double erfc(double x) { return ::erfc(x); }
  static SR_HD inline double tgamma(double x) { return ::tgamma(x); }
  static SR_HD inline double rint(double x) { return ::rint(x); }
  static SR_HD inline double floor(double x) { return ::floor(x); }
  static SR_HD inline double ceil(double x) { return ::ceil(x); }
  static SR_HD inline double exp2(double x) { return ::exp2(x); }
  static SR_HD inline double expm1(double x) { return ::expm1(x); }
  static SR_HD inline double pow(double x, double y) { return ::pow(x, y); }
  static SR_HD inline double fmod(double x, double y) { return ::fmod(x, y); }
  static SR_HD inline double atan2(double y, double x) { return ::atan2(y, x); }
  static SR_HD inline double trunc(double x) { return ::trunc(x); }
  static SR_HD inline double copysign(double x, double y) { return ::copysign(x, y); }
  static SR_HD inline double fabs(double x) { return ::fabs(x); }
  static constexpr double max_exp = 709.7827128933841;
  static constexpr double big = 1.7976931348623157e308;
};

template <typename T> SR_HD inline T sr_qnan() { return T(__builtin_nan("")); }
template <typename T> SR_HD inline T sr_inf() { return T(__builtin_inf()); }
template <typename T> SR_HD inline bool sr_isfinite(T x) { return __builtin_isfinite(x); }
template <typename T> SR_HD inline bool sr_isnan(T x) { return __builtin_isnan(x); }
// Julia Bool*Float: true*x == x, false*x == copysign(0, x)   (Base: bool.jl)
template <typename T> SR_HD inline T sr_bool_mul(bool b, T x) { return b ? x : SrM<T>::copysign(T(0), x); }

// ---------------------------------------------------------------------------------------
// Unary operators.
// ---------------------------------------------------------------------------------------
template <typename T>
SR_HD inline T sr_unary(uint32_t op, T x) {
  using M = SrM<T>;
  switch (op) {
    case SR_U_NEG: return -x;
    case SR_U_SQUARE: return x * x;                       // Operators.jl:81
    case SR_U_CUBE: return x * x * x;                     // Operators.jl:82
    case SR_U_EXP: return x > M::max_exp ? sr_inf<T>() : M::exp(x);
    case SR_U_COS: return M::cos(x);
    case SR_U_SIN: return M::sin(x);
    case SR_U_TAN: return M::tan(x);
    case SR_U_LOG: return x > T(0) ? M::log(x) : sr_qnan<T>();        // safe_log  :50-52
    case SR_U_LOG2: return x > T(0) ? M::log2(x) : sr_qnan<T>();      // safe_log2 :53-55
    case SR_U_LOG10: return x > T(0) ? M::log10(x) : sr_qnan<T>();    // safe_log10 :56-58
    case SR_U_LOG1P: return x > T(-1) ? M::log1p(x) : sr_qnan<T>();   // safe_log1p :59-61
    case SR_U_SQRT: return x >= T(0) ? M::sqrt(x) : sr_qnan<T>();     // safe_sqrt :74-76
    case SR_U_ABS: return x < T(0) ? -x : (x == T(0) ? T(0) : x);
    case SR_U_SIGN: return x < T(0) ? T(-1) : (x > T(0) ? T(1) : x);  // Julia sign (NaN -> NaN)
    case SR_U_TANH: return M::tanh(x);
    case SR_U_SINH: return M::sinh(x);
    case SR_U_COSH: return M::cosh(x);
    case SR_U_ATAN: return M::atan(x);
    case SR_U_ASIN: return (T(-1) <= x && x <= T(1)) ? M::asin(x) : sr_qnan<T>();   // :62-64
    case SR_U_ACOS: return (T(-1) <= x && x <= T(1)) ? M::acos(x) : sr_qnan<T>();   // :65-67
    case SR_U_ACOSH: return x >= T(1) ? M::acosh(x) : sr_qnan<T>();                 // :68-70
    case SR_U_ATANH: return (T(-1) <= x && x <= T(1)) ? M::atanh(x) : sr_qnan<T>(); // :71-73
    case SR_U_ASINH: return M::asinh(x);
    case SR_U_RELU: return sr_bool_mul<T>(x > T(0), x);                              // :115
    case SR_U_INV: return T(1) / x;
    case SR_U_ERF: return M::erf(x);
    case SR_U_ERFC: return M::erfc(x);
    case SR_U_GAMMA: { T g = M::tgamma(x); return __builtin_isinf(g) ? sr_qnan<T>() : g; } // :14-17
    case SR_U_ROUND: return M::rint(x);   // Julia round: RoundNearest (ties to even)
    case SR_U_FLOOR: return M::floor(x);
    case SR_U_CEIL: return M::ceil(x);
    case SR_U_EXP2: return M::exp2(x);
    case SR_U_EXPM1: return M::expm1(x);
    default: return sr_qnan<T>();
  }
}

// safe_pow (src/Operators.jl:35-49): NaN on the invalid branches, else x^y.
template <typename T>
SR_HD inline T sr_safe_pow(T x, T y) {
  const bool isint = (y - SrM<T>::trunc(y)) == T(0);   // Julia isinteger (false for Inf/NaN)
  if (isint) {
    if (y < T(0) && x == T(0)) return sr_qnan<T>();
  } else {
    if (y > T(0) && x < T(0)) return sr_qnan<T>();
    if (y < T(0) && x <= T(0)) return sr_qnan<T>();
  }
  return SrM<T>::pow(x, y);
}

// Julia Base.max / Base.min on floats: NaN-propagating, -0.0 < 0.0.
template <typename T>
SR_HD inline T sr_jl_max(T x, T y) {
  if (sr_isnan(x)) return x;
  if (sr_isnan(y)) return y;
  const bool sx = __builtin_signbit(x) != 0, sy = __builtin_signbit(y) != 0;
  return (y > x || (sx && !sy && x == y)) ? y : x;
}
template <typename T>
SR_HD inline T sr_jl_min(T x, T y) {
  if (sr_isnan(x)) return x;
  if (sr_isnan(y)) return y;
  const bool sx = __builtin_signbit(x) != 0, sy = __builtin_signbit(y) != 0;
  return (y < x || (sy && !sx && x == y)) ? y : x;
}
// Julia Base.mod on floats: r = rem(x, y); r == 0 -> copysign(r, y); sign mismatch -> r + y.
template <typename T>
SR_HD inline T sr_jl_mod(T x, T y) {
  const T r = SrM<T>::fmod(x, y);
  if (r == T(0)) return SrM<T>::copysign(r, y);
  if ((r > T(0)) != (y > T(0))) return r + y;
  return r;
}

template <typename T>
SR_HD inline T sr_binary(uint32_t op, T x, T y) {
  switch (op) {
    case SR_B_ADD: return x + y;
    case SR_B_SUB: return x - y;
    case SR_B_MUL: return x * y;
    case SR_B_DIV: return x / y;
    case SR_B_POW: return sr_safe_pow<T>(x, y);
    case SR_B_MAX: return sr_jl_max<T>(x, y);
    case SR_B_MIN: return sr_jl_min<T>(x, y);
    case SR_B_MOD: return sr_jl_mod<T>(x, y);
    case SR_B_GREATER: return (x > y) ? T(1) : T(0);          // Operators.jl:98-100
    case SR_B_LESS: return (x < y) ? T(1) : T(0);             // :101-103
    case SR_B_GREATER_EQUAL: return (x >= y) ? T(1) : T(0);   // :104-106
    case SR_B_LESS_EQUAL: return (x <= y) ? T(1) : T(0);      // :107-109
    case SR_B_COND: return sr_bool_mul<T>(x > T(0), y);       // :110-112
    case SR_B_LOGICAL_OR: return ((x > T(0)) || (y > T(0))) ? T(1) : T(0);   // :118-120
    case SR_B_LOGICAL_AND: return ((x > T(0)) && (y > T(0))) ? T(1) : T(0);  // :121-123
    case SR_B_ATAN2: return SrM<T>::atan2(x, y);              // Julia atan(y, x) with (x=y_arg)
    default: return sr_qnan<T>();
  }
}

// ---------------------------------------------------------------------------------------
// Derivatives for the forward-mode constant gradient (ConstantOptimization.jl with a forward-mode
// autodiff backend).  Only evaluated on complete trees, i.e. on the valid branch of every safe
// operator.  sr_grad_supported() says whether an operator has a rule here.
// ---------------------------------------------------------------------------------------
inline bool sr_unary_grad_supported(uint32_t op) { return op != SR_U_GAMMA && op != SR_U_NONE && op < SR_U_COUNT; }
inline bool sr_binary_grad_supported(uint32_t op) { return op != SR_B_NONE && op < SR_B_COUNT; }

// d op(x) / dx, given y = op(x)
template <typename T>
SR_HD inline T sr_unary_deriv(uint32_t op, T x, T y) {
  using M = SrM<T>;
  switch (op) {
    case SR_U_NEG: return T(-1);
    case SR_U_SQUARE: return T(2) * x;
    case SR_U_CUBE: return T(3) * x * x;
    case SR_U_EXP: return y;
    case SR_U_COS: return -M::sin(x);
    case SR_U_SIN: return M::cos(x);
    case SR_U_TAN: return T(1) + y * y;
    case SR_U_LOG: return T(1) / x;
    case SR_U_LOG2: return T(1) / (x * T(0.6931471805599453));
    case SR_U_LOG10: return T(1) / (x * T(2.302585092994046));
    case SR_U_LOG1P: return T(1) / (T(1) + x);
    case SR_U_SQRT: return T(0.5) / y;
    case SR_U_ABS: return __builtin_signbit(x) ? T(-1) : T(1);  // Julia abs(::Dual)
    case SR_U_SIGN: return T(0);
    case SR_U_TANH: return T(1) - y * y;
    case SR_U_SINH: return M::cosh(x);
    case SR_U_COSH: return M::sinh(x);
    case SR_U_ATAN: return T(1) / (T(1) + x * x);
    case SR_U_ASIN: return T(1) / M::sqrt(T(1) - x * x);
    case SR_U_ACOS: return T(-1) / M::sqrt(T(1) - x * x);
    case SR_U_ACOSH: return T(1) / M::sqrt(x * x - T(1));
    case SR_U_ATANH: return T(1) / (T(1) - x * x);
    case SR_U_ASINH: return T(1) / M::sqrt(T(1) + x * x);
    case SR_U_RELU: return x > T(0) ? T(1) : T(0);
    case SR_U_INV: return -(y * y);
    case SR_U_ERF: return T(1.1283791670955126) * M::exp(-(x * x));
    case SR_U_ERFC: return T(-1.1283791670955126) * M::exp(-(x * x));
    case SR_U_ROUND: case SR_U_FLOOR: case SR_U_CEIL: return T(0);
    case SR_U_EXP2: return T(0.6931471805599453) * y;
    case SR_U_EXPM1: return y + T(1);
    default: return sr_qnan<T>();
  }
}

// partial derivatives (d/da, d/db) of r = op(a, b)
template <typename T>
SR_HD inline void sr_binary_partials(uint32_t op, T a, T b, T r, T* pa, T* pb) {
  using M = SrM<T>;
  switch (op) {
    case SR_B_ADD: *pa = T(1); *pb = T(1); return;
    case SR_B_SUB: *pa = T(1); *pb = T(-1); return;
    case SR_B_MUL: *pa = b; *pb = a; return;
    case SR_B_DIV: *pa = T(1) / b; *pb = -r / b; return;
    case SR_B_POW:
      *pa = (a == T(0)) ? b * M::pow(a, b - T(1)) : b * r / a;
      *pb = a > T(0) ? r * M::log(a) : T(0);
      return;
    case SR_B_MAX: { const bool ta = !(b > a); *pa = ta ? T(1) : T(0); *pb = ta ? T(0) : T(1); return; }  // ties: first
    case SR_B_MIN: { const bool ta = !(b < a); *pa = ta ? T(1) : T(0); *pb = ta ? T(0) : T(1); return; }
    case SR_B_MOD: *pa = T(1); *pb = -M::floor(a / b); return;
    case SR_B_COND: *pa = T(0); *pb = a > T(0) ? T(1) : T(0); return;
    case SR_B_ATAN2: { const T d = a * a + b * b; *pa = b / d; *pb = -a / d; return; }
    default: *pa = T(0); *pb = T(0); return;  // comparisons / logical: piecewise constant
  }
}

// Julia's max(0, x): NaN propagates.
template <typename T>
SR_HD inline T sr_pos(T x) {
  return (x != x) ? x : (x > T(0) ? x : T(0));
}

// Elementwise loss value (LossFunctions.jl restated; `p` = the loss's parameter).
template <typename T>
SR_HD inline T sr_elem_loss(int32_t kind, T pred, T target, T p = T(0)) {
  using M = SrM<T>;
  const T d = pred - target;
  const T ad = d < T(0) ? -d : d;
  const T a = target * pred;
  switch (kind) {
    case SR_LOSS_L1: return ad;
    case SR_LOSS_LP: return M::pow(ad, p);
    case SR_LOSS_LOGIT: return -M::log(T(4)) - d + T(2) * M::log(T(1) + M::exp(d));
    case SR_LOSS_HUBER: return ad <= p ? d * d / T(2) : p * (ad - p / T(2));
    case SR_LOSS_L1_EPS_INS: return sr_pos<T>(ad - p);
    case SR_LOSS_L2_EPS_INS: { const T e = sr_pos<T>(ad - p); return e * e; }
    case SR_LOSS_PERIODIC: return T(1) - M::cos(d * (T(2) * T(3.14159265358979323846) / p));
    case SR_LOSS_QUANTILE: return d * ((d > T(0) ? T(1) : T(0)) - p);
    case SR_LOSS_ZERO_ONE: return (a < T(0)) ? T(1) : T(0);
    case SR_LOSS_PERCEPTRON: return sr_pos<T>(-a);
    case SR_LOSS_L1_HINGE: return sr_pos<T>(T(1) - a);
    case SR_LOSS_L2_HINGE: { const T e = sr_pos<T>(T(1) - a); return e * e; }
    case SR_LOSS_SMOOTH_L1_HINGE: {
      if (a >= T(1) - p) { const T e = sr_pos<T>(T(1) - a); return e * e / (T(2) * p); }
      return T(1) - p / T(2) - a;
    }
    case SR_LOSS_MODIFIED_HUBER: {
      if (a >= T(-1)) { const T e = sr_pos<T>(T(1) - a); return e * e; }
      return T(-4) * a;
    }
    case SR_LOSS_L2_MARGIN: { const T e = T(1) - a; return e * e; }
    case SR_LOSS_EXP: return M::exp(-a);
    case SR_LOSS_SIGMOID: return T(1) - M::tanh(a);
    case SR_LOSS_DWD_MARGIN: {
      if (a <= p / (p + T(1))) return T(1) - a;
      return (M::pow(p, p) / M::pow(p + T(1), p + T(1))) / M::pow(a, p);
    }
    default: return d * d;  // SR_LOSS_L2
  }
}
// d loss / d pred (a = target * pred: d/dpred = target * dL/da); kinks take the one-sided value
// LossFunctions' `deriv` takes there
template <typename T>
SR_HD inline T sr_elem_loss_deriv(int32_t kind, T pred, T target, T p = T(0)) {
  using M = SrM<T>;
  const T d = pred - target;
  const T ad = d < T(0) ? -d : d;
  const T sd = d > T(0) ? T(1) : (d < T(0) ? T(-1) : T(0));
  const T a = target * pred;
  switch (kind) {
    case SR_LOSS_L1: return sd;
    case SR_LOSS_LP: return ad == T(0) ? T(0) : p * M::pow(ad, p - T(1)) * sd;
    case SR_LOSS_LOGIT: return M::tanh(d / T(2));
    case SR_LOSS_HUBER: return ad <= p ? d : p * sd;
    case SR_LOSS_L1_EPS_INS: return ad > p ? sd : T(0);
    case SR_LOSS_L2_EPS_INS: return ad > p ? T(2) * (ad - p) * sd : T(0);
    case SR_LOSS_PERIODIC: { const T k = T(2) * T(3.14159265358979323846) / p; return k * M::sin(d * k); }
    case SR_LOSS_QUANTILE: return (d > T(0) ? T(1) : T(0)) - p;
    case SR_LOSS_ZERO_ONE: return T(0);
    case SR_LOSS_PERCEPTRON: return a < T(0) ? -target : T(0);
    case SR_LOSS_L1_HINGE: return a < T(1) ? -target : T(0);
    case SR_LOSS_L2_HINGE: return a < T(1) ? T(-2) * (T(1) - a) * target : T(0);
    case SR_LOSS_SMOOTH_L1_HINGE:
      if (a >= T(1) - p) return a < T(1) ? -(T(1) - a) / p * target : T(0);
      return -target;
    case SR_LOSS_MODIFIED_HUBER:
      if (a >= T(-1)) return a < T(1) ? T(-2) * (T(1) - a) * target : T(0);
      return T(-4) * target;
    case SR_LOSS_L2_MARGIN: return T(-2) * (T(1) - a) * target;
    case SR_LOSS_EXP: return -M::exp(-a) * target;
    case SR_LOSS_SIGMOID: { const T t = M::tanh(a); return -(T(1) - t * t) * target; }
    case SR_LOSS_DWD_MARGIN:
      if (a <= p / (p + T(1))) return -target;
      return -(M::pow(p, p + T(1)) / M::pow(p + T(1), p + T(1))) / M::pow(a, p + T(1)) * target;
    default: return T(2) * d;  // SR_LOSS_L2
  }
}
