// sr_libm.h — Float32 exp / log / cos / sin for the evaluator (host + device).
//
// The reference evaluates these with Julia's Base.Math, accurate to < 1 ulp (its Float32 trig and
// log kernels work in Float64).  ROCm's OCML Float32 log / cos / sin measured 1.75 / 1.26 / 1.49 ulp
// on the fixture points of tests/golden/libm_ulp.json (profiles/r02_libm_ocml.txt), so those three
// are computed here in double and rounded once, table-driven so the work per value stays close to
// OCML's: log from a 64-cell table of an offset octave and a degree-4 log1p (within 2^-30 relative
// before the final rounding: <= 0.5101 ulp), cos / sin from (sin, cos)(k pi/128) and degree-4 Taylor terms on |r| <= pi/256 (<= 0.5025
// ulp over every Float32 |x| < 2^20, checked
// exhaustively by tools/libm_exhaustive.cpp; profiles/r03_libm_exhaustive.txt).  OCML's Float32 exp
// measured 0.675 ulp and is kept on the device (sr_expf below, also correctly rounded but for
// 2^-46-close midpoints, serves the host's constant folding).
//
// The device reads the tables from a per-workgroup LDS copy (sr_libm_lds_fill, every kernel that
// evaluates operators runs it before its first barrier); the host reads them from constant memory.
// Host and device run the same double arithmetic (fused multiply-adds, no contraction).
#pragma once
#include <math.h>
#include <stdint.h>

#include "sr_libm_tables.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SRL_HD __host__ __device__
#else
#define SRL_HD
#endif

namespace srl {

// fits (tools/gen_libm_coeffs.py), highest degree first
// exp(r), |r| <= ln2/2: degree 9, fit error 1.4e-14 (2^-46)
constexpr double kExp[10] = {0x1.72e107c874de9p-19, 0x1.a17df0d914d6cp-16, 0x1.a01994c849582p-13,
                             0x1.6c162bb7d965cp-10, 0x1.11111123bf154p-7,  0x1.55555588b8403p-5,
                             0x1.5555555550d88p-3,  0x1.ffffffffe74f1p-2,  0x1.0000000000006p+0,
                             0x1.000000000003dp+0};
// sin(y) = y + y^3 S(y^2), y^2 <= (pi/4)^2: degree 4, error 2.8e-14 * y^3
constexpr double kSin[5] = {-0x1.aa285788aaa42p-26, 0x1.71d9a9f41c5a9p-19, -0x1.a019fd9b35ee5p-13,
                            0x1.1111110fd3d43p-7, -0x1.555555555516bp-3};
// cos(y) = 1 - y^2/2 + y^4 C(y^2): degree 4, error 2.0e-15 * y^4
constexpr double kCos[5] = {0x1.1c81c3531fff2p-29, -0x1.27e25f4bb4e6fp-22, 0x1.a019ff53a6a1cp-16,
                            -0x1.6c16c16b614fcp-10, 0x1.5555555555437p-5};
// log1p(f) = f - f^2/2 + f^3 L(f), f in [sqrt(1/2) - 1, sqrt(2) - 1]: degree 14, error 5.0e-13 * |f|^3
constexpr double kLog[15] = {0x1.34a3062fa13dap-5,  -0x1.306de714fa1b3p-4, 0x1.37899b8c443dap-4,
                             -0x1.23f5f5fbd8892p-4, 0x1.36199280460d9p-4,  -0x1.54e02c02891e6p-4,
                             0x1.74aa7980a0ff2p-4,  -0x1.99a399e5da0a2p-4, 0x1.c71a0ec530d0fp-4,
                             -0x1.ffffadf31c080p-4, 0x1.24924daef848dp-3,  -0x1.555555d97f9a5p-3,
                             0x1.99999992e84ecp-3,  -0x1.ffffffff8bc75p-3, 0x1.55555555562e9p-2};
constexpr double kLog2e = 0x1.71547652b82fep+0;
constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
constexpr double kTwoOverPi = 0x1.45f306dc9c883p-1;
constexpr double kPio2_1 = 0x1.921fb54442d18p+0, kPio2_2 = 0x1.1a62633145c07p-54, kPio2_3 = -0x1.f1976b7ed8fbcp-110;
constexpr double kSqrtHalf = 0x1.6a09e667f3bcdp-1;
constexpr double k128OverPi = 0x1.45f306dc9c883p+5;
constexpr double kPi128_1 = 0x1.921fb54442d18p-6, kPi128_2 = 0x1.1a62633145c07p-60;
// 2/pi in 32-bit words: bit 1 of word 0 is the 2^-1 bit (Payne-Hanek reduction of huge arguments)
constexpr uint32_t kTwoOverPiBits[12] = {0xA2F9836Eu, 0x4E441529u, 0xFC2757D1u, 0xF534DDC0u, 0xDB629599u, 0x3C439041u,
                                         0xFE5163ABu, 0xDEBBC561u, 0xB7246E3Au, 0x424DD2E0u, 0x06492EEAu, 0x09D1921Cu};
// |x| below this reduces with three-part Cody-Waite in double (n < 2^20: every step exact enough)
constexpr float kTrigFastLimit = 0x1p20f;

template <int N>
SRL_HD inline double horner(const double (&c)[N], double x) {
  double p = c[0];
#pragma unroll
  for (int i = 1; i < N; ++i) p = fma(p, x, c[i]);
  return p;
}

SRL_HD inline int to_int(double k) { return k == k ? int(k) : 0; }

}  // namespace srl

// exp(x) = 2^k e^r (the evaluator returns +Inf above Julia's MAX_EXP = 88.72284f0 before calling).
SRL_HD inline float sr_expf(float x) {
  const bool tiny = x < -104.0f;  // below e^-104 everything rounds to 0 (also -Inf)
  const double xd = tiny ? -104.0 : (x > 100.0f ? 100.0 : double(x));  // (above 88.73: +Inf)
  const double k = rint(xd * srl::kLog2e);
  double r = fma(-k, srl::kLn2Hi, xd);
  r = fma(-k, srl::kLn2Lo, r);
  const double p = srl::horner(srl::kExp, r);
  const float v = float(ldexp(p, srl::to_int(k)));
  return tiny ? 0.0f : v;
}

// log(x) = k ln2 + logc_i + log1p(z invc_i - 1) for x = 2^k z with z's Float32 bits in
// [0x3f330000, 0x3fb30000) (z ~ [0.699, 1.398): an offset octave, so x just below 1 keeps k = 0 with
// no branch), cell i = the 6 bits below the offset (64 cells, |z invc_i - 1| <= 2^-7), log1p by
// Taylor to r^4 (error <= 2^-37.3 absolute, <= 2^-30 relative to the result).  Every other step is
// exact or double: <= 0.5101 ulp after the final rounding (every positive normal Float32 checked,
// tools/libm_exhaustive.cpp).
// The f64 polynomial coefficients come in `c` (the device row function materialises them once per
// call in scalar registers: 64-bit constants cannot be VOP3 literals, and rematerialising them costs
// two v_mov per use and row).
struct SrLogC {
  double c3, c4, ln2;
};
constexpr SrLogC kSrLogC = {0x1.5555555555555p-2, -0.25, 0x1.62e42fefa39efp-1};
constexpr uint32_t kLogOff = 0x3f330000u;

// positive normal finite x (Float32 bits ix), scaled by 2^-kadj
SRL_HD inline double sr_log_normal(uint32_t ix, int kadj, const double* tab, const SrLogC& c) {
  const uint32_t tmp = ix - kLogOff;
  const uint32_t i = (tmp >> 17) & 63u;
  const int k = int32_t(tmp) >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  float z;
  __builtin_memcpy(&z, &iz, 4);
  const double invc = tab[2 * i], logc = tab[2 * i + 1];
  const double r = fma(double(z), invc, -1.0);
  // log1p(r) = r (1 + r (-1/2 + r (1/3 - r/4))) in Horner form, added to k ln2 + log c by the last
  // fused multiply-add: the dropped r^5/5 is <= 2^-37.3 absolute, <= 2^-30 of the result (|log x| >=
  // 2^-7.4 outside the cell of 1; |r| inside it).  Six f64 operations (round 3; was seven)
  double q = fma(r, c.c4, c.c3);
  q = fma(r, q, -0.5);
  q = fma(r, q, 1.0);
  return fma(r, q, fma(double(k + kadj), c.ln2, logc));
}

// Base.log over every Float32: +Inf -> +Inf, +-0 -> -Inf, x < 0 or NaN -> NaN; subnormals scaled by
// 2^23 (exact) first.  (The evaluator's safe_log maps x <= 0 to NaN before calling.)
SRL_HD inline float sr_logf_core(float x, const double* tab, const SrLogC& c) {
  uint32_t ix;
  __builtin_memcpy(&ix, &x, 4);
  if (ix - 0x00800000u < 0x7f000000u) return float(sr_log_normal(ix, 0, tab, c));  // positive normal
  if ((ix & 0x7fffffffu) == 0u) return -__builtin_inff();
  if (ix > 0x7f800000u) return __builtin_nanf("");  // negative (sign bit set) or NaN
  if (ix == 0x7f800000u) return x;
  const float xs = x * 0x1p23f;  // positive subnormal
  uint32_t is;
  __builtin_memcpy(&is, &xs, 4);
  return float(sr_log_normal(is, -23, tab, c));
}
SRL_HD inline float sr_logf_tab(float x, const double* tab) { return sr_logf_core(x, tab, kSrLogC); }

#if defined(__HIP_DEVICE_COMPILE__)
// a double constant in a scalar register pair (opaque to constant folding, so it stays there)
template <uint64_t B>
__device__ inline double srl_sconst() {
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"(uint32_t(B & 0xffffffffu)));
  asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"(uint32_t(B >> 32)));
  return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}
#define SRL_SCONST(v) srl_sconst<__builtin_bit_cast(uint64_t, double(v))>()
__device__ inline SrLogC sr_logc_sgpr() {
  return SrLogC{SRL_SCONST(kSrLogC.c3), SRL_SCONST(kSrLogC.c4), SRL_SCONST(kSrLogC.ln2)};
}
#elif defined(__HIPCC__)
// (host pass of device code: never executed)
__device__ inline SrLogC sr_logc_sgpr() { return kSrLogC; }
#endif

// sin / cos of the reduced argument y (|y| <= pi/4 + tiny) in quadrant q: sin(x) = (q & 1 ? cos : sin)
// with the sign of q & 2; cos(x) = the sin case of quadrant q + 1.
SRL_HD inline float sr_trig_kernel(double y, int q) {
  const double z = y * y;
  const double s = fma(y * z, srl::horner(srl::kSin, z), y);
  const double c = fma(z * z, srl::horner(srl::kCos, z), fma(-0.5, z, 1.0));
  const double v = (q & 1) ? c : s;
  return float((q & 2) ? -v : v);
}

// Payne-Hanek for |x| >= 2^20 (finite): x * 2/pi mod 4 from a 96-bit window of 2/pi's bits.
SRL_HD inline double sr_rem_pio2f_large(float x, int* q) {
  uint32_t bits;
  __builtin_memcpy(&bits, &x, 4);
  const int ex = int((bits >> 23) & 0xffu) - 127;  // x = M 2^(ex - 23), M 24 bits
  const uint64_t M = (bits & 0x7fffffu) | 0x800000u;
  // window = bits b_s .. b_{s+95} of 2/pi with s = ex - 24: x 2/pi mod 4 = M * window / 2^94 mod 4
  const int s0 = ex - 24 + 31;  // 0-based bit position in a table with one leading zero word
  auto word = [](int i) -> uint32_t { return i <= 0 ? 0u : srl::kTwoOverPiBits[i - 1]; };
  const int k = s0 >> 5, o = s0 & 31;
  auto win = [&](int j) -> uint32_t {  // 32 bits starting at bit (s0 + 32 j)
    const uint32_t a = word(k + j), b = word(k + j + 1);
    return o ? (a << o) | (b >> (32 - o)) : a;
  };
  const uint64_t w0 = win(0), w1 = win(1), w2 = win(2);
  const uint64_t p0 = M * w0, p1 = M * w1, p2 = M * w2;  // P = p0 2^64 + p1 2^32 + p2 (120 bits)
  const uint64_t lo_part = p2 + (p1 << 32);
  const uint64_t carry = lo_part < p2 ? 1u : 0u;
  const uint64_t hi = p0 + (p1 >> 32) + carry;
  int quad = int((hi >> 30) & 3u);
  const uint64_t top = ((hi & 0x3fffffffull) << 34) | (lo_part >> 30);  // fraction bits 93..30
  const uint64_t low = lo_part & 0x3fffffffull;                          // fraction bits 29..0
  double f = double(top) * 0x1p-64 + double(low) * 0x1p-94;
  const bool up = f >= 0.5;  // nearest quadrant: f in [-1/2, 1/2)
  f = up ? f - 1.0 : f;
  *q = up ? ((quad + 1) & 3) : quad;
  return f * srl::kPio2_1 + f * srl::kPio2_2;
}

// x mod pi/2 -> (y, quadrant)
SRL_HD inline double sr_rem_pio2f_fast(float x, int* q) {
  const double xd = double(x);
  const double n = rint(xd * srl::kTwoOverPi);
  double y = fma(-n, srl::kPio2_1, xd);
  y = fma(-n, srl::kPio2_2, y);
  y = fma(-n, srl::kPio2_3, y);
  *q = srl::to_int(n) & 3;
  return y;
}

// |x| < 2^20: x = n pi/128 + r (Cody-Waite in double), |r| <= pi/256; with (s_k, c_k) =
// (sin, cos)(k pi/128), k = n mod 256: sin x = s_k cos r + c_k sin r, cos x = c_k cos r - s_k sin r,
// with the Taylor terms of cos r and sin r through r^4 (round 5; -DSR_TRIG_DEG3 keeps rounds 3-4's
// cos r = 1 - r^2/2, sin r = r (1 - r^2/6), whose dropped r^4/24 <= 2^-30 of c_k gave <= 0.5223 ulp).
// The dropped r^5/120 <= 2^-38 stays far below the result's ulp wherever it is (next to a zero of the
// function c_k = 0 exactly and the result is -s_k sin r itself): <= 0.5025 ulp after the final
// rounding (tools/libm_exhaustive.cpp: every Float32 |x| < 2^20).  Seven f64 operations after the
// reduction, the terms in Horner form in r.
// (One copy of the (sin, cos)(k pi/128) table in LDS: round 5 measured 2 / 4 / 8 interleaved copies —
//  conflict-free reads — slower on every population, the extra LDS costing resident workgroups;
//  profiles/r05_ab_trig_copies.txt.  The option was removed in round 6.)
struct SrTrigArg {
  double r, sk, ck;
};
SRL_HD inline SrTrigArg sr_trig_arg(float x, const double* tab) {
  const double xd = double(x);
  // n = x 128/pi rounded to an integer by the 1.5 * 2^52 shifter: k = n mod 256 is the shifter's
  // low bits (no conversions; a NaN x only yields a NaN result).  Two-part Cody-Waite with fused
  // multiply-adds: |n| < 2^26, so the dropped third part (n * 2^-114 < 2^-88) is far below |r|'s ulp.
  const double t = fma(xd, srl::k128OverPi, 0x1.8p52);
  const double n = t - 0x1.8p52;
  double r = fma(-n, srl::kPi128_1, xd);
  r = fma(-n, srl::kPi128_2, r);
  uint64_t tb;
  __builtin_memcpy(&tb, &t, 8);
  // entry k = 16 bytes at byte offset 16 k
  const double* e = reinterpret_cast<const double*>(reinterpret_cast<const char*>(tab) + ((uint32_t(tb) << 4) & 0xff0u));
  return SrTrigArg{r, e[0], e[1]};
}
template <bool COS>
SRL_HD inline float sr_trig_poly(const SrTrigArg& p) {
  const double r = p.r, sk = p.sk, ck = p.ck;
  // cos x = ck + r (-sk + r (-ck/2 + r sk/6)), sin x = sk + r (ck + r (-sk/2 - r ck/6)): the same
  // Taylor terms in Horner form, five f64 operations (round 3; was six)
  const double a = COS ? ck : sk, b = COS ? -sk : ck;
  const double c2 = -0.5 * a, c3 = b * -0x1.5555555555555p-3;
#ifndef SR_TRIG_DEG3
  // round 5 default: one Taylor term more, r^4 a / 24 (two f64 operations per row).  Julia's Float32
  // cos / sin round a Float64 result; against that rounded double this body disagrees on 6,270 (cos)
  // and 32,478 (sin) of the 2.47e9 Float32 |x| < 2^20, the round-3/4 degree-3 body (-DSR_TRIG_DEG3)
  // on 1,274,326 and 1,170,066 (profiles/r04_trig_accuracy_ab.txt): parity comes before the 1-3 %
  const double c4 = a * 0x1.5555555555555p-5;
  return float(fma(r, fma(r, fma(r, fma(r, c4, c3), c2), b), a));
#else
  return float(fma(r, fma(r, fma(r, c3, c2), b), a));
#endif
}
template <bool COS>
SRL_HD inline float sr_sincosf_tab(float x, const double* tab) {
  return sr_trig_poly<COS>(sr_trig_arg(x, tab));
}

// Full range: the table path below 2^20, Payne-Hanek above (the device only comes here when some
// lane of the wave holds a huge argument, so the branch costs nothing in the common case).
template <bool COS>
SRL_HD inline float sr_sincosf_full(float x, const double* tab) {
  const float ax = fabsf(x);
  if (ax < srl::kTrigFastLimit) return sr_sincosf_tab<COS>(x, tab);
  if (!(ax <= 3.4028235e38f)) return __builtin_nanf("");  // sin/cos(+-Inf), NaN -> NaN
  int q = 0;
  const double y = sr_rem_pio2f_large(ax, &q);
  const float v = COS ? sr_trig_kernel(y, q + 1) : sr_trig_kernel(y, q);
  return (!COS && x < 0.0f) ? -v : v;
}

// ---------------------------------------------------------------- tables: host / device
#if defined(__HIPCC__)
// per-workgroup LDS copy of the tables (trig then log; 5 KiB: it must not cost the interpreter a
// workgroup per CU)
static __shared__ __attribute__((aligned(16))) double sr_lds_libm[512 + 128];
// Copy the tables into LDS: every thread of the block calls this before the block's first barrier.
__device__ inline void sr_libm_lds_fill(int tid, int nthreads) {
  for (int i = tid; i < 512; i += nthreads) sr_lds_libm[i] = srl::kTrigTab[i];
  for (int i = tid; i < 128; i += nthreads) sr_lds_libm[512 + i] = srl::kLogTab[i];
}
#endif
SRL_HD inline const double* sr_trig_tab() {
#if defined(__HIP_DEVICE_COMPILE__)
  return sr_lds_libm;
#else
  return srl::kTrigTab;
#endif
}
SRL_HD inline const double* sr_log_tab() {
#if defined(__HIP_DEVICE_COMPILE__)
  return sr_lds_libm + 512;
#else
  return srl::kLogTab;
#endif
}

SRL_HD inline float sr_sinf(float x) { return sr_sincosf_full<false>(x, sr_trig_tab()); }
SRL_HD inline float sr_cosf(float x) { return sr_sincosf_full<true>(x, sr_trig_tab()); }
SRL_HD inline float sr_sinf_fast(float x) { return sr_sincosf_tab<false>(x, sr_trig_tab()); }
SRL_HD inline float sr_cosf_fast(float x) { return sr_sincosf_tab<true>(x, sr_trig_tab()); }
SRL_HD inline float sr_logf(float x) { return sr_logf_tab(x, sr_log_tab()); }
