// sr_libm.h — Float32 exp / log / cos / sin for the evaluator (host + device), computed in double
// and rounded once.
//
// The reference evaluates these with Julia's Base.Math, accurate to < 1 ulp (its Float32 trig and
// log kernels work in Float64, as these do).  ROCm's OCML Float32 versions measured 1.26-1.75 ulp
// on the fixture points of tests/golden/libm_ulp.json (profiles/r02_libm_ocml.txt), so the device
// uses these instead: every fast-path result is within 2^-40 relative of the exact value before the
// final rounding (polynomial fits and bounds: tools/gen_libm_coeffs.py), i.e. correctly rounded
// unless the exact value lies within 2^-40 of a rounding midpoint, and never more than
// 0.5 + 2^-16 ulp off.  MI355X runs FP64 FMA at the FP32 (non-packed) rate, so the double work
// costs about what OCML's Float32 range reductions and slow-path branches do.
//
// The same functions run on the host (constant folding in sr_compile.cpp, tools/libm_check.cpp):
// IEEE double with fused multiply-adds and no contraction, so host and device agree bit for bit.
#pragma once
#include <math.h>
#include <stdint.h>

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

// log(x): x = 2^e m, m in [sqrt(1/2), sqrt(2)), log = e ln2 + log1p(m - 1).
SRL_HD inline float sr_logf(float x) {
  int e = 0;
  double m = frexp(double(x), &e);  // [0.5, 1)
  const bool lo = m < srl::kSqrtHalf;
  m = lo ? m * 2.0 : m;
  const double ed = double(lo ? e - 1 : e);
  const double f = m - 1.0;  // exact (Sterbenz)
  const double f2 = f * f;
  const double l = fma(f2 * f, srl::horner(srl::kLog, f), fma(-0.5, f2, f));
  const float v = float(fma(ed, srl::kLn2Hi, fma(ed, srl::kLn2Lo, l)));
  // (+Inf -> +Inf; outside safe_log's domain as Base.log: 0 -> -Inf, x < 0 or NaN -> NaN)
  return x == __builtin_inff() ? x : (x > 0.0f ? v : (x == 0.0f ? -__builtin_inff() : __builtin_nanf("")));
}

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

// fast path only: |x| < 2^20 (the kernel checks the whole wave once and takes sr_sinf / sr_cosf
// otherwise)
SRL_HD inline float sr_sinf_fast(float x) {
  int q = 0;
  const double y = sr_rem_pio2f_fast(x, &q);
  return sr_trig_kernel(y, q);
}
SRL_HD inline float sr_cosf_fast(float x) {
  int q = 0;
  const double y = sr_rem_pio2f_fast(x, &q);
  return sr_trig_kernel(y, q + 1);
}

// Full range, branch-free (selects: no divergent control flow in the interpreter's unrolled rows).
SRL_HD inline float sr_sinf(float x) {
  const float ax = fabsf(x);
  const bool fast = ax < srl::kTrigFastLimit;
  const float xl = (fast || !(ax <= 3.4028235e38f)) ? 0x1p20f : ax;  // (a finite stand-in)
  int ql = 0, qf = 0;
  const double yl = sr_rem_pio2f_large(xl, &ql);
  const double yf = sr_rem_pio2f_fast(fast ? x : 0.0f, &qf);
  const float vl = sr_trig_kernel(yl, ql);
  const float v = fast ? sr_trig_kernel(yf, qf) : (x < 0.0f ? -vl : vl);
  return ax <= 3.4028235e38f ? v : __builtin_nanf("");  // sin(+-Inf), NaN -> NaN
}
SRL_HD inline float sr_cosf(float x) {
  const float ax = fabsf(x);
  const bool fast = ax < srl::kTrigFastLimit;
  const float xl = (fast || !(ax <= 3.4028235e38f)) ? 0x1p20f : ax;
  int ql = 0, qf = 0;
  const double yl = sr_rem_pio2f_large(xl, &ql);
  const double yf = sr_rem_pio2f_fast(fast ? x : 0.0f, &qf);
  const float v = fast ? sr_trig_kernel(yf, qf + 1) : sr_trig_kernel(yl, ql + 1);
  return ax <= 3.4028235e38f ? v : __builtin_nanf("");
}
