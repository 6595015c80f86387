// Exhaustive host check of the Float32 cos / sin / log fast paths of csrc/sr_libm.h (the device runs
// the same arithmetic): every Float32 x in the fast path's domain against glibc's double-precision
// function (within 0.5 ulp of double: ~2^-29 ulp of float), reporting the maximum error in Float32 ulps
// and how many results differ from the double result rounded to Float32.
//   g++ -O2 -fopenmp -ffp-contract=off -I symbolicregression.jl_amd/csrc tools/libm_exhaustive.cpp -o /tmp/libm_ex
//   /tmp/libm_ex [cos|sin|log]
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "sr_libm.h"

static double ulp_err(float got, double ref) {
  if (ref == 0.0) return got == 0.0f ? 0.0 : 1e30;
  int e;
  frexp(ref, &e);                      // |ref| in [2^(e-1), 2^e)
  const double ulp = ldexp(1.0, (e - 1) - 23 < -149 ? -149 : (e - 1) - 23);
  return fabs(double(got) - ref) / ulp;
}

int main(int argc, char** argv) {
  const char* fn = argc > 1 ? argv[1] : "cos";
  const bool is_log = strcmp(fn, "log") == 0, is_sin = strcmp(fn, "sin") == 0;
  // domain: trig |x| < 2^20 (the fast path); log: positive normal finite
  const uint32_t lo = is_log ? 0x00800000u : 0u, hi = is_log ? 0x7f800000u : 0x49800000u;
  double maxe = 0.0;
  float worst = 0.0f;
  long long ndiff = 0, n = 0;
#pragma omp parallel
  {
    double me = 0.0;
    float mw = 0.0f;
    long long nd = 0, nn = 0;
#pragma omp for schedule(dynamic, 1 << 16)
    for (long long b = lo; b < (long long)hi; ++b) {
      for (int s = 0; s < (is_log ? 1 : 2); ++s) {
        const uint32_t bits = uint32_t(b) | (s ? 0x80000000u : 0u);
        float x;
        memcpy(&x, &bits, 4);
        float got;
        double ref;
        if (is_log) {
          got = sr_logf(x);
          ref = log(double(x));
        } else if (is_sin) {
          got = sr_sinf_fast(x);
          ref = sin(double(x));
        } else {
          got = sr_cosf_fast(x);
          ref = cos(double(x));
        }
        const double e = ulp_err(got, ref);
        if (e > me) {
          me = e;
          mw = x;
        }
        nd += got != float(ref);
        ++nn;
      }
    }
#pragma omp critical
    {
      if (me > maxe) {
        maxe = me;
        worst = mw;
      }
      ndiff += nd;
      n += nn;
    }
  }
  printf("%s: %lld inputs, max error %.6f ulp at x = %a, %lld results differ from the double result rounded\n", fn,
         n, maxe, worst, ndiff);
  return maxe <= 1.0 ? 0 : 1;
}
