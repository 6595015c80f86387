// sr_rng.h — the native search's random streams (host only).
//
// One xoshiro256** stream per island (seeded from (seed, island) by splitmix64), so an island's
// trajectory does not depend on which rank owns it or on how many islands share a device launch.
// The draws are defined here once and restated bit for bit by the test oracle
// (oracle/search_oracle.py), which is what pins the C++ search to an independent implementation:
//   rand()        (u >> 11) * 2^-53                  Float64 in [0, 1)      (Julia rand())
//   rand(Float32) (u >> 40) * 2^-24                  Float32 in [0, 1)      (rand(rng, Float32))
//   rand(1:n)     1 + ((u >> 32) * n >> 32)          n < 2^32               (rand(rng, 1:n))
//   rand(Bool)    u >> 63
//   randn()       Box-Muller on two rand(): sqrt(-2 log(1 - u1)) cos(2 pi u2) (one value per pair)
// Julia's own streams (Xoshiro + ziggurat randn) are not reproduced: a run is reproducible from its
// seed, not equal to a Julia run's.
#pragma once
#include <math.h>
#include <stdint.h>

struct SrRng {
  uint64_t s[4] = {1, 2, 3, 4};

  static uint64_t splitmix(uint64_t* x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  // stream for key (a, b): the state words are four splitmix64 outputs from a ^ rotl(b, 32)
  void seed(uint64_t a, uint64_t b) {
    uint64_t x = a ^ ((b << 32) | (b >> 32)) ^ 0x5d6a7e1f3c2b4a99ull;
    for (auto& w : s) w = splitmix(&x);
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  double uniform() { return double(next() >> 11) * 0x1p-53; }
  float uniform_f32() { return float(next() >> 40) * 0x1p-24f; }
  template <typename T>
  T uniform_t() {
    if constexpr (sizeof(T) == 4)
      return uniform_f32();
    else
      return uniform();
  }
  // 0-based uniform index below n (n >= 1)
  int64_t below(int64_t n) { return int64_t(((next() >> 32) * uint64_t(n)) >> 32); }
  bool coin() { return (next() >> 63) != 0; }
  double normal() {
    const double u1 = uniform(), u2 = uniform();
    return sqrt(-2.0 * log(1.0 - u1)) * cos(6.283185307179586 * u2);
  }
};
