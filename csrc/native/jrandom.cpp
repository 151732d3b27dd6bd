// java.util.Random-compatible generator (48-bit LCG, polar-method nextGaussian).
//
// The reference seeds every random model initialisation with java.util.Random
// (J/utils/RandomParamsUtils.java: normal = nextGaussian*std+mean, uniform =
// a + (b-a)*nextDouble; FM/FFM latent init, GBMLR per-tree init with seed 99999 +
// finished*seed). Reproducing the exact stream makes a model initialised here match one
// initialised by the reference for the same seed.
#include <cmath>
#include <cstdint>
#include <vector>

#include "native.h"

namespace ytk_native {

JavaRandom::JavaRandom(int64_t seed) { set_seed(seed); }

void JavaRandom::set_seed(int64_t seed) {
  s_ = ((uint64_t)seed ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1);
  have_next_ = false;
}

int32_t JavaRandom::next(int bits) {
  s_ = (s_ * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
  return (int32_t)(int64_t)(s_ >> (48 - bits));
}

double JavaRandom::next_double() {
  const int64_t a = (int64_t)(uint32_t)next(26);
  const int64_t b = (int64_t)(uint32_t)next(27);
  return (double)((a << 27) + b) * 0x1.0p-53;
}

float JavaRandom::next_float() { return (float)(uint32_t)next(24) / (float)(1 << 24); }

int32_t JavaRandom::next_int(int32_t bound) {
  if ((bound & -bound) == bound) return (int32_t)(((int64_t)bound * (int64_t)(uint32_t)next(31)) >> 31);
  int32_t bits, val;
  do {
    bits = (int32_t)((uint32_t)next(31));
    val = bits % bound;
  } while (bits - val + (bound - 1) < 0);
  return val;
}

double JavaRandom::next_gaussian() {
  if (have_next_) {
    have_next_ = false;
    return next_g_;
  }
  double v1, v2, s;
  do {
    v1 = 2 * next_double() - 1;
    v2 = 2 * next_double() - 1;
    s = v1 * v1 + v2 * v2;
  } while (s >= 1 || s == 0);
  const double mul = std::sqrt(-2 * std::log(s) / s);
  next_g_ = v2 * mul;
  have_next_ = true;
  return v1 * mul;
}

std::vector<double> java_random_fill(int64_t seed, int64_t n, int mode, double a, double b) {
  JavaRandom r(seed);
  std::vector<double> out((size_t)std::max<int64_t>(n, 0));
  for (auto& v : out) {
    switch (mode) {
      case 0: v = r.next_gaussian() * b + a; break;          // normal(mean=a, std=b)
      case 1: v = a + (b - a) * r.next_double(); break;     // uniform[a, b)
      case 2: v = (double)r.next_float(); break;            // nextFloat
      default: v = r.next_double(); break;                  // nextDouble
    }
  }
  return out;
}

}  // namespace ytk_native
