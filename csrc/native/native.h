// Host-side (CPU) native runtime for ytk-learn-amd.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace ytk_native {

int64_t murmur3_128_aslong(const char* data, size_t len, uint32_t seed);

// java.util.Random stream (jrandom.cpp)
class JavaRandom {
 public:
  explicit JavaRandom(int64_t seed);
  void set_seed(int64_t seed);
  int32_t next(int bits);
  double next_double();
  float next_float();
  int32_t next_int(int32_t bound);
  double next_gaussian();

 private:
  uint64_t s_ = 0;
  bool have_next_ = false;
  double next_g_ = 0.0;
};

// mode 0: nextGaussian*b + a, 1: a + (b-a)*nextDouble, 2: nextFloat, 3: nextDouble
std::vector<double> java_random_fill(int64_t seed, int64_t n, int mode, double a, double b);

// weighted mergeable quantile summary (wquantile.cpp)
struct WQSummary {
  struct Entry {
    double v, rmin, rmax, wmin;
  };
  std::vector<Entry> e;
  static WQSummary from_sorted(const double* v, const double* w, size_t n);
  static WQSummary combine(const WQSummary& a, const WQSummary& b);
  WQSummary prune(size_t size) const;
  double query(double rank) const;
  double total() const;
};

}  // namespace ytk_native
