// Host-side stress driver for the native runtime pieces (parser, murmur hash, java
// random, weighted quantile summary), built with -fsanitize=address,undefined and,
// separately, -fsanitize=thread by tools/sanitize_native.sh (sanitizers on
// the C++ parser). It feeds malformed and adversarial lines, checks the multi-threaded
// parse against the single-threaded one, and exercises summary prune/combine/query.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../native.h"
#include "../parser.h"

using namespace ytk_native;

static int fails = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      ++fails;                                                       \
    }                                                                \
  } while (0)

static std::string make_corpus(int lines, uint64_t seed) {
  std::mt19937_64 g(seed);
  std::string out;
  const char* junk[] = {"", "###", "1###", "1###x###", "###1###a:1", "1###1###:", "1###1###a:", "1###1###a:b",
                        "1###1###a:1,,b:2", "2###0,1###f@a:1,f@b:2###0.5", "nan###1###a:1", "1###1###a:1e400"};
  for (int i = 0; i < lines; ++i) {
    if (g() % 17 == 0) {
      out += junk[g() % (sizeof(junk) / sizeof(junk[0]))];
    } else {
      out += std::to_string(1 + g() % 3) + "###" + std::to_string(g() % 2) + "###";
      int k = 1 + g() % 12;
      for (int j = 0; j < k; ++j) {
        if (j) out += ",";
        out += "fld" + std::to_string(g() % 5) + "@x" + std::to_string(g() % 400) + ":" +
               std::to_string((g() % 1000) / 100.0);
      }
    }
    out += (g() % 50 == 0) ? "\r\n" : "\n";
  }
  return out;
}

int main() {
  const std::string corpus = make_corpus(40000, 7);
  ParseOptions o;
  o.max_error_tol = 1 << 30;
  o.split_field = true;
  o.want_stats = true;
  o.threads = 1;
  ParseResult a = parse_ytk(corpus.data(), corpus.size(), o);
  o.threads = 8;
  ParseResult b = parse_ytk(corpus.data(), corpus.size(), o);
  CHECK(a.n_rows == b.n_rows && a.n_rows > 30000);
  CHECK(a.names == b.names && a.feat == b.feat && a.val == b.val && a.indptr == b.indptr);
  CHECK(a.field == b.field && a.labels == b.labels && a.weight == b.weight);
  CHECK(a.n_errors == b.n_errors && a.n_errors > 0);
  // hashing + sampling + sharding paths
  o.feature_hash = true;
  o.hash_bucket = 97;
  o.y_sampling = {0.5f, 1.0f};
  o.sample_seed = 3;
  o.line_mod = 3;
  o.line_rem = 2;
  ParseResult c = parse_ytk(corpus.data(), corpus.size(), o);
  CHECK(c.n_rows > 0 && c.names.size() <= 97);
  // truncated buffer (no trailing newline) and empty input
  ParseResult d = parse_ytk(corpus.data(), 1000, o);
  CHECK(d.n_lines > 0);
  ParseResult e = parse_ytk("", 0, o);
  CHECK(e.n_rows == 0);
  // error tolerance aborts with an exception
  ParseOptions strict;
  bool threw = false;
  try {
    parse_ytk("bad\nworse\n", 10, strict);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  // hash / random helpers
  CHECK((uint64_t)murmur3_128_aslong("hello", 5, 0) == 0xcbd8a7b341bd9b02ULL);
  std::vector<double> r = java_random_fill(42, 1000, 3, 0.0, 1.0);
  CHECK(r.size() == 1000 && std::fabs(r[0] - 0.7275636800328681) < 1e-15);
  // weighted quantile summaries: build, combine, prune, query
  std::mt19937_64 g(1);
  std::vector<double> v(5000), w(5000);
  for (size_t i = 0; i < v.size(); ++i) {
    v[i] = (double)(g() % 100000) / 7.0;
    w[i] = 1.0 + (double)(g() % 5);
  }
  std::vector<size_t> idx(v.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return v[x] < v[y]; });
  std::vector<double> vs, ws;
  for (size_t i : idx) {
    if (!vs.empty() && vs.back() == v[i]) {
      ws.back() += w[i];
    } else {
      vs.push_back(v[i]);
      ws.push_back(w[i]);
    }
  }
  size_t half = vs.size() / 2;
  WQSummary s1 = WQSummary::from_sorted(vs.data(), ws.data(), half);
  WQSummary s2 = WQSummary::from_sorted(vs.data() + half, ws.data() + half, vs.size() - half);
  WQSummary all = WQSummary::combine(s1, s2).prune(64);
  CHECK(all.e.size() <= 64);
  double tot = all.total();
  double prev = -1e300;
  for (int q = 0; q <= 16; ++q) {
    double x = all.query(tot * q / 16.0);
    CHECK(x >= prev);
    prev = x;
  }
  if (fails) {
    std::fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  std::printf("native stress ok: %lld rows, %zu names, %lld errors\n", (long long)a.n_rows, a.names.size(),
              (long long)a.n_errors);
  return 0;
}
