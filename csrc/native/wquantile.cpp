// Weighted, mergeable epsilon-approximate quantile summary (host runtime).
//
// Reference component: J/utils/WeightApproximateQuantile.java (Zhang & Wang style
// multi-level summary, cited at docs/gbdt_features.md:141), used for
// sample_by_quantile candidate generation, quantile missing-value fill and the l1 leaf
// refine. Each entry keeps (value, rmin, rmax, wmin): the rank interval of the value and
// the weight of exactly that value. Building from sorted (value, weight) data is exact;
// prune() keeps `size` entries at evenly spaced ranks (error <= W / size); combine() merges
// two summaries (errors add); query() returns the value whose rank interval is closest to
// the requested rank. Summaries are plain arrays so ranks can ship them through any
// object collective and merge them in a fixed order (deterministic).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "native.h"

namespace ytk_native {

WQSummary WQSummary::from_sorted(const double* v, const double* w, size_t n) {
  WQSummary s;
  s.e.reserve(n);
  double r = 0.0;
  for (size_t i = 0; i < n;) {
    const double x = v[i];
    double wx = 0.0;
    while (i < n && v[i] == x) wx += w[i++];  // merge equal values
    s.e.push_back({x, r, r + wx, wx});
    r += wx;
  }
  return s;
}

double WQSummary::total() const { return e.empty() ? 0.0 : e.back().rmax; }

WQSummary WQSummary::prune(size_t size) const {
  if (e.size() <= size || size < 3) return *this;
  WQSummary out;
  out.e.reserve(size);
  const double W = total();
  out.e.push_back(e.front());
  size_t i = 1;
  const size_t n = e.size();
  for (size_t k = 1; k + 1 < size; ++k) {
    const double d = W * (double)k / (double)(size - 1);  // target rank
    // advance to the first entry whose (rmin + rmax) / 2 >= d, then take the nearer of it
    // and its predecessor
    while (i + 1 < n && (e[i].rmin + e[i].rmax) * 0.5 < d) ++i;
    size_t j = i;
    if (i > 1) {
      const double a = std::fabs((e[i - 1].rmin + e[i - 1].rmax) * 0.5 - d);
      const double b = std::fabs((e[i].rmin + e[i].rmax) * 0.5 - d);
      if (a < b) j = i - 1;
    }
    if (j >= 1 && j + 1 < n && e[j].v != out.e.back().v) out.e.push_back(e[j]);
  }
  if (e.back().v != out.e.back().v) out.e.push_back(e.back());
  return out;
}

WQSummary WQSummary::combine(const WQSummary& a, const WQSummary& b) {
  if (a.e.empty()) return b;
  if (b.e.empty()) return a;
  WQSummary out;
  out.e.reserve(a.e.size() + b.e.size());
  size_t i = 0, j = 0;
  double a_prev_rmin = 0.0, b_prev_rmin = 0.0;
  while (i < a.e.size() && j < b.e.size()) {
    const Entry& x = a.e[i];
    const Entry& y = b.e[j];
    if (x.v == y.v) {
      out.e.push_back({x.v, x.rmin + y.rmin, x.rmax + y.rmax, x.wmin + y.wmin});
      a_prev_rmin = x.rmin + x.wmin;
      b_prev_rmin = y.rmin + y.wmin;
      ++i;
      ++j;
    } else if (x.v < y.v) {
      out.e.push_back({x.v, x.rmin + b_prev_rmin, x.rmax + (y.rmax - y.wmin), x.wmin});
      a_prev_rmin = x.rmin + x.wmin;
      ++i;
    } else {
      out.e.push_back({y.v, y.rmin + a_prev_rmin, y.rmax + (x.rmax - x.wmin), y.wmin});
      b_prev_rmin = y.rmin + y.wmin;
      ++j;
    }
  }
  const double a_tot = a.total(), b_tot = b.total();
  for (; i < a.e.size(); ++i) {
    const Entry& x = a.e[i];
    out.e.push_back({x.v, x.rmin + b_prev_rmin, x.rmax + b_tot, x.wmin});
  }
  for (; j < b.e.size(); ++j) {
    const Entry& y = b.e[j];
    out.e.push_back({y.v, y.rmin + a_prev_rmin, y.rmax + a_tot, y.wmin});
  }
  return out;
}

double WQSummary::query(double rank) const {
  if (e.empty()) throw std::runtime_error("quantile query on an empty summary");
  const double d2 = 2.0 * rank;
  if (d2 <= e.front().rmin + e.front().rmax) return e.front().v;
  if (d2 >= e.back().rmin + e.back().rmax) return e.back().v;
  size_t lo = 0, hi = e.size() - 1;  // first entry with rmin + rmax >= d2
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (e[mid].rmin + e[mid].rmax < d2) lo = mid + 1;
    else hi = mid;
  }
  const double a = d2 - (e[lo - 1].rmin + e[lo - 1].rmax);
  const double b = (e[lo].rmin + e[lo].rmax) - d2;
  return (a < b) ? e[lo - 1].v : e[lo].v;
}

}  // namespace ytk_native
