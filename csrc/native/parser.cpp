// Multithreaded ytk text-format parser (host runtime; the GPU consumes its CSR output).
//
// Reference behaviour (J/dataflow/CoreData.java:322-447,536-611; FeatureHash.java:94-116):
//  * weight, labels (y_delim separated), features "name:value" (features_delim separated),
//    optional 4th field = init prediction(s);
//  * per line the features form a name->value map (a repeated name keeps the LAST value),
//    then optional signed feature hashing: bucket = (h & 0x7fffffff) % B, sign = bit 40,
//    colliding hashed names are summed;
//  * y_sampling keeps a row with probability rate (weight *= 1/rate for rate <= 1, *= rate
//    otherwise);
//  * malformed lines count as errors; more than max_error_tol aborts.
// Differences (documented): delimiters are literal strings (the reference passes them to
// Java's regex split), blank lines are skipped, a row may have no feature field, and the
// sampling RNG is a per-line counter hash so results do not depend on the thread count.
//
// Design: the buffer is cut at newlines into one chunk per thread; each thread keeps a
// local name dictionary (first-appearance order) and local CSR; chunks are merged in
// order so dictionary ids and row order are deterministic.
#include "parser.h"

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <limits>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <fstream>
#include <stdexcept>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "native.h"

namespace ytk_native {
namespace {

using sv = std::string_view;

inline sv trim(sv s) {
  size_t b = 0, e = s.size();
  while (b < e && (unsigned char)s[b] <= ' ') ++b;
  while (e > b && (unsigned char)s[e - 1] <= ' ') --e;
  return s.substr(b, e - b);
}

// Java Float.parseFloat-compatible enough: optional '+', trailing f/F/d/D, NaN; rejects
// +-Infinity (NumConvertUtils.parseFloat) and garbage.
inline bool parse_float(sv s, float* out) {
  s = trim(s);
  if (s.empty()) return false;
  if (s.front() == '+') s.remove_prefix(1);
  if (!s.empty()) {
    const char c = s.back();
    if (c == 'f' || c == 'F' || c == 'd' || c == 'D') s.remove_suffix(1);
  }
  if (s.empty()) return false;
  if (s == "NaN" || s == "-NaN") {
    *out = std::nanf("");
    return true;
  }
  // from_chars also takes "nan"/"inf"/"infinity" in any case; Java only "NaN" / "Infinity"
  {
    const char c0 = s.front() == '-' && s.size() > 1 ? s[1] : s.front();
    if (c0 == 'n' || c0 == 'N' || c0 == 'i' || c0 == 'I') return false;
  }
  // fast exact path: [-]digits[.digits][e[+-]digits] with <= 9 significant digits and a
  // mantissa < 2^24 and |exp10| <= 10 -- both operands exact in float, so one IEEE
  // multiply / divide is the correctly rounded result (what from_chars / Java return)
  {
    const char* c = s.data();
    const char* e = c + s.size();
    bool neg = false;
    if (*c == '-') { neg = true; ++c; }
    uint32_t m = 0;
    int nd = 0, frac = 0;
    bool dot = false, any = false, ok = c < e;
    for (; c < e; ++c) {
      const unsigned d = (unsigned)(*c - '0');
      if (d < 10) {
        any = true;
        if (nd || d) ++nd;
        if (nd > 9) { ok = false; break; }
        m = m * 10 + d;
        frac += dot;
      } else if (*c == '.' && !dot) {
        dot = true;
      } else {
        break;
      }
    }
    int ex = 0;
    if (ok && c < e && (*c == 'e' || *c == 'E')) {
      ++c;
      bool eneg = false;
      if (c < e && (*c == '-' || *c == '+')) eneg = *c++ == '-';
      if (c == e) ok = false;
      for (; ok && c < e; ++c) {
        const unsigned d = (unsigned)(*c - '0');
        if (d >= 10 || ex > 100) { ok = false; break; }
        ex = ex * 10 + (int)d;
      }
      if (eneg) ex = -ex;
    }
    ex -= frac;
    if (ok && any && c == e && m < (1u << 24) && ex >= -10 && ex <= 10) {
      static const float p10[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
      float v = (float)m;
      v = ex >= 0 ? v * p10[ex] : v / p10[-ex];
      *out = neg ? -v : v;
      return true;
    }
  }
  float v;
  auto r = std::from_chars(s.data(), s.data() + s.size(), v);
  if (r.ec != std::errc() || r.ptr != s.data() + s.size()) {
    // from_chars rejects values that underflow/overflow float; fall back to strtod
    if (r.ec == std::errc::result_out_of_range) {
      std::string tmp(s);
      char* end = nullptr;
      const double d = std::strtod(tmp.c_str(), &end);
      if (end != tmp.c_str() + tmp.size()) return false;
      v = (float)d;
    } else {
      return false;
    }
  }
  if (std::isinf(v)) return false;
  *out = v;
  return true;
}

// Split s by a literal delimiter into at most max_parts pieces (the last keeps the rest).
inline int split_n(sv s, const std::string& d, sv* parts, int max_parts) {
  int n = 0;
  size_t pos = 0;
  while (n < max_parts - 1) {
    const size_t q = s.find(d, pos);
    if (q == sv::npos) break;
    parts[n++] = s.substr(pos, q - pos);
    pos = q + d.size();
  }
  parts[n++] = s.substr(pos);
  return n;
}

template <typename F>
inline void for_each_split(sv s, const std::string& d, F&& f) {
  size_t pos = 0;
  while (true) {
    const size_t q = s.find(d, pos);
    if (q == sv::npos) {
      f(s.substr(pos));
      return;
    }
    f(s.substr(pos, q - pos));
    pos = q + d.size();
  }
}

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct SvHash {
  size_t operator()(sv s) const noexcept { return std::hash<sv>()(s); }
};

struct Local {
  // rows
  std::vector<float> weight, labels, init, val;
  std::vector<int64_t> row_line;
  std::vector<int64_t> label_ptr{0}, init_ptr{0}, indptr{0};
  std::vector<int32_t> feat, field;
  // dictionary (names owned here; map keys view into `names`)
  std::vector<std::string> names;
  std::deque<std::string> store;                    // stable storage the dict keys view into
  std::unordered_map<sv, int32_t, SvHash> dict;
  std::vector<int64_t> stamp;                       // last line index each id appeared on
  std::vector<int32_t> slot;                        // its position in that row
  std::vector<int32_t> pos_guess;                   // id seen at each token position last line
  std::vector<int64_t> counts;
  std::vector<double> st_sum, st_sum2, st_max, st_min;
  std::vector<std::string> fields;
  std::unordered_map<std::string, int32_t> fdict;
  int64_t n_lines = 0, n_errors = 0, n_sampled_out = 0;
  std::vector<std::string> errs;

  int32_t id_of(sv name, bool stats) {
    auto it = dict.find(name);
    if (it != dict.end()) return it->second;
    const int32_t id = (int32_t)names.size();
    store.emplace_back(name);
    names.emplace_back(name);
    dict.emplace(sv(store.back()), id);
    counts.push_back(0);
    stamp.push_back(-1);
    slot.push_back(0);
    if (stats) {
      st_sum.push_back(0.0);
      st_sum2.push_back(0.0);
      st_max.push_back(-INFINITY);
      st_min.push_back(INFINITY);
    }
    return id;
  }
  int32_t field_of(const std::string& f) {
    auto it = fdict.find(f);
    if (it != fdict.end()) return it->second;
    const int32_t id = (int32_t)fields.size();
    fields.push_back(f);
    fdict.emplace(f, id);
    return id;
  }
};

struct LineScratch {
  std::vector<std::pair<sv, float>> kv;          // raw (name, value) of a line
  std::unordered_map<sv, int, SvHash> seen;      // name -> slot in kv
  std::vector<std::pair<std::string, float>> hashed;
  std::unordered_map<std::string, int> hseen;
  std::vector<float> tmp, initv;
};

void parse_chunk(const char* p, size_t n, int64_t first_line, const ParseOptions& opt, Local& L) {
  LineScratch S;
  const bool stats = opt.want_stats;
  size_t pos = 0;
  int64_t li = first_line;
  while (pos < n) {
    const char* nl = static_cast<const char*>(std::memchr(p + pos, '\n', n - pos));
    const size_t end = nl ? (size_t)(nl - p) : n;
    sv line(p + pos, end - pos);
    pos = end + 1;
    const int64_t idx = li++;
    if (opt.line_mod > 1 && (idx % opt.line_mod) != opt.line_rem) continue;
    line = trim(line);
    if (line.empty()) continue;
    L.n_lines++;
    auto fail = [&]() {
      L.n_errors++;
      if (L.errs.size() < 5) L.errs.emplace_back(line.substr(0, 512));
    };
    sv parts[4];
    const int np = split_n(line, opt.x_delim, parts, 4);
    if (np < 2) { fail(); continue; }
    float w;
    if (!parse_float(parts[0], &w)) { fail(); continue; }
    // labels (may be empty for predict/test lines)
    S.tmp.clear();
    bool bad = false;
    sv ys = trim(parts[1]);
    if (!ys.empty()) {
      for_each_split(ys, opt.y_delim, [&](sv t) {
        float v;
        if (!parse_float(t, &v)) bad = true;
        else S.tmp.push_back(v);
      });
    }
    if (bad) { fail(); continue; }
    if (!opt.y_sampling.empty() && !S.tmp.empty()) {
      const int lab = (int)S.tmp[0];
      const float rate = (lab >= 0 && lab < (int)opt.y_sampling.size()) ? opt.y_sampling[lab] : 1.0f;
      if (rate <= 1.0f) w *= (1.0f / rate);
      else w *= rate;
      const uint64_t r = mix64(opt.sample_seed ^ mix64((uint64_t)idx));
      const float u = (float)((r >> 40) * (1.0 / 16777216.0));
      if (!(u <= rate)) { L.n_sampled_out++; continue; }
    }
    // features -> per-line map, last value wins
    S.kv.clear();
    S.seen.clear();
    if (np >= 3) {
      sv fs = trim(parts[2]);
      if (!fs.empty()) {
        for_each_split(fs, opt.feat_delim, [&](sv tok) {
          if (bad) return;
          tok = trim(tok);
          if (tok.empty()) return;
          const size_t q = tok.find(opt.kv_delim);
          if (q == sv::npos) { bad = true; return; }
          sv name = trim(tok.substr(0, q));
          sv vs = tok.substr(q + opt.kv_delim.size());
          const size_t q2 = vs.find(opt.kv_delim);
          if (q2 != sv::npos) vs = vs.substr(0, q2);
          float v;
          if (name.empty() || !parse_float(vs, &v)) { bad = true; return; }
          if (!opt.feature_hash) {  // deduplicated by dictionary id at commit
            S.kv.emplace_back(name, v);
            return;
          }
          auto it = S.seen.find(name);
          if (it != S.seen.end()) S.kv[it->second].second = v;
          else {
            S.seen.emplace(name, (int)S.kv.size());
            S.kv.emplace_back(name, v);
          }
        });
      }
    }
    if (bad) { fail(); continue; }
    // init prediction(s)
    auto& initv = S.initv;
    initv.clear();
    if (np >= 4) {
      sv is = trim(parts[3]);
      if (!is.empty()) {
        for_each_split(is, opt.y_delim, [&](sv t) {
          float v;
          if (!parse_float(t, &v)) bad = true;
          else initv.push_back(v);
        });
      }
    }
    if (bad) { fail(); continue; }
    // commit row
    L.weight.push_back(w);
    L.row_line.push_back(idx);
    L.labels.insert(L.labels.end(), S.tmp.begin(), S.tmp.end());
    L.label_ptr.push_back((int64_t)L.labels.size());
    L.init.insert(L.init.end(), initv.begin(), initv.end());
    L.init_ptr.push_back((int64_t)L.init.size());
    // row entries: first-appearance order, last value wins (stamp/slot by dictionary id)
    const size_t row0 = L.feat.size();
    size_t pos_k = 0;
    auto put = [&](sv name, float v) {
      // dense data repeats the previous line's name at each position: check that guess
      // before hashing
      int32_t id;
      if (pos_k < L.pos_guess.size() && L.names[L.pos_guess[pos_k]] == name) {
        id = L.pos_guess[pos_k];
      } else {
        id = L.id_of(name, stats);
        if (pos_k < L.pos_guess.size()) L.pos_guess[pos_k] = id;
        else L.pos_guess.push_back(id);
      }
      ++pos_k;
      if (L.stamp[id] == idx) {
        L.val[row0 + L.slot[id]] = v;
        return;
      }
      L.stamp[id] = idx;
      L.slot[id] = (int32_t)(L.feat.size() - row0);
      L.feat.push_back(id);
      L.val.push_back(v);
    };
    if (opt.feature_hash) {
      S.hashed.clear();
      S.hseen.clear();
      for (auto& kv : S.kv) {
        const int64_t h = murmur3_128_aslong(kv.first.data(), kv.first.size(), opt.hash_seed);
        const int64_t bucket = (int64_t)((uint64_t)h & 0x7fffffffULL) % opt.hash_bucket;
        const float sign = 2.0f * (float)(((uint64_t)h & 0x10000000000ULL) >> 40) - 1.0f;
        std::string hn = opt.hash_prefix + std::to_string(bucket);
        auto it = S.hseen.find(hn);
        if (it != S.hseen.end()) S.hashed[it->second].second += sign * kv.second;
        else {
          S.hseen.emplace(hn, (int)S.hashed.size());
          S.hashed.emplace_back(std::move(hn), sign * kv.second);
        }
      }
      for (auto& hv : S.hashed) put(sv(hv.first), hv.second);
    } else {
      for (auto& kv : S.kv) put(kv.first, kv.second);
    }
    for (size_t e = row0; e < L.feat.size(); ++e) {
      const int32_t id = L.feat[e];
      const float v = L.val[e];
      L.counts[id]++;
      if (stats) {
        L.st_sum[id] += v;
        L.st_sum2[id] += (double)(v * v);
        L.st_max[id] = std::max(L.st_max[id], (double)v);
        L.st_min[id] = std::min(L.st_min[id], (double)v);
      }
      if (opt.split_field) {  // field = name prefix before field_delim (whole name if absent)
        const std::string& name = L.names[id];
        const size_t q = name.find(opt.field_delim);
        L.field.push_back(L.field_of(q == std::string::npos ? name : name.substr(0, q)));
      }
    }
    L.indptr.push_back((int64_t)L.feat.size());
  }
}

int64_t count_lines(const char* p, size_t n) {
  int64_t c = 0;
  size_t pos = 0;
  while (pos < n) {
    const char* nl = static_cast<const char*>(std::memchr(p + pos, '\n', n - pos));
    if (!nl) { ++c; break; }
    ++c;
    pos = (size_t)(nl - p) + 1;
  }
  return c;
}

}  // namespace

int default_threads() {
  // the process's CPU share, not the machine's: OMP_NUM_THREADS if set (the GPU pool sets
  // it to the job's share), else the affinity mask
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return v;
  }
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) return std::max(1, CPU_COUNT(&cs));
  return (int)std::max(1u, std::thread::hardware_concurrency());
}

void csr_to_dense(const int64_t* indptr, const int32_t* feat, const float* val, int64_t n_rows, const int64_t* lut,
                  int64_t n_lut, int64_t F, float* out, int threads) {
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads > 0 ? threads : default_threads(),
                                                            n_rows / 65536 + 1));
  auto work = [&](int t) {
    const int64_t r0 = n_rows * t / T, r1 = n_rows * (t + 1) / T;
    std::fill(out + r0 * F, out + r1 * F, std::numeric_limits<float>::quiet_NaN());
    for (int64_t r = r0; r < r1; ++r) {
      float* o = out + r * F;
      for (int64_t e = indptr[r]; e < indptr[r + 1]; ++e) {
        const int32_t f = feat[e];
        if (f < 0 || f >= n_lut) continue;
        const int64_t c = lut[f];
        if (c >= 0 && c < F) o[c] = val[e];
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}

ParseResult parse_ytk(const char* data, size_t len, const ParseOptions& opt) {
  if (opt.line_mod < 1 || opt.line_rem < 0 || opt.line_rem >= opt.line_mod)
    throw std::invalid_argument("parse_ytk: bad line sharding");
  if (opt.feature_hash && opt.hash_bucket <= 0)
    throw std::invalid_argument("parse_ytk: hash bucket_size must be > 0");
  int T = opt.threads > 0 ? opt.threads : default_threads();
  if (len < (size_t)(1 << 20)) T = 1;
  T = std::max(1, std::min(T, 64));
  // chunk boundaries at newlines
  std::vector<size_t> cut{0};
  for (int t = 1; t < T; ++t) {
    size_t c = std::max(cut.back(), len * (size_t)t / (size_t)T);
    if (c >= len) break;
    const char* nl = static_cast<const char*>(std::memchr(data + c, '\n', len - c));
    c = nl ? (size_t)(nl - data) + 1 : len;
    if (c > cut.back() && c < len) cut.push_back(c);
  }
  cut.push_back(len);
  const int C = (int)cut.size() - 1;
  // global line index of every chunk's first line: sharding (line_mod), y-sampling (keyed
  // by line index) and row_line must not depend on the thread count
  std::vector<int64_t> first_line(C, 0);
  if (C > 1) {
    std::vector<int64_t> nlines(C);
    std::vector<std::thread> th;
    for (int c = 0; c < C; ++c)
      th.emplace_back([&, c] { nlines[c] = count_lines(data + cut[c], cut[c + 1] - cut[c]); });
    for (auto& t : th) t.join();
    for (int c = 1; c < C; ++c) first_line[c] = first_line[c - 1] + nlines[c - 1];
  }
  std::vector<Local> loc(C);
  std::vector<std::exception_ptr> errs(C);
  {
    std::vector<std::thread> th;
    for (int c = 0; c < C; ++c)
      th.emplace_back([&, c] {
        try {
          parse_chunk(data + cut[c], cut[c + 1] - cut[c], first_line[c], opt, loc[c]);
        } catch (...) {
          errs[c] = std::current_exception();
        }
      });
    for (auto& t : th) t.join();
  }
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);

  ParseResult R;
  for (auto& L : loc) {
    R.n_lines += L.n_lines;
    R.n_errors += L.n_errors;
    R.n_sampled_out += L.n_sampled_out;
    for (auto& s : L.errs)
      if (R.error_samples.size() < 5) R.error_samples.push_back(s);
  }
  if (R.n_errors > opt.max_error_tol) {
    std::string msg = "[ERROR] error num:" + std::to_string(R.n_errors) + " > max tol:" +
                      std::to_string(opt.max_error_tol) + "; first bad line: ";
    msg += R.error_samples.empty() ? std::string("?") : R.error_samples[0];
    throw std::runtime_error(msg);
  }
  // global dictionary in chunk order
  std::unordered_map<std::string, int32_t> gdict, gfdict;
  std::vector<std::vector<int32_t>> remap(C), fremap(C);
  for (int c = 0; c < C; ++c) {
    auto& L = loc[c];
    remap[c].resize(L.names.size());
    for (size_t i = 0; i < L.names.size(); ++i) {
      auto it = gdict.find(L.names[i]);
      int32_t g;
      if (it == gdict.end()) {
        g = (int32_t)R.names.size();
        gdict.emplace(L.names[i], g);
        R.names.push_back(L.names[i]);
        R.counts.push_back(0);
        if (opt.want_stats) {
          R.st_sum.push_back(0.0);
          R.st_sum2.push_back(0.0);
          R.st_max.push_back(-INFINITY);
          R.st_min.push_back(INFINITY);
        }
      } else {
        g = it->second;
      }
      remap[c][i] = g;
      R.counts[g] += L.counts[i];
      if (opt.want_stats) {
        R.st_sum[g] += L.st_sum[i];
        R.st_sum2[g] += L.st_sum2[i];
        R.st_max[g] = std::max(R.st_max[g], L.st_max[i]);
        R.st_min[g] = std::min(R.st_min[g], L.st_min[i]);
      }
    }
    fremap[c].resize(L.fields.size());
    for (size_t i = 0; i < L.fields.size(); ++i) {
      auto it = gfdict.find(L.fields[i]);
      if (it == gfdict.end()) {
        const int32_t g = (int32_t)R.fields.size();
        gfdict.emplace(L.fields[i], g);
        R.fields.push_back(L.fields[i]);
        fremap[c][i] = g;
      } else {
        fremap[c][i] = it->second;
      }
    }
  }
  // concatenate rows: per-chunk output offsets, then every chunk copies (and remaps its
  // local ids) into the preallocated result on its own thread
  std::vector<size_t> ro(C + 1, 0), fo(C + 1, 0), lo(C + 1, 0), io(C + 1, 0);
  for (int c = 0; c < C; ++c) {
    ro[c + 1] = ro[c] + loc[c].weight.size();
    fo[c + 1] = fo[c] + loc[c].feat.size();
    lo[c + 1] = lo[c] + loc[c].labels.size();
    io[c + 1] = io[c] + loc[c].init.size();
  }
  const size_t nrows = ro[C], nnz = fo[C];
  R.n_rows = (int64_t)nrows;
  R.weight.resize(nrows);
  R.row_line.resize(nrows);
  R.label_ptr.resize(nrows + 1);
  R.init_ptr.resize(nrows + 1);
  R.indptr.resize(nrows + 1);
  R.labels.resize(lo[C]);
  R.init.resize(io[C]);
  R.feat.resize(nnz);
  R.val.resize(nnz);
  if (opt.split_field) R.field.resize(nnz);
  R.label_ptr[0] = R.init_ptr[0] = R.indptr[0] = 0;
  auto copy_chunk = [&](int c) {
    Local& L = loc[c];
    const size_t r0 = ro[c];
    std::copy(L.weight.begin(), L.weight.end(), R.weight.begin() + r0);
    std::copy(L.row_line.begin(), L.row_line.end(), R.row_line.begin() + r0);
    std::copy(L.labels.begin(), L.labels.end(), R.labels.begin() + lo[c]);
    std::copy(L.init.begin(), L.init.end(), R.init.begin() + io[c]);
    for (size_t i = 1; i < L.label_ptr.size(); ++i) R.label_ptr[r0 + i] = L.label_ptr[i] + (int64_t)lo[c];
    for (size_t i = 1; i < L.init_ptr.size(); ++i) R.init_ptr[r0 + i] = L.init_ptr[i] + (int64_t)io[c];
    for (size_t i = 1; i < L.indptr.size(); ++i) R.indptr[r0 + i] = L.indptr[i] + (int64_t)fo[c];
    const int32_t* rm = remap[c].data();
    int32_t* dst = R.feat.data() + fo[c];
    for (size_t i = 0; i < L.feat.size(); ++i) dst[i] = rm[L.feat[i]];
    std::copy(L.val.begin(), L.val.end(), R.val.begin() + fo[c]);
    if (opt.split_field) {
      const int32_t* fm = fremap[c].data();
      for (size_t i = 0; i < L.field.size(); ++i) R.field[fo[c] + i] = fm[L.field[i]];
    }
    L = Local();  // release
  };
  if (C == 1) {
    copy_chunk(0);
  } else {
    std::vector<std::thread> th;
    for (int c = 0; c < C; ++c) th.emplace_back(copy_chunk, c);
    for (auto& t : th) t.join();
  }
  return R;
}

ParseResult parse_ytk_files(const std::vector<std::string>& paths, const ParseOptions& opt) {
  if (paths.size() == 1) {  // one file: parse the mapped pages in place (no 3-GB copy)
    const int fd = ::open(paths[0].c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open data file: " + paths[0]);
    struct stat st;
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      throw std::runtime_error("cannot stat data file: " + paths[0]);
    }
    const size_t sz = (size_t)st.st_size;
    if (sz == 0) {
      ::close(fd);
      return parse_ytk("", 0, opt);
    }
    void* p = ::mmap(nullptr, sz, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("cannot map data file: " + paths[0]);
    ::madvise(p, sz, MADV_SEQUENTIAL);
    try {
      ParseResult r = parse_ytk(static_cast<const char*>(p), sz, opt);
      ::munmap(p, sz);
      return r;
    } catch (...) {
      ::munmap(p, sz);
      throw;
    }
  }
  std::string buf;
  for (const auto& path : paths) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open data file: " + path);
    f.seekg(0, std::ios::end);
    const std::streamoff sz = f.tellg();
    f.seekg(0, std::ios::beg);
    const size_t off = buf.size();
    buf.resize(off + (size_t)sz);
    f.read(&buf[off], sz);
    if (!buf.empty() && buf.back() != '\n') buf.push_back('\n');
  }
  return parse_ytk(buf.data(), buf.size(), opt);
}

}  // namespace ytk_native
