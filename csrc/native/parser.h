// Multithreaded parser for the ytk-learn text data format.
//
// Line format (reference docs/data_format.md; J/dataflow/CoreData.java:536-611):
//   weight <x> label[<y>label...] <x> name<kv>value<f>name<kv>value... [<x> init[<y>init...]]
// with <x> = x_delim ("###"), <y> = y_delim (","), <f> = features_delim (","),
// <kv> = feature_name_val_delim (":"). Delimiters are literal strings.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ytk_native {

struct ParseOptions {
  std::string x_delim = "###";
  std::string y_delim = ",";
  std::string feat_delim = ",";
  std::string kv_delim = ":";
  std::string field_delim = "@";
  bool feature_hash = false;       // FeatureHash.line2Map (J/feature/FeatureHash.java:94-116)
  int64_t hash_bucket = 1000000;
  uint32_t hash_seed = 39916801u;
  std::string hash_prefix = "hash_";
  bool split_field = false;        // FFM: field = name prefix before field_delim
  int64_t max_error_tol = 0;       // errors beyond this abort the parse
  std::vector<float> y_sampling;   // keep-rate per integer label (empty: off)
  uint64_t sample_seed = 0;
  int64_t line_mod = 1;            // "lines_avg" sharding: keep lines with idx % mod == rem
  int64_t line_rem = 0;
  bool want_stats = false;         // per-feature (sum, sum2, max, min) for transforms
  int threads = 0;                 // 0 = hardware concurrency
};

struct ParseResult {
  int64_t n_lines = 0;   // non-blank lines seen (after sharding)
  int64_t n_rows = 0;    // rows kept
  int64_t n_errors = 0;
  int64_t n_sampled_out = 0;
  std::vector<float> weight;
  std::vector<int64_t> row_line;   // source line index (0-based, all lines counted) per row
  std::vector<int64_t> label_ptr;  // [n_rows + 1]
  std::vector<float> labels;
  std::vector<int64_t> init_ptr;   // [n_rows + 1] (4th field; empty ranges when absent)
  std::vector<float> init;
  std::vector<int64_t> indptr;     // [n_rows + 1]
  std::vector<int32_t> feat;       // local dictionary ids (first-appearance order)
  std::vector<float> val;
  std::vector<int32_t> field;      // local field ids (split_field only)
  std::vector<std::string> names;  // local dictionary
  std::vector<int64_t> counts;     // rows containing each name
  std::vector<double> st_sum, st_sum2, st_max, st_min;  // want_stats only
  std::vector<std::string> fields;
  std::vector<std::string> error_samples;  // first few malformed lines (for messages)
};

// Threads for host work: OMP_NUM_THREADS if set, else the CPU affinity count.
int default_threads();

// CSR rows (local feature ids) -> dense row-major float32 [n_rows, F], NaN where absent;
// column = lut[local id] (-1 drops the feature). Multithreaded over row blocks.
void csr_to_dense(const int64_t* indptr, const int32_t* feat, const float* val, int64_t n_rows, const int64_t* lut,
                  int64_t n_lut, int64_t F, float* out, int threads);

// Parse a whole buffer (e.g. file contents or transformed lines joined by '\n').
ParseResult parse_ytk(const char* data, size_t len, const ParseOptions& opt);

// Read and parse several files in order (line indices are global over the list).
ParseResult parse_ytk_files(const std::vector<std::string>& paths, const ParseOptions& opt);

}  // namespace ytk_native
