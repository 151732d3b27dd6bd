// pybind11 bindings of the host native runtime.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "native.h"
#include "leafwise.h"
#include "parser.h"

namespace py = pybind11;
using namespace ytk_native;

namespace {

// Hand a std::vector to numpy without copying (the capsule owns the heap vector).
template <typename T>
py::array_t<T> to_numpy(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}

ParseOptions options_from(const py::dict& d) {
  ParseOptions o;
  auto get_s = [&](const char* k, std::string& dst) {
    if (d.contains(k)) dst = d[k].cast<std::string>();
  };
  get_s("x_delim", o.x_delim);
  get_s("y_delim", o.y_delim);
  get_s("features_delim", o.feat_delim);
  get_s("feature_name_val_delim", o.kv_delim);
  get_s("field_delim", o.field_delim);
  get_s("hash_prefix", o.hash_prefix);
  if (d.contains("feature_hash")) o.feature_hash = d["feature_hash"].cast<bool>();
  if (d.contains("hash_bucket")) o.hash_bucket = d["hash_bucket"].cast<int64_t>();
  if (d.contains("hash_seed")) o.hash_seed = (uint32_t)d["hash_seed"].cast<int64_t>();
  if (d.contains("split_field")) o.split_field = d["split_field"].cast<bool>();
  if (d.contains("max_error_tol")) o.max_error_tol = d["max_error_tol"].cast<int64_t>();
  if (d.contains("y_sampling")) o.y_sampling = d["y_sampling"].cast<std::vector<float>>();
  if (d.contains("sample_seed")) o.sample_seed = d["sample_seed"].cast<uint64_t>();
  if (d.contains("line_mod")) o.line_mod = d["line_mod"].cast<int64_t>();
  if (d.contains("line_rem")) o.line_rem = d["line_rem"].cast<int64_t>();
  if (d.contains("want_stats")) o.want_stats = d["want_stats"].cast<bool>();
  if (d.contains("threads")) o.threads = d["threads"].cast<int>();
  return o;
}

py::dict result_to_dict(ParseResult&& r) {
  py::dict out;
  out["n_lines"] = r.n_lines;
  out["n_rows"] = r.n_rows;
  out["n_errors"] = r.n_errors;
  out["n_sampled_out"] = r.n_sampled_out;
  out["weight"] = to_numpy(std::move(r.weight));
  out["row_line"] = to_numpy(std::move(r.row_line));
  out["label_ptr"] = to_numpy(std::move(r.label_ptr));
  out["labels"] = to_numpy(std::move(r.labels));
  out["init_ptr"] = to_numpy(std::move(r.init_ptr));
  out["init"] = to_numpy(std::move(r.init));
  out["indptr"] = to_numpy(std::move(r.indptr));
  out["feat"] = to_numpy(std::move(r.feat));
  out["val"] = to_numpy(std::move(r.val));
  out["field"] = to_numpy(std::move(r.field));
  out["names"] = py::cast(r.names);
  out["counts"] = to_numpy(std::move(r.counts));
  out["st_sum"] = to_numpy(std::move(r.st_sum));
  out["st_sum2"] = to_numpy(std::move(r.st_sum2));
  out["st_max"] = to_numpy(std::move(r.st_max));
  out["st_min"] = to_numpy(std::move(r.st_min));
  out["fields"] = py::cast(r.fields);
  out["error_samples"] = py::cast(r.error_samples);
  return out;
}

WQSummary summary_from(const py::array_t<double, py::array::c_style | py::array::forcecast>& a) {
  WQSummary s;
  if (a.ndim() != 2 || (a.shape(0) > 0 && a.shape(1) != 4))
    throw std::invalid_argument("summary must be a [n, 4] float64 array (v, rmin, rmax, wmin)");
  auto r = a.unchecked<2>();
  s.e.resize((size_t)a.shape(0));
  for (py::ssize_t i = 0; i < a.shape(0); ++i) s.e[(size_t)i] = {r(i, 0), r(i, 1), r(i, 2), r(i, 3)};
  return s;
}

py::array_t<double> summary_to(const WQSummary& s) {
  py::array_t<double> out({(py::ssize_t)s.e.size(), (py::ssize_t)4});
  auto w = out.mutable_unchecked<2>();
  for (size_t i = 0; i < s.e.size(); ++i) {
    w((py::ssize_t)i, 0) = s.e[i].v;
    w((py::ssize_t)i, 1) = s.e[i].rmin;
    w((py::ssize_t)i, 2) = s.e[i].rmax;
    w((py::ssize_t)i, 3) = s.e[i].wmin;
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_ytk_native, m) {
  using darr = py::array_t<double, py::array::c_style | py::array::forcecast>;
  m.def(
      "wq_build",
      [](const darr& v, const darr& w, int64_t size) {
        // sort (value, weight) pairs, build the exact summary, prune to `size` entries
        const py::ssize_t n = v.size();
        if (w.size() != n) throw std::invalid_argument("values / weights length mismatch");
        std::vector<std::pair<double, double>> p((size_t)n);
        const double* pv = v.data();
        const double* pw = w.data();
        for (py::ssize_t i = 0; i < n; ++i) p[(size_t)i] = {pv[i], pw[i]};
        WQSummary s;
        {
          py::gil_scoped_release nogil;
          std::sort(p.begin(), p.end(),
                    [](const std::pair<double, double>& a, const std::pair<double, double>& b) {
                      return a.first < b.first;
                    });
          std::vector<double> sv(p.size()), sw(p.size());
          for (size_t i = 0; i < p.size(); ++i) { sv[i] = p[i].first; sw[i] = p[i].second; }
          s = WQSummary::from_sorted(sv.data(), sw.data(), sv.size());
          if (size > 0) s = s.prune((size_t)size);
        }
        return summary_to(s);
      },
      py::arg("values"), py::arg("weights"), py::arg("size") = 0);
  m.def(
      "csr_to_dense",
      [](const py::array_t<int64_t, py::array::c_style | py::array::forcecast>& indptr,
         const py::array_t<int32_t, py::array::c_style | py::array::forcecast>& feat,
         const py::array_t<float, py::array::c_style | py::array::forcecast>& val,
         const py::array_t<int64_t, py::array::c_style | py::array::forcecast>& lut, int64_t F, int threads) {
        const int64_t n = indptr.size() - 1;
        if (n < 0 || feat.size() != val.size() || (n > 0 && indptr.at(n) > feat.size()))
          throw std::invalid_argument("csr_to_dense: inconsistent CSR arrays");
        py::array_t<float> out({(py::ssize_t)std::max<int64_t>(n, 0), (py::ssize_t)F});
        if (n > 0) {
          const int64_t* ip = indptr.data();
          const int32_t* fp = feat.data();
          const float* vp = val.data();
          const int64_t* lp = lut.data();
          const int64_t nl = lut.size();
          float* op = out.mutable_data();
          py::gil_scoped_release nogil;
          csr_to_dense(ip, fp, vp, n, lp, nl, F, op, threads);
        }
        return out;
      },
      py::arg("indptr"), py::arg("feat"), py::arg("val"), py::arg("lut"), py::arg("F"), py::arg("threads") = 0);
  m.def("default_threads", &default_threads);
  m.def("wq_combine", [](const darr& a, const darr& b, int64_t size) {
    WQSummary s = WQSummary::combine(summary_from(a), summary_from(b));
    if (size > 0) s = s.prune((size_t)size);
    return summary_to(s);
  }, py::arg("a"), py::arg("b"), py::arg("size") = 0);
  m.def("wq_prune", [](const darr& a, int64_t size) { return summary_to(summary_from(a).prune((size_t)size)); });
  m.def("wq_query", [](const darr& a, const darr& ranks) {
    const WQSummary s = summary_from(a);
    py::array_t<double> out(ranks.size());
    auto o = out.mutable_unchecked<1>();
    const double* r = ranks.data();
    for (py::ssize_t i = 0; i < ranks.size(); ++i) o(i) = s.query(r[i]);
    return out;
  });
  m.doc() = "ytk-learn-amd native host runtime";
  m.def("murmur3_128_aslong", [](const std::string& s, uint32_t seed) {
    return murmur3_128_aslong(s.data(), s.size(), seed);
  });
  m.def("murmur3_128_aslong_many", [](const std::vector<std::string>& names, uint32_t seed) {
    py::array_t<int64_t> out(names.size());
    auto o = out.mutable_unchecked<1>();
    for (size_t i = 0; i < names.size(); ++i)
      o(i) = murmur3_128_aslong(names[i].data(), names[i].size(), seed);
    return out;
  });
  m.def(
      "java_random",
      [](int64_t seed, int64_t n, int mode, double a, double b) {
        std::vector<double> v;
        {
          py::gil_scoped_release nogil;
          v = java_random_fill(seed, n, mode, a, b);
        }
        return to_numpy(std::move(v));
      },
      py::arg("seed"), py::arg("n"), py::arg("mode"), py::arg("a") = 0.0, py::arg("b") = 1.0);
  m.def(
      "java_random_seq",
      [](int64_t seed, const std::vector<std::tuple<int, int64_t, double, double>>& segs) {
        // several draw segments from ONE java.util.Random stream (e.g. GBSDT: dim draws of
        // next(), then K leaf draws of nextUniform(range))
        std::vector<double> v;
        {
          py::gil_scoped_release nogil;
          JavaRandom r(seed);
          for (const auto& s : segs) {
            const int mode = std::get<0>(s);
            const double a = std::get<2>(s), b = std::get<3>(s);
            for (int64_t i = 0; i < std::get<1>(s); ++i) {
              double x;
              switch (mode) {
                case 0: x = r.next_gaussian() * b + a; break;
                case 1: x = a + (b - a) * r.next_double(); break;
                case 2: x = (double)r.next_float(); break;
                default: x = r.next_double(); break;
              }
              v.push_back(x);
            }
          }
        }
        return to_numpy(std::move(v));
      },
      py::arg("seed"), py::arg("segments"));
  m.def(
      "parse_buffer",
      [](py::bytes data, const py::dict& opts) {
        const ParseOptions o = options_from(opts);
        std::string_view s = data;  // keep the bytes object alive in this frame
        ParseResult r;
        {
          py::gil_scoped_release nogil;
          r = parse_ytk(s.data(), s.size(), o);
        }
        return result_to_dict(std::move(r));
      },
      py::arg("data"), py::arg("opts"));
  m.def(
      "parse_files",
      [](const std::vector<std::string>& paths, const py::dict& opts) {
        const ParseOptions o = options_from(opts);
        ParseResult r;
        {
          py::gil_scoped_release nogil;
          r = parse_ytk_files(paths, o);
        }
        return result_to_dict(std::move(r));
      },
      py::arg("paths"), py::arg("opts"));

  // ---- exact leaf-wise growth planner (leafwise.h)
  using i32arr = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
  using i64arr = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
  py::class_<LwParams>(m, "LwParams")
      .def(py::init<>())
      .def_readwrite("max_leaf", &LwParams::max_leaf)
      .def_readwrite("max_depth", &LwParams::max_depth)
      .def_readwrite("min_split_samples", &LwParams::min_split_samples)
      .def_readwrite("min_split_loss", &LwParams::min_split_loss)
      .def_readwrite("mcw", &LwParams::mcw)
      .def_readwrite("l1", &LwParams::l1)
      .def_readwrite("l2", &LwParams::l2)
      .def_readwrite("max_abs_leaf", &LwParams::max_abs_leaf)
      .def_readwrite("mcw2", &LwParams::mcw2)
      .def_readwrite("lr", &LwParams::lr)
      .def_readwrite("speculate", &LwParams::speculate);
  py::class_<LeafGrower>(m, "LeafGrower")
      .def(py::init<const LwParams&, int>())
      .def("root", &LeafGrower::root)
      .def("apply_recs",
           [](LeafGrower& g, const i32arr& ids, const py::array& recs) {
             if ((size_t)recs.nbytes() != (size_t)ids.size() * sizeof(LwRec))
               throw std::invalid_argument("apply_recs: recs must hold 48 bytes per id");
             g.apply_recs(ids.data(), reinterpret_cast<const LwRec*>(recs.data()), (int)ids.size());
           })
      .def("replay", &LeafGrower::replay)
      .def("expand",
           [](LeafGrower& g, const std::vector<int32_t>& batch) {
             auto ex = g.expand(batch);
             return py::make_tuple(ex.split_sid, ex.count_sid);
           })
      .def("segments",  // parents -> (begin, count, feat, thr) int64 arrays
           [](const LeafGrower& g, const std::vector<int32_t>& sids) {
             const py::ssize_t n = (py::ssize_t)sids.size();
             i64arr out({(py::ssize_t)4, n});
             auto w = out.mutable_unchecked<2>();
             for (py::ssize_t i = 0; i < n; ++i) {
               w(0, i) = g.begin(sids[i]);
               w(1, i) = g.cnt_local(sids[i]);
               w(2, i) = g.feat(sids[i]);
               w(3, i) = g.thr(sids[i]);
             }
             return out;
           })
      .def("set_children",
           [](LeafGrower& g, const std::vector<int32_t>& parents, const i64arr& lloc, const i64arr& lglob,
              bool with_begin) {
             if ((size_t)lloc.size() != parents.size() || (size_t)lglob.size() != parents.size())
               throw std::invalid_argument("set_children: size mismatch");
             g.set_children(parents, lloc.data(), lglob.data(), with_begin);
           })
      .def("plan_hist",
           [](LeafGrower& g, const std::vector<int32_t>& parents) {
             auto hp = g.plan_hist(parents);
             const py::ssize_t n = (py::ssize_t)hp.order.size();
             i32arr items({n, (py::ssize_t)4});
             std::copy(hp.items.begin(), hp.items.end(), items.mutable_data());
             return py::make_tuple(hp.order, hp.slots, hp.nbuild, i64arr((py::ssize_t)hp.begin.size(), hp.begin.data()),
                                   i64arr((py::ssize_t)hp.count.size(), hp.count.data()), items);
           })
      .def("pack_partition",
           [](const LeafGrower& g, const std::vector<int32_t>& parents, int part_chunk, int target_blocks,
              int min_rows) {
             auto pk = g.pack_partition(parents, part_chunk, target_blocks, min_rows);
             return py::make_tuple(i32arr((py::ssize_t)pk.data.size(), pk.data.data()), pk.off, pk.n_items,
                                   pk.n_blocks);
           })
      .def("plan_hist_packed",  // plan_hist + pack_hist: (order, nbuild, pack, offsets, nwork)
           [](LeafGrower& g, const std::vector<int32_t>& parents, int target_blocks, int min_rows) {
             auto hp = g.plan_hist(parents);
             auto pk = LeafGrower::pack_hist(hp, target_blocks, min_rows);
             return py::make_tuple(hp.order, hp.nbuild, i32arr((py::ssize_t)pk.data.size(), pk.data.data()),
                                   pk.off, pk.n_items);
           })
      .def("release_batch", &LeafGrower::release_batch)
      .def("finish",
           [](LeafGrower& g) {
             auto t = g.finish();
             py::dict d;
             d["left"] = t.left;
             d["right"] = t.right;
             d["parent"] = t.parent;
             d["feat"] = t.feat;
             d["slot_a"] = t.slot_a;
             d["slot_b"] = t.slot_b;
             d["cond"] = t.cond;
             d["leaf"] = std::vector<double>(t.leaf.begin(), t.leaf.end());
             d["is_leaf"] = std::vector<bool>(t.is_leaf.begin(), t.is_leaf.end());
             d["loss_chg"] = std::vector<double>(t.loss_chg.begin(), t.loss_chg.end());
             d["hess_sum"] = std::vector<double>(t.hess_sum.begin(), t.hess_sum.end());
             d["sample_cnt"] = t.sample_cnt;
             return d;
           })
      .def_readonly("batches", &LeafGrower::batches)
      .def_readonly("expanded", &LeafGrower::expanded)
      .def_readonly("hist_miss", &LeafGrower::hist_miss);
}
