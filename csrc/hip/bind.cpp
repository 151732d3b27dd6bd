// pybind11 bindings for the HIP kernel launchers. Pointers travel as integers
// (tensor.data_ptr()), streams as the raw hipStream_t of the current torch stream.
// Shape/dtype/device validation happens in ytk_learn_amd/ops/*.py before any call.
#include <pybind11/pybind11.h>

#include <cstdint>

extern "C" {
// gbdt_hist.hip
void ytk_hist_fx(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int,
                 float, float, uintptr_t);
void ytk_hist_fx_global(uintptr_t, int, long long, int, uintptr_t, uintptr_t, uintptr_t, int,
                        uintptr_t, int, float, float, uintptr_t);
// gbdt_split.hip
void ytk_split_find(uintptr_t, int, int, uintptr_t, uintptr_t, int, uintptr_t, int, uintptr_t,
                    float, float, float, float, double, double, uintptr_t);
// gbdt_partition.hip
void ytk_partition(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                   uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                   uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_partition_count(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, int,
                         uintptr_t, uintptr_t, uintptr_t, uintptr_t);
// gbdt_score.hip
void ytk_tree_add_bins(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                       uintptr_t, int, uintptr_t, int, int, uintptr_t);
void ytk_forest_predict(uintptr_t, long long, long long, uintptr_t, uintptr_t, uintptr_t,
                        uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int,
                        float, uintptr_t, uintptr_t);
void ytk_bin_assign(uintptr_t, long long, long long, int, uintptr_t, uintptr_t, uintptr_t, int,
                    long long, uintptr_t, uintptr_t);
void ytk_grad_hess(uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, int, int, float, float,
                   uintptr_t, uintptr_t, uintptr_t, int, uintptr_t);
void ytk_tree_grad(uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int,
                   uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, int, float, float,
                   uintptr_t, uintptr_t, uintptr_t, int, uintptr_t);
}

namespace py = pybind11;

PYBIND11_MODULE(_ytk_hip, m) {
  m.doc() = "ytk-learn-amd HIP kernels (gfx950)";
  m.def("hist_fx", &ytk_hist_fx);
  m.def("hist_fx_global", &ytk_hist_fx_global);
  m.def("split_find", &ytk_split_find);
  m.def("partition", &ytk_partition);
  m.def("partition_count", &ytk_partition_count);
  m.def("tree_add_bins", &ytk_tree_add_bins);
  m.def("forest_predict", &ytk_forest_predict);
  m.def("bin_assign", &ytk_bin_assign);
  m.def("grad_hess", &ytk_grad_hess);
  m.def("tree_grad", &ytk_tree_grad);
  m.attr("arch") = "gfx950";
}
