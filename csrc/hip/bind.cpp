// pybind11 bindings for the HIP kernel launchers. Pointers travel as integers
// (tensor.data_ptr()), streams as the raw hipStream_t of the current torch stream.
// Shape/dtype/device validation happens in ytk_learn_amd/ops/*.py before any call.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

extern "C" {
// gbdt_hist.hip
void ytk_hist_fx(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int,
                 float, float, uintptr_t, uintptr_t, uintptr_t);
void ytk_hist_fx_staged(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t,
                        int, float, float, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, uintptr_t,
                        uintptr_t, int, uintptr_t, int);
void ytk_hist_fx_global(uintptr_t, int, long long, int, uintptr_t, uintptr_t, uintptr_t, int,
                        uintptr_t, int, float, float, uintptr_t);
void ytk_hist_set_fw(int);
int ytk_hist_get_fw();
int ytk_hist_wide(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int, float,
                  float, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
int ytk_hist_wide_group(int, int);
int ytk_hist_wide_rm(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int, float, float,
                     uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, long long, uintptr_t);
// gbdt_split.hip
void ytk_split_find(uintptr_t, int, int, uintptr_t, uintptr_t, int, uintptr_t, int, uintptr_t,
                    float, float, float, float, double, double, uintptr_t, uintptr_t, uintptr_t,
                    uintptr_t, uintptr_t);
void ytk_split_combine(uintptr_t, int, int, uintptr_t, int, int, uintptr_t, uintptr_t);
// gbst.hip
int ytk_gbst_wide_max();
void ytk_gbst_epilogue(uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, double, uintptr_t, int, int, int,
                       int, int, double, int, int, int, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
// gbdt_partition.hip
void ytk_partition_atomic(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                          uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                          int, uintptr_t, uintptr_t);
void ytk_segment_copy(uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_zero_slots(uintptr_t, long long, uintptr_t, int, uintptr_t);
void ytk_memset_async(uintptr_t, int, long long, uintptr_t);
void ytk_partition(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                   uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                   uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_partition_count(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, int,
                         uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
// gbdt_score.hip
void ytk_tree_add_bins(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                       uintptr_t, int, uintptr_t, int, int, uintptr_t);
int ytk_forest_loss_regs(uintptr_t, long long, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                         uintptr_t, int, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, float, float,
                         uintptr_t, uintptr_t, int, uintptr_t);
void ytk_acc_finish(uintptr_t, int, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t);
int ytk_forest_predict_regs(uintptr_t, long long, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                            uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, int, float, uintptr_t, uintptr_t);
void ytk_forest_predict(uintptr_t, long long, long long, uintptr_t, uintptr_t, uintptr_t,
                        uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int,
                        float, uintptr_t, uintptr_t);
void ytk_bin_assign(uintptr_t, long long, long long, int, uintptr_t, uintptr_t, uintptr_t, int,
                    long long, uintptr_t, uintptr_t);
void ytk_grad_hess(uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, int, int, float, float,
                   uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t);
int ytk_tree_grad(uintptr_t, int, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                   uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, int,
                   float, float, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t,
                   uintptr_t);
int ytk_tree_grad_grid(long long);
// sparse.hip
void ytk_seg_spmm(uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, long long, int,
                  uintptr_t, long long, float, int, int, int, uintptr_t, uintptr_t);
void ytk_chunk_reduce(uintptr_t, int, uintptr_t, int, uintptr_t, long long, float, int, uintptr_t, uintptr_t, int,
                      uintptr_t);
void ytk_fixed_spmv(uintptr_t, uintptr_t, long long, int, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, float, int, int,
                    uintptr_t);
void ytk_seg_tile_spmv(uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, float, int,
                       int, uintptr_t);
// ffm.hip
void ytk_ffm_pairs(uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, uintptr_t, int, int,
                   uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, uintptr_t);
void ytk_ffm_grad_csc(uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                      uintptr_t, int, uintptr_t, uintptr_t, long long, int, int, uintptr_t, uintptr_t,
                      int, int, uintptr_t);
void ytk_ffm_sgd_grad(uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                      uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, long long, int, uintptr_t);
void ytk_ffm_pairs_lds(uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, uintptr_t, int, uintptr_t, int, int,
                       uintptr_t, long long, int, uintptr_t);
void ytk_ffm_pairs_fwd_e(uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, uintptr_t, int, uintptr_t, int,
                         uintptr_t, long long, int, uintptr_t);
void ytk_ffm_sgd_ecol(uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                      uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, float,
                      float, float, int, int, int, int, uintptr_t, uintptr_t);
void ytk_ffm_grad_stream(uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                         long long, uintptr_t, int, uintptr_t, long long, int, int, uintptr_t, uintptr_t);
// fm.hip
void ytk_fm_sgd_update(uintptr_t, uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, int, uintptr_t,
                       uintptr_t, float, float, float, int, int, int, uintptr_t, uintptr_t, uintptr_t);
void ytk_sgd_count(uintptr_t, uintptr_t, long long, long long, uintptr_t, int, uintptr_t);
void ytk_sgd_apply(uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int, uintptr_t, int, uintptr_t, uintptr_t, int,
                   uintptr_t, uintptr_t, long long, float, float, float, int, int, int, int, uintptr_t);
void ytk_fm_forward(uintptr_t, uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, int, uintptr_t,
                    uintptr_t, int, uintptr_t);
void ytk_fm_backward(uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int,
                     uintptr_t, uintptr_t);
// blas.hip
void ytk_dot(uintptr_t, uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t);
void ytk_row_loss(int, uintptr_t, int, uintptr_t, uintptr_t, long long, uintptr_t, long long, uintptr_t, uintptr_t,
                  uintptr_t, uintptr_t, uintptr_t);
void ytk_axpy_dot(uintptr_t, uintptr_t, float, float, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t);
void ytk_mc_row_loss(int, uintptr_t, int, uintptr_t, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, int,
                     uintptr_t, uintptr_t);
// gbdt_level.hip
void ytk_lv_step(int, const uintptr_t*, const int*, const float*, int, int, uintptr_t);
void ytk_lv_raw_tree(const uintptr_t*, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t,
                     uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_lv_scales(uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_lv_init_scales(const uintptr_t*, const int*, const float*, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_lv_tail(const uintptr_t*, const int*, const float*, int, int, int, int, uintptr_t, uintptr_t, uintptr_t, int,
                 uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t);
void ytk_hist_fx_stage(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, uintptr_t,
                       uintptr_t, uintptr_t, int);
void ytk_lv_reduce_split(const uintptr_t*, uintptr_t, uintptr_t, int, int, int, int, uintptr_t, uintptr_t, int,
                         const float*, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, int);
void ytk_lv_split_plan(const uintptr_t*, const int*, const float*, uintptr_t, int, int, uintptr_t, uintptr_t, int, int,
                       const float*, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t);
int ytk_split_node_grouped(uintptr_t, int, int, uintptr_t, uintptr_t, int, uintptr_t, int, uintptr_t, float, float,
                           float, float, uintptr_t, uintptr_t, int, uintptr_t);
void ytk_lv_partition_children(const uintptr_t*, const int*, const float*, uintptr_t, long long, uintptr_t, uintptr_t,
                               uintptr_t, uintptr_t, int, int, int, int, int, uintptr_t, int, int, uintptr_t);
// gbdt_leafwise.hip
int ytk_lw_create(const uintptr_t*, const int*, const float*);
void ytk_lw_set_lr(int, float);
void ytk_lw_set_batch_cap(int, int);
long long ytk_lw_ws_bytes(int, int);
uintptr_t ytk_host_device_ptr(uintptr_t);
void ytk_lw_step(int, int, uintptr_t);
void ytk_lw_partition(int, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t,
                      uintptr_t);
void ytk_lw_zero_slots(uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t);
void ytk_lw_subtree(int, uintptr_t, long long, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                    uintptr_t, uintptr_t, int, int, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t);
// gbdt_comm.hip
void ytk_seg_median(uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, int, int, uintptr_t, uintptr_t);
void ytk_seg_prune(uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, int, uintptr_t, uintptr_t);
int ytk_tree_grad_hist(uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t,
                       uintptr_t, uintptr_t, uintptr_t, uintptr_t, long long, int, float, float, uintptr_t, uintptr_t, uintptr_t,
                       uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, int,
                       uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, long long, uintptr_t);
void ytk_copy_to_mapped(uintptr_t, uintptr_t, long long, uintptr_t);
int ytk_tree_grad_hist_grid(long long);
void ytk_hist_reduce(uintptr_t, uintptr_t, int, uintptr_t, int, int, int, int, uintptr_t);
void ytk_hist_wide_staged_dev(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t,
                              int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t);
void ytk_lw_msg(int, uintptr_t, long long, uintptr_t, int, int, uintptr_t);
int ytk_peer_create(int, int, long long, uintptr_t);
int ytk_ex_create(const uintptr_t*, const long long*, const float*);
void ytk_ex_tree(int, uintptr_t, uintptr_t, int, int, int, double, double, int, float, uintptr_t);
int ytk_ex_tile();
void ytk_peer_open(int, uintptr_t);
void ytk_peer_allreduce(int, uintptr_t, long long, int, double, uintptr_t);
void ytk_peer_reduce_scatter(int, uintptr_t, long long, int, double, uintptr_t);
void ytk_peer_allgather(int, uintptr_t, long long, int, double, uintptr_t, uintptr_t);
void ytk_peer_reduce_scatter_dev(int, uintptr_t, long long, uintptr_t, uintptr_t, int, uintptr_t, double, uintptr_t);
void ytk_lw_owner(int, uintptr_t, long long, int, int, int, int, int, uintptr_t, int, int, uintptr_t);
void ytk_peer_allreduce_slots(int, uintptr_t, long long, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t,
                              double, uintptr_t);
int ytk_peer_check(int);
long long ytk_peer_epoch(int);
void ytk_peer_abort(int);
void ytk_peer_set_grid_cap(int, int);
void ytk_peer_timing(int, uintptr_t);
void ytk_peer_destroy(int);
void ytk_owner_pack(uintptr_t, uintptr_t, int, int, int, int, int, uintptr_t, int, uintptr_t);
void ytk_owner_unpack(uintptr_t, uintptr_t, int, int, int, int, int, uintptr_t, int, uintptr_t);
// gbdt_hist.hip (device-driven staged histogram)
void ytk_hist_fx_staged_dev(uintptr_t, long long, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t,
                            int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, int);
}

namespace py = pybind11;

PYBIND11_MODULE(_ytk_hip, m) {
  m.doc() = "ytk-learn-amd HIP kernels (gfx950)";
  m.def("hist_fx", &ytk_hist_fx);
  m.def("hist_fx_global", &ytk_hist_fx_global);
  m.def("hist_fx_staged", [](uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows, uintptr_t work,
                             int nwork, uintptr_t hist, int B, float sg, float sh, uintptr_t nwork_dev,
                             uintptr_t scales_dev, uintptr_t staging, int slot_base, int nslots, uintptr_t slot_ids,
                             uintptr_t work_off_dev, uintptr_t stream, int gh_rows, uintptr_t slot_first,
                             int one_slot) {
    ytk_hist_fx_staged(bins, stride, F, ghp, rows, work, nwork, hist, B, sg, sh, nwork_dev, scales_dev, staging,
                       slot_base, nslots, slot_ids, work_off_dev, stream, gh_rows, slot_first, one_slot);
  }, pybind11::arg("bins"), pybind11::arg("stride"), pybind11::arg("F"), pybind11::arg("ghp"), pybind11::arg("rows"),
     pybind11::arg("work"), pybind11::arg("nwork"), pybind11::arg("hist"), pybind11::arg("B"), pybind11::arg("sg"),
     pybind11::arg("sh"), pybind11::arg("nwork_dev"), pybind11::arg("scales_dev"), pybind11::arg("staging"),
     pybind11::arg("slot_base"), pybind11::arg("nslots"), pybind11::arg("slot_ids"), pybind11::arg("work_off_dev"),
     pybind11::arg("stream"), pybind11::arg("gh_rows") = 0, pybind11::arg("slot_first") = 0,
     pybind11::arg("one_slot") = 0);
  m.def("hist_wide", &ytk_hist_wide);
  m.def("hist_set_fw", &ytk_hist_set_fw);
  m.def("hist_get_fw", &ytk_hist_get_fw);
  m.def("hist_wide_group", &ytk_hist_wide_group);
  m.def("hist_wide_rm", &ytk_hist_wide_rm);
  m.def("split_find", &ytk_split_find);
  m.def("split_combine", &ytk_split_combine);
  m.def("gbst_epilogue", &ytk_gbst_epilogue);
  m.def("gbst_wide_max", &ytk_gbst_wide_max);
  m.def("partition", &ytk_partition);
  m.def("partition_count", &ytk_partition_count);
  m.def("segment_copy", &ytk_segment_copy);
  m.def("zero_slots", &ytk_zero_slots);
  m.def("memset_async", &ytk_memset_async);
  m.def("partition_atomic", &ytk_partition_atomic);
  m.def("tree_add_bins", &ytk_tree_add_bins);
  m.def("forest_predict", &ytk_forest_predict);
  m.def("forest_predict_regs", &ytk_forest_predict_regs);
  m.def("forest_loss_regs", &ytk_forest_loss_regs);
  m.def("acc_finish", &ytk_acc_finish);
  m.def("bin_assign", &ytk_bin_assign);
  m.def("grad_hess", &ytk_grad_hess);
  m.def("tree_grad", &ytk_tree_grad);
  m.def("tree_grad_grid", &ytk_tree_grad_grid);
  m.def("seg_spmm", &ytk_seg_spmm);
  m.def("chunk_reduce", [](uintptr_t cbeg, int ncol, uintptr_t part, int J, uintptr_t out, long long ldo, float alpha,
                           int accumulate, uintptr_t ids, uintptr_t stream, uintptr_t heavy, int nheavy) {
    ytk_chunk_reduce(cbeg, ncol, part, J, out, ldo, alpha, accumulate, ids, heavy, nheavy, stream);
  }, pybind11::arg("cbeg"), pybind11::arg("ncol"), pybind11::arg("part"), pybind11::arg("J"), pybind11::arg("out"),
     pybind11::arg("ldo"), pybind11::arg("alpha"), pybind11::arg("accumulate"), pybind11::arg("ids"),
     pybind11::arg("stream"), pybind11::arg("heavy") = 0, pybind11::arg("nheavy") = 0);
  m.def("seg_tile_spmv", &ytk_seg_tile_spmv);
  m.def("fixed_spmv", &ytk_fixed_spmv);
  m.def("ffm_pairs", &ytk_ffm_pairs);
  m.def("ffm_grad_csc", &ytk_ffm_grad_csc);
  m.def("ffm_sgd_grad", &ytk_ffm_sgd_grad);
  m.def("ffm_pairs_fwd_e", &ytk_ffm_pairs_fwd_e);
  m.def("ffm_pairs_lds", &ytk_ffm_pairs_lds);
  m.def("ffm_sgd_ecol", &ytk_ffm_sgd_ecol);
  m.def("ffm_grad_stream", &ytk_ffm_grad_stream);
  m.def("dot", &ytk_dot);
  m.def("row_loss", &ytk_row_loss);
  m.def("axpy_dot", &ytk_axpy_dot);
  m.def("mc_row_loss", &ytk_mc_row_loss);
  m.def("fm_forward", &ytk_fm_forward);
  m.def("fm_backward", &ytk_fm_backward);
  m.def("fm_sgd_update", &ytk_fm_sgd_update);
  m.def("sgd_count", &ytk_sgd_count);
  m.def("sgd_apply", &ytk_sgd_apply);
  m.def("lv_step", [](int which, const std::vector<uintptr_t>& ptrs, const std::vector<int>& ip,
                      const std::vector<float>& fp, int a0, int a1, uintptr_t stream) {
    if (ptrs.size() != 27 || ip.size() != 9 || fp.size() != 6)
      throw std::invalid_argument("lv_step: bad argument sizes");
    ytk_lv_step(which, ptrs.data(), ip.data(), fp.data(), a0, a1, stream);
  });
  m.def("lv_raw_tree", [](const std::vector<uintptr_t>& ptrs, int max_nodes, uintptr_t cand,
                          uintptr_t coff, uintptr_t fill, int split_median, uintptr_t nfeat,
                          uintptr_t nthr, uintptr_t nleft, uintptr_t nright, uintptr_t ndefl,
                          uintptr_t nval, uintptr_t stream) {
    if (ptrs.size() != 27) throw std::invalid_argument("lv_raw_tree: bad ptrs");
    ytk_lv_raw_tree(ptrs.data(), max_nodes, cand, coff, fill, split_median, nfeat, nthr, nleft,
                    nright, ndefl, nval, stream);
  });
  m.def("lv_scales", &ytk_lv_scales);
  m.def("lv_init_scales", [](const std::vector<uintptr_t>& ptrs, const std::vector<int>& ip,
                             const std::vector<float>& fp, uintptr_t mx, uintptr_t scales, uintptr_t inv,
                             uintptr_t stream) {
    if (ptrs.size() != 27 || ip.size() < 9 || fp.size() < 6) throw std::invalid_argument("lv_init_scales: bad sizes");
    ytk_lv_init_scales(ptrs.data(), ip.data(), fp.data(), mx, scales, inv, stream);
  });
  m.def("lv_tail", [](const std::vector<uintptr_t>& ptrs, const std::vector<int>& ip, const std::vector<float>& fp,
                      int children, int a0, int a1, int max_nodes, uintptr_t cand, uintptr_t coff, uintptr_t fill,
                      int median, uintptr_t nfeat, uintptr_t nthr, uintptr_t nleft, uintptr_t nright, uintptr_t ndefl,
                      uintptr_t nval, uintptr_t stream) {
    if (ptrs.size() != 27 || ip.size() < 9 || fp.size() < 6) throw std::invalid_argument("lv_tail: bad sizes");
    ytk_lv_tail(ptrs.data(), ip.data(), fp.data(), children, a0, a1, max_nodes, cand, coff, fill, median, nfeat, nthr,
                nleft, nright, ndefl, nval, stream);
  });
  m.def("lv_partition_children", [](const std::vector<uintptr_t>& ptrs, const std::vector<int>& ip,
                                     const std::vector<float>& fp, uintptr_t binsT, long long ncol, uintptr_t rows,
                                     uintptr_t ghp, uintptr_t rows_out, uintptr_t gh_out, int max_blocks,
                                     int count_only, int a0, int a1, int maxp, uintptr_t stream, int bin_bytes,
                                     int gh_rows, uintptr_t chunk_io) {
    if (ptrs.size() != 27 || ip.size() != 9 || fp.size() != 6)
      throw std::invalid_argument("lv_partition_children: bad argument sizes");
    ytk_lv_partition_children(ptrs.data(), ip.data(), fp.data(), binsT, ncol, rows, ghp, rows_out, gh_out,
                              max_blocks, count_only, a0, a1, maxp, stream, bin_bytes, gh_rows, chunk_io);
  }, pybind11::arg("ptrs"), pybind11::arg("ip"), pybind11::arg("fp"), pybind11::arg("binsT"), pybind11::arg("ncol"),
     pybind11::arg("rows"), pybind11::arg("ghp"), pybind11::arg("rows_out"), pybind11::arg("gh_out"),
     pybind11::arg("max_blocks"), pybind11::arg("count_only"), pybind11::arg("a0"), pybind11::arg("a1"),
     pybind11::arg("maxp"), pybind11::arg("stream"), pybind11::arg("bin_bytes") = 1, pybind11::arg("gh_rows") = 0,
     pybind11::arg("chunk_io") = 0);
  m.def("split_node_grouped", &ytk_split_node_grouped);
  m.def("hist_fx_stage", &ytk_hist_fx_stage);
  m.def("lv_reduce_split", [](const std::vector<uintptr_t>& ptrs, uintptr_t staging, uintptr_t hist, int B, int F,
                                int slot_base, int nslots, uintptr_t nbins_f, uintptr_t fmask, int f0,
                                const std::vector<float>& gpf, uintptr_t inv_dev, uintptr_t counters, int zs,
                                uintptr_t stream, uintptr_t prof, int group) {
    if (ptrs.size() != 27 || gpf.size() != 4) throw std::invalid_argument("lv_reduce_split: bad argument sizes");
    ytk_lv_reduce_split(ptrs.data(), staging, hist, B, F, slot_base, nslots, nbins_f, fmask, f0, gpf.data(), inv_dev,
                        counters, zs, stream, prof, group);
  });
  m.def("lv_split_plan", [](const std::vector<uintptr_t>& ptrs, const std::vector<int>& ip,
                              const std::vector<float>& fp, uintptr_t hist, int B, int F, uintptr_t nbins_f,
                              uintptr_t fmask, int f0, int nitems, const std::vector<float>& gpf, uintptr_t inv_dev,
                              uintptr_t part, uintptr_t counters, int implicit_items, int maxp, uintptr_t stream) {
    if (ptrs.size() != 27 || ip.size() != 9 || fp.size() != 6 || gpf.size() != 4)
      throw std::invalid_argument("lv_split_plan: bad argument sizes");
    ytk_lv_split_plan(ptrs.data(), ip.data(), fp.data(), hist, B, F, nbins_f, fmask, f0, nitems, gpf.data(), inv_dev,
                      part, counters, implicit_items, maxp, stream);
  });
  m.def("lw_create", [](const std::vector<uintptr_t>& ptrs, const std::vector<int>& ip, const std::vector<float>& fp) {
    if (ptrs.size() != 40 || ip.size() != 13 || fp.size() != 7) throw std::invalid_argument("lw_create: bad argument sizes");
    return ytk_lw_create(ptrs.data(), ip.data(), fp.data());
  });
  m.def("lw_set_lr", &ytk_lw_set_lr);
  m.def("lw_set_batch_cap", &ytk_lw_set_batch_cap);
  m.def("lw_ws_bytes", &ytk_lw_ws_bytes);
  m.def("host_device_ptr", &ytk_host_device_ptr);
  m.def("lw_step", &ytk_lw_step);
  m.def("lw_partition", &ytk_lw_partition, pybind11::arg("h"), pybind11::arg("binsT"), pybind11::arg("ncol"),
        pybind11::arg("rows"), pybind11::arg("ghp"), pybind11::arg("rows_out"), pybind11::arg("gh_out"),
        pybind11::arg("max_blocks"), pybind11::arg("stream"), pybind11::arg("chunk_io") = 0);
  m.def("lw_zero_slots", &ytk_lw_zero_slots);
  m.def("lw_subtree", &ytk_lw_subtree);
  m.def("hist_fx_staged_dev", &ytk_hist_fx_staged_dev);
  m.def("owner_pack", &ytk_owner_pack);
  m.def("peer_create", &ytk_peer_create);
  m.def("ex_create", [](std::vector<uintptr_t> p, std::vector<long long> ip, std::vector<float> fp) {
    if (p.size() != 30 || ip.size() != 7 || fp.size() != 6) throw std::invalid_argument("ex_create: bad arity");
    return ytk_ex_create(p.data(), ip.data(), fp.data());
  });
  m.def("ex_tree", &ytk_ex_tree);
  m.def("ex_tile", &ytk_ex_tile);
  m.def("peer_open", &ytk_peer_open);
  m.def("peer_allreduce", &ytk_peer_allreduce);
  m.def("peer_reduce_scatter", &ytk_peer_reduce_scatter);
  m.def("peer_allgather", &ytk_peer_allgather);
  m.def("peer_reduce_scatter_dev", &ytk_peer_reduce_scatter_dev);
  m.def("lw_owner", &ytk_lw_owner);
  m.def("peer_allreduce_slots", &ytk_peer_allreduce_slots);
  m.def("peer_check", &ytk_peer_check);
  m.def("peer_epoch", &ytk_peer_epoch);
  m.def("peer_abort", &ytk_peer_abort);
  m.def("peer_timing", &ytk_peer_timing);
  m.def("peer_set_grid_cap", &ytk_peer_set_grid_cap);
  m.def("peer_destroy", &ytk_peer_destroy);
  m.def("lw_msg", &ytk_lw_msg);
  m.def("hist_wide_staged_dev", &ytk_hist_wide_staged_dev);
  m.def("tree_grad_hist", &ytk_tree_grad_hist);
  m.def("copy_to_mapped", &ytk_copy_to_mapped);
  m.def("tree_grad_hist_grid", &ytk_tree_grad_hist_grid);
  m.def("hist_reduce", &ytk_hist_reduce);
  m.def("seg_median", &ytk_seg_median);
  m.def("seg_prune", &ytk_seg_prune);
  m.def("owner_unpack", &ytk_owner_unpack);
  m.attr("arch") = "gfx950";
}
