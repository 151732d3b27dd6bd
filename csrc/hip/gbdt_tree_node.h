// Tree node record shared by the GPU-resident tree builders (gbdt_level.hip level-wise,
// gbdt_leafwise.hip leaf-wise) and read on the host as DNODE_DTYPE
// (ytk_learn_amd/models/gbdt/device_builder.py): one definition, layout static_assert'ed.
#pragma once

namespace ytk {

struct DNode {
  double G, H;           // node sums
  double gl, hl;         // best split: left sums
  long long cnt_global;  // rows in the node (all ranks)
  int begin, cnt_local;  // this rank's segment of the row permutation
  int depth, slot;
  int feat, bin_a, bin_b;
  int left, right;
  float loss_chg;
  float value;           // leaf value (x learning rate)
  int is_leaf;           // 1 leaf, 0 internal
};
static_assert(sizeof(DNode) == 88, "DNode layout (DNODE_DTYPE on the host)");

__device__ __forceinline__ double thr_l1d(double w, double lam) {
  if (w > lam) return w - lam;
  if (w < -lam) return w + lam;
  return 0.0;
}

// UpdateStrategy.java:83-100 nodeValue, then (float) value * learning_rate
__device__ __forceinline__ float node_leaf_value(double g, double h, float mcw, float l1, float l2,
                                                 float max_abs_leaf, float lr) {
  double v = 0.0;
  if (h >= (double)mcw) {
    v = (l1 == 0.f) ? -g / (h + l2) : -thr_l1d(g, l1) / (h + l2);
    if (max_abs_leaf > 0.f) {
      if (v > max_abs_leaf) v = max_abs_leaf;
      else if (v < -max_abs_leaf) v = -max_abs_leaf;
    }
  }
  return (float)v * lr;
}

}  // namespace ytk
