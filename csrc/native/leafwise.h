// Exact leaf-wise (loss-guided) tree growth planner: the host side of the GBDT
// builder's speculative batches, in native code.
//
// Reference order: DataParallelTreeMaker.java make() :229-295 with the priority queue
// ordered by lossChg (:104-115,219-225), pop-time leaf rules (:249-253), children made
// leaves right away (:266-273), smaller-child histogram + subtraction and the LRU
// histogram pool (:489-508, HistogramPool.java:36-273).
//
// The device work (partition, histograms, split search, collectives) stays with the
// Python driver; this class owns every per-node decision between two device round
// trips: the replay of the priority queue from the known gains, the choice of the
// speculative batch (a virtual continuation of the replay), child bookkeeping, the
// small/large child choice, histogram slot recycling with LRU eviction, and the tree
// under construction. Semantics are those of TreeBuilder._grow_loss_guided
// (ytk_learn_amd/models/gbdt/builder.py), which stays as the reference implementation.
#pragma once
#include <cstdint>
#include <queue>
#include <vector>

namespace ytk_native {

struct LwParams {
  int max_leaf = 255;          // max_leaf_cnt (<= 0: unlimited)
  int max_depth = -1;          // < 0: unlimited
  int64_t min_split_samples = -1;
  double min_split_loss = 0;   // float32-rounded, as the kernels compare
  double mcw = 0, l1 = 0, l2 = 0, max_abs_leaf = -1;  // float32-rounded gain params
  double mcw2 = 0;             // 2 * min_child_hessian_sum (canSplit, full precision)
  float lr = 0.1f;
  bool speculate = true;
};

// one split-search result (layout of SplitOut in csrc/hip/gbdt_split_node.h)
struct LwRec {
  float loss_chg;
  int32_t feat, bin_a, bin_b;
  double gl, hl, g, h;
};
static_assert(sizeof(LwRec) == 48, "LwRec layout");

class LeafGrower {
 public:
  LeafGrower(const LwParams& p, int n_slots);

  // root: node 0 holds (n_local, n_global) rows; returns its histogram slot
  int root(int64_t n_local, int64_t n_global);
  // split results of nodes `ids` (canSplit applied here)
  void apply_recs(const int32_t* ids, const LwRec* recs, int n);
  // replay the queue; returns the next expansion batch (empty: the tree is complete)
  std::vector<int32_t> replay();
  // children ids for the batch; splits (need rows) and counts_only (children at
  // max_depth) parents, each with the parent segment and the split
  struct Expand {
    std::vector<int32_t> split_sid, count_sid;
  };
  Expand expand(const std::vector<int32_t>& batch);
  // per-parent left row counts (local, global) -> child nodes
  void set_children(const std::vector<int32_t>& parents, const int64_t* lloc, const int64_t* lglob,
                    bool with_begin);
  // histogram plan for the split parents: builds (small child; large too on a pool
  // miss) and derivations; slots allocated with LRU eviction
  struct HistPlan {
    std::vector<int32_t> order;    // build sids then derived sids (split-item order)
    std::vector<int32_t> slots;    // slot per order entry
    std::vector<int64_t> begin, count;  // segments of the build nodes
    std::vector<int32_t> items;    // (slot, parent_slot, sibling_slot, derived) per order entry
    int nbuild = 0;
  };
  HistPlan plan_hist(const std::vector<int32_t>& split_parents);

  // Launch-ready int32 packs for the device steps (one pinned upload each). Chunking:
  // ch = max(min_rows, ceil(rows / target_blocks)) rows per item, as TreeBuilder._chunk.
  // partition: [items (split, b, e, k) x nitems | feat | thr | begin | count | first_blk
  //   (exclusive scan of ceil(count / part_chunk)) | hdr (n, nblocks)]
  struct Pack {
    std::vector<int32_t> data;
    std::vector<int64_t> off;  // section offsets (int32 elements)
    int64_t n_items = 0, n_blocks = 0;
  };
  Pack pack_partition(const std::vector<int32_t>& parents, int part_chunk, int target_blocks,
                      int min_rows) const;
  // histogram step of `hp`: [work (slot, b, e, 0) x nwork | items x norder | build slots]
  static Pack pack_hist(const HistPlan& hp, int target_blocks, int min_rows);
  void release_batch(const std::vector<int32_t>& batch);

  // node accessors for the driver
  int64_t begin(int sid) const { return nodes_[sid].begin; }
  int64_t cnt_local(int sid) const { return nodes_[sid].cnt_local; }
  int feat(int sid) const { return nodes_[sid].feat; }
  int thr(int sid) const { return (nodes_[sid].bin_a + nodes_[sid].bin_b) >> 1; }

  // finished tree (after replay() returned empty); stats written per tree node
  struct TreeOut {
    std::vector<int32_t> left, right, parent, feat, slot_a, slot_b;
    std::vector<double> cond;
    std::vector<float> leaf, loss_chg, hess_sum;
    std::vector<uint8_t> is_leaf;
    std::vector<int64_t> sample_cnt;
  };
  TreeOut finish();

  int batches = 0, expanded = 0, hist_miss = 0;

 private:
  struct Node {
    int64_t begin = 0, cnt_local = 0, cnt_global = 0;
    int slot = -1, depth = 0, tid = -1;
    int64_t seq = 0;
    bool has_rec = false, rec_used = true;
    double loss_chg = 0;  // exact double of the float32 gain
    int feat = -1, bin_a = -1, bin_b = -1;
    double gl = 0, hl = 0, G = 0, H = 0;
    int lc = -1, rc = -1;  // children (speculative ids) once expanded
  };
  struct Entry {  // heap key (-loss_chg, seq, sid), smallest first
    double neg;
    int64_t seq;
    int sid;
    bool operator<(const Entry& o) const {  // std::priority_queue is a max-heap
      if (neg != o.neg) return neg > o.neg;
      if (seq != o.seq) return seq > o.seq;
      return sid > o.sid;
    }
  };
  bool pop_is_leaf(const Node& n, int num_leaf) const;
  bool children_terminal(const Node& l, const Node& r, int num_leaf) const;
  void make_leaf(int sid, int t);
  void leafify_children(int sid, int lc, int rc, int lt, int rt);
  void release(int sid);
  void evict(const std::vector<int>& keep);
  int tree_alloc(int parent);

  LwParams p_;
  std::vector<Node> nodes_;
  std::vector<int> free_slots_;  // back = next slot handed out
  std::vector<int> lru_;         // speculative ids holding a slot, oldest first
  std::priority_queue<Entry> heap_;
  bool started_ = false;
  int num_leaf_ = 1;
  int64_t seq_ = 1;
  TreeOut t_;
};

}  // namespace ytk_native
