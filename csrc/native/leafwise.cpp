// Exact leaf-wise growth planner (see leafwise.h).
#include "leafwise.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <limits>
#include <stdexcept>

namespace ytk_native {

namespace {

double thr_l1(double w, double lam) {
  if (w > lam) return w - lam;
  if (w < -lam) return w + lam;
  return 0.0;
}

// UpdateStrategy.java:83-100 (node_value_py in ytk_learn_amd/ops/gbdt.py)
double node_value(double g, double h, const LwParams& p) {
  if (h < p.mcw) return 0.0;
  double v = (p.l1 == 0.0) ? -g / (h + p.l2) : -thr_l1(g, p.l1) / (h + p.l2);
  if (p.max_abs_leaf > 0) v = std::min(std::max(v, -p.max_abs_leaf), p.max_abs_leaf);
  return v;
}

int64_t floor_div(int64_t a, int64_t b) {  // Python //
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

}  // namespace

LeafGrower::LeafGrower(const LwParams& p, int n_slots) : p_(p) {
  if (n_slots < 1) throw std::invalid_argument("LeafGrower: n_slots must be >= 1");
  free_slots_.reserve(n_slots);
  for (int s = n_slots - 1; s >= 0; --s) free_slots_.push_back(s);  // back() = 0 first
  nodes_.reserve(4 * std::max(p.max_leaf, 1) + 8);
  tree_alloc(-1);  // tree root
}

int LeafGrower::tree_alloc(int parent) {
  const int id = (int)t_.left.size();
  t_.left.push_back(-1);
  t_.right.push_back(-1);
  t_.parent.push_back(parent);
  t_.feat.push_back(-1);
  t_.slot_a.push_back(0);
  t_.slot_b.push_back(0);
  t_.cond.push_back(0.0);
  t_.leaf.push_back(0.f);
  t_.is_leaf.push_back(1);
  t_.loss_chg.push_back(0.f);
  t_.hess_sum.push_back(0.f);
  t_.sample_cnt.push_back(0);
  return id;
}

int LeafGrower::root(int64_t n_local, int64_t n_global) {
  if (!nodes_.empty()) throw std::logic_error("LeafGrower::root called twice");
  Node r;
  r.cnt_local = n_local;
  r.cnt_global = n_global;
  r.tid = 0;
  nodes_.push_back(r);
  const int sl = free_slots_.back();
  free_slots_.pop_back();
  lru_.push_back(0);
  nodes_[0].slot = sl;
  return sl;
}

void LeafGrower::apply_recs(const int32_t* ids, const LwRec* recs, int n) {
  for (int i = 0; i < n; ++i) {
    Node& nd = nodes_.at(ids[i]);
    const LwRec& r = recs[i];
    nd.has_rec = true;
    nd.loss_chg = (double)r.loss_chg;
    nd.feat = r.feat;
    nd.bin_a = r.bin_a;
    nd.bin_b = r.bin_b;
    nd.gl = r.gl;
    nd.hl = r.hl;
    nd.G = r.g;
    nd.H = r.h;
    // canSplit (UpdateStrategy.java:50-53): H >= 2 * mcw and n >= min_split_samples
    if (!(nd.H >= p_.mcw2 && nd.cnt_global >= p_.min_split_samples)) {
      nd.loss_chg = -std::numeric_limits<double>::infinity();
      nd.feat = -1;
    }
  }
}

bool LeafGrower::pop_is_leaf(const Node& n, int num_leaf) const {
  return n.loss_chg <= p_.min_split_loss || (p_.max_depth >= 0 && p_.max_depth == n.depth) ||
         (p_.max_leaf > 0 && p_.max_leaf == num_leaf) ||
         (p_.min_split_samples > 0 && n.cnt_global < p_.min_split_samples);
}

bool LeafGrower::children_terminal(const Node& l, const Node& r, int num_leaf) const {
  return (p_.max_depth >= 0 && p_.max_depth == l.depth) || (p_.max_leaf > 0 && p_.max_leaf == num_leaf) ||
         (p_.min_split_samples > 0 && l.cnt_global < p_.min_split_samples &&
          r.cnt_global < p_.min_split_samples);
}

void LeafGrower::make_leaf(int sid, int t) {
  const Node& nd = nodes_[sid];
  const float v = (float)node_value(nd.G, nd.H, p_);
  t_.is_leaf[t] = 1;
  t_.left[t] = -1;
  t_.right[t] = -1;
  t_.leaf[t] = v * p_.lr;  // float32 product, as np.float32 * np.float32
}

void LeafGrower::leafify_children(int sid, int lc, int rc, int lt, int rt) {
  const Node& P = nodes_[sid];
  Node& L = nodes_[lc];
  Node& R = nodes_[rc];
  L.G = P.gl;
  L.H = P.hl;
  R.G = P.G - L.G;
  R.H = P.H - L.H;
  make_leaf(lc, lt);
  make_leaf(rc, rt);
}

void LeafGrower::release(int sid) {
  Node& nd = nodes_[sid];
  if (nd.slot < 0) return;
  auto it = std::find(lru_.begin(), lru_.end(), sid);
  if (it != lru_.end()) lru_.erase(it);
  free_slots_.push_back(nd.slot);
  nd.slot = -1;
}

void LeafGrower::evict(const std::vector<int>& keep) {
  for (size_t i = 0; i < lru_.size(); ++i) {
    const int sid = lru_[i];
    if (std::find(keep.begin(), keep.end(), sid) != keep.end()) continue;
    lru_.erase(lru_.begin() + (long)i);
    free_slots_.push_back(nodes_[sid].slot);
    nodes_[sid].slot = -1;
    return;
  }
  throw std::runtime_error("histogram_pool_capacity too small for one expansion");
}

std::vector<int32_t> LeafGrower::replay() {
  if (nodes_.empty() || !nodes_[0].has_rec) throw std::logic_error("LeafGrower: root not searched");
  if (!started_) {
    heap_.push(Entry{-nodes_[0].loss_chg, 0, 0});
    started_ = true;
  }
  // the sequential priority-queue growth, as far as the known gains allow
  bool blocked = false;
  while (!heap_.empty()) {
    const int sid = heap_.top().sid;
    Node& nd = nodes_[sid];
    if (pop_is_leaf(nd, num_leaf_)) {
      heap_.pop();
      make_leaf(sid, nd.tid);
      if (nd.lc < 0) release(sid);
      continue;
    }
    if (nd.lc < 0) {
      blocked = true;
      break;
    }
    heap_.pop();
    const int t = nd.tid;
    const int lt = tree_alloc(t), rt = tree_alloc(t);
    t_.left[t] = lt;
    t_.right[t] = rt;
    t_.is_leaf[t] = 0;
    t_.feat[t] = nd.feat;
    t_.slot_a[t] = nd.bin_a;
    t_.slot_b[t] = nd.bin_b;
    t_.cond[t] = 0.5 * ((double)nd.bin_a + (double)nd.bin_b);
    ++num_leaf_;
    const int lcs = nd.lc, rcs = nd.rc;
    Node& nl = nodes_[lcs];
    Node& nr = nodes_[rcs];
    nl.tid = lt;
    nr.tid = rt;
    if (children_terminal(nl, nr, num_leaf_)) {
      leafify_children(sid, lcs, rcs, lt, rt);
      nodes_[lcs].rec_used = nodes_[rcs].rec_used = false;
      for (int c : {lcs, rcs})
        if (nodes_[c].lc < 0) release(c);
    } else {
      nl.seq = seq_;
      nr.seq = seq_ + 1;
      heap_.push(Entry{-nl.loss_chg, seq_, lcs});
      heap_.push(Entry{-nr.loss_chg, seq_ + 1, rcs});
      seq_ += 2;
    }
  }
  if (!blocked) return {};
  // expansion batch: the blocked leaf + the next candidates in pop order
  const int64_t remaining = p_.max_leaf > 0 ? (int64_t)p_.max_leaf - num_leaf_ : 1;
  // each expansion takes 2 slots and frees its own; keep one net slot per future split
  const int64_t slack = floor_div((int64_t)free_slots_.size() - remaining - 1, 2);
  const int64_t k = p_.speculate ? std::max<int64_t>(1, std::min(remaining, slack)) : 1;
  const int blocked_sid = heap_.top().sid;
  std::vector<int32_t> batch{blocked_sid};
  if (k > 1) {
    // continue the replay VIRTUALLY, treating the not-yet-computed children of
    // unexpanded splits as absent: the unexpanded nodes it pops as splits (within the
    // leaf budget) are the ones the real replay splits unless an unknown child
    // outranks them -> expand them now
    auto vheap = heap_;
    int vleaf = num_leaf_;
    int64_t vseq = seq_;
    while (!vheap.empty() && (int64_t)batch.size() < k) {
      const int sid = vheap.top().sid;
      vheap.pop();
      const Node& nd = nodes_[sid];
      if (pop_is_leaf(nd, vleaf)) continue;
      ++vleaf;
      if (nd.lc < 0) {
        if (std::find(batch.begin(), batch.end(), sid) == batch.end()) batch.push_back(sid);
        continue;
      }
      const Node& nl = nodes_[nd.lc];
      const Node& nr = nodes_[nd.rc];
      if (!nl.has_rec || !nr.has_rec || children_terminal(nl, nr, vleaf)) continue;
      vheap.push(Entry{-nl.loss_chg, vseq, nd.lc});
      vheap.push(Entry{-nr.loss_chg, vseq + 1, nd.rc});
      vseq += 2;
    }
  }
  return batch;
}

LeafGrower::Expand LeafGrower::expand(const std::vector<int32_t>& batch) {
  Expand ex;
  for (int sid : batch) {
    const int lc = (int)nodes_.size();
    nodes_.emplace_back();
    nodes_.emplace_back();
    Node& nd = nodes_[sid];
    nd.lc = lc;
    nd.rc = lc + 1;
    // children at max_depth are always terminal: only their counts are needed
    if (p_.max_depth >= 0 && nd.depth + 1 == p_.max_depth) ex.count_sid.push_back(sid);
    else ex.split_sid.push_back(sid);
  }
  ++batches;
  expanded += (int)batch.size();
  return ex;
}

void LeafGrower::set_children(const std::vector<int32_t>& parents, const int64_t* lloc, const int64_t* lglob,
                              bool with_begin) {
  for (size_t i = 0; i < parents.size(); ++i) {
    const Node& P = nodes_[parents[i]];
    Node L, R;
    L.depth = R.depth = P.depth + 1;
    if (with_begin) {
      L.begin = P.begin;
      R.begin = P.begin + lloc[i];
    }
    L.cnt_local = lloc[i];
    L.cnt_global = lglob[i];
    R.cnt_local = P.cnt_local - lloc[i];
    R.cnt_global = P.cnt_global - lglob[i];
    const int lc = P.lc, rc = P.rc;
    nodes_[lc] = L;
    nodes_[rc] = R;
  }
}

LeafGrower::HistPlan LeafGrower::plan_hist(const std::vector<int32_t>& split_parents) {
  std::vector<int> build;
  std::vector<std::array<int, 3>> derived;  // (large, parent, small)
  for (int sid : split_parents) {
    const Node& P = nodes_[sid];
    const bool left_small = nodes_[P.lc].cnt_global < nodes_[P.rc].cnt_global;
    const int small = left_small ? P.lc : P.rc, large = left_small ? P.rc : P.lc;
    build.push_back(small);
    if (P.slot >= 0) {
      derived.push_back({large, sid, small});
    } else {  // parent histogram evicted from the pool: rebuild (pool miss)
      build.push_back(large);
      ++hist_miss;
    }
  }
  HistPlan hp;
  const int nb = (int)build.size(), nd = (int)derived.size(), need = nb + nd;
  std::vector<int> keep;
  keep.reserve(nd);
  for (const auto& d : derived) keep.push_back(d[1]);
  while ((int)free_slots_.size() < need) evict(keep);
  hp.order.reserve(need);
  for (int b : build) hp.order.push_back(b);
  for (const auto& d : derived) hp.order.push_back(d[0]);
  hp.slots.resize(need);
  for (int i = 0; i < need; ++i) {
    hp.slots[i] = free_slots_.back();
    free_slots_.pop_back();
    lru_.push_back(hp.order[i]);
    nodes_[hp.order[i]].slot = hp.slots[i];
  }
  hp.nbuild = nb;
  hp.items.assign(4 * (size_t)need, 0);
  for (int i = 0; i < nb; ++i) {
    hp.items[4 * i] = hp.slots[i];
    hp.begin.push_back(nodes_[build[i]].begin);
    hp.count.push_back(nodes_[build[i]].cnt_local);
  }
  for (int j = 0; j < nd; ++j) {
    int32_t* it = &hp.items[4 * (size_t)(nb + j)];
    it[0] = nodes_[derived[j][0]].slot;
    it[1] = nodes_[derived[j][1]].slot;
    it[2] = nodes_[derived[j][2]].slot;
    it[3] = 1;
  }
  return hp;
}

namespace {

int64_t chunk_rows(int64_t total, int target_blocks, int min_rows) {
  return std::max<int64_t>(min_rows, (total + target_blocks - 1) / std::max(1, target_blocks));
}

// segment i = [begin[i], begin[i] + count[i]) -> items (tag[i], b, e, k) of <= ch rows
void emit_chunks(const std::vector<int64_t>& begin, const std::vector<int64_t>& count,
                 const std::vector<int32_t>& tag, int64_t ch, bool blk_index, std::vector<int32_t>& out) {
  for (size_t i = 0; i < begin.size(); ++i) {
    const int64_t end = begin[i] + count[i];
    int64_t k = 0;
    for (int64_t b = begin[i]; b < end; b += ch, ++k) {
      out.push_back(tag[i]);
      out.push_back((int32_t)b);
      out.push_back((int32_t)std::min(b + ch, end));
      out.push_back(blk_index ? (int32_t)k : 0);
    }
  }
}

}  // namespace

LeafGrower::Pack LeafGrower::pack_partition(const std::vector<int32_t>& parents, int part_chunk,
                                            int target_blocks, int min_rows) const {
  Pack pk;
  const size_t n = parents.size();
  std::vector<int64_t> begin(n), count(n);
  std::vector<int32_t> tag(n);
  int64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    begin[i] = nodes_[parents[i]].begin;
    count[i] = nodes_[parents[i]].cnt_local;
    tag[i] = (int32_t)i;
    total += count[i];
  }
  auto& d = pk.data;
  pk.off.push_back(0);
  emit_chunks(begin, count, tag, chunk_rows(total, target_blocks, min_rows), true, d);
  pk.n_items = (int64_t)d.size() / 4;
  pk.off.push_back((int64_t)d.size());
  for (int sid : parents) d.push_back(nodes_[sid].feat);
  pk.off.push_back((int64_t)d.size());
  for (int sid : parents) d.push_back((nodes_[sid].bin_a + nodes_[sid].bin_b) >> 1);
  pk.off.push_back((int64_t)d.size());
  for (size_t i = 0; i < n; ++i) d.push_back((int32_t)begin[i]);
  pk.off.push_back((int64_t)d.size());
  for (size_t i = 0; i < n; ++i) d.push_back((int32_t)count[i]);
  pk.off.push_back((int64_t)d.size());
  int64_t acc = 0;
  for (size_t i = 0; i < n; ++i) {
    d.push_back((int32_t)acc);
    acc += (count[i] + part_chunk - 1) / part_chunk;
  }
  pk.n_blocks = acc;
  pk.off.push_back((int64_t)d.size());
  d.push_back((int32_t)n);
  d.push_back((int32_t)acc);
  return pk;
}

LeafGrower::Pack LeafGrower::pack_hist(const HistPlan& hp, int target_blocks, int min_rows) {
  Pack pk;
  int64_t total = 0;
  for (int64_t c : hp.count) total += c;
  std::vector<int32_t> tag(hp.slots.begin(), hp.slots.begin() + hp.nbuild);
  auto& d = pk.data;
  pk.off.push_back(0);
  if (hp.nbuild > 0) emit_chunks(hp.begin, hp.count, tag, chunk_rows(total, target_blocks, min_rows), false, d);
  pk.n_items = (int64_t)d.size() / 4;
  pk.off.push_back((int64_t)d.size());
  d.insert(d.end(), hp.items.begin(), hp.items.end());
  pk.off.push_back((int64_t)d.size());
  d.insert(d.end(), tag.begin(), tag.end());
  return pk;
}

void LeafGrower::release_batch(const std::vector<int32_t>& batch) {
  for (int sid : batch) release(sid);
}

LeafGrower::TreeOut LeafGrower::finish() {
  for (const Node& nd : nodes_) {
    if (nd.tid < 0) continue;
    t_.loss_chg[nd.tid] = (nd.has_rec && nd.rec_used) ? (float)nd.loss_chg
                                                      : -std::numeric_limits<float>::infinity();
    t_.hess_sum[nd.tid] = (float)nd.H;
    t_.sample_cnt[nd.tid] = nd.cnt_global;
  }
  return t_;
}

}  // namespace ytk_native
