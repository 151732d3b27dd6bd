// GPU-resident level-wise tree construction (gfx950).
//
// Reference control flow: J/optimizer/gbdt/DataParallelTreeMaker.java make() :229-295
// -- FIFO expansion queue (level-wise), leaf conditions at pop time (lossChg <=
// min_split_loss, depth == max_depth, leaves == max_leaf_cnt, samples <
// min_split_samples), children made leaves right away when their depth reaches
// max_depth / the leaf budget is used / both children are below min_split_samples,
// smaller child histogram + sibling subtraction, canSplit (UpdateStrategy:50-53).
//
// MI355X design: the decisions of a level (<= 2^depth nodes) run in one 256-thread
// "planner" workgroup: node fields are staged in LDS by all lanes, the FIFO leaf
// budget (running leaf count under max_leaf_cnt) is a block scan over the candidate
// flags, and the work lists (partition chunks, histogram chunks, split items) are
// emitted in parallel after block scans (wave64 shuffle scans, no serial loops). The heavy kernels (partition / histogram /
// split) are launched with FIXED maximal grids and read their item counts from
// device memory, so a whole tree is a fixed launch sequence: no device->host
// synchronisation inside a tree, and multi-GPU all-reduces are fixed-size RCCL calls
// on the same stream.
#include "common.h"

#include <algorithm>
#include "gbdt_split_node.h"  // SplitOut (one definition, layout static_assert'ed there)
#include "gbdt_tree_node.h"  // DNode, node_leaf_value
#include "gbdt_partition_atomic.h"  // partition_atomic_body

namespace ytk {

enum {
  ST_NUM_NODES = 0, ST_NUM_LEAF, ST_N_PENDING, ST_N_SPLIT, ST_N_PART, ST_N_HIST,
  ST_N_SITEMS, ST_N_BUILD, ST_N_HIST_A, ST_PART_DONE, ST_WORDS = 16
};

constexpr int kPlanThreads = 256;
constexpr int kMaxPend = 4096;  // 2^12 = MAX_DEPTH_DEVICE

struct LvParams {
  int max_depth, max_leaf_cnt, min_split_samples;
  float min_split_loss, mcw, l1, l2, max_abs_leaf, lr;
  int hist_target, part_target, min_rows;
  int part_chunk;  // rows per single-pass partition chunk (fused kernel: 256 x rows per thread)
  int split_groups;  // split records per item (feature groups of split_node_kernel; 1 = one)
  // 1: the last level is not partitioned (leaf counts come from the gradient pass), so at
  // the level before it only the child that gets a histogram is ever read again -- its
  // partition writes that child's rows alone (scatter mask in part_thr, see keep_row)
  int small_only;
};

// The child whose histogram is built (the other is parent - built): by the hessian sums,
// which every rank knows before the partition (exact int64 histograms make the choice
// result neutral). Used wherever the choice must precede the row counts.
__device__ __forceinline__ bool left_small_by_hess(double hl, double H) { return hl < H - hl; }
__device__ __forceinline__ bool small_only_level(int small_only, int max_depth, int depth) {
  return small_only && max_depth >= 0 && depth + 2 == max_depth;
}

struct LvBufs {
  int* st;
  DNode* nodes;
  int* pending;
  int* next_pending;
  int* split_nid;
  int* split_snap;
  int4* part_items;
  int* part_feat;
  int* part_thr;
  int* part_begin;
  int* part_first;
  int* part_nblk;
  int* part_counts;      // per partition block
  long long* left_loc;   // per split (accumulated by the partition flag kernel)
  long long* left_glob;  // per split (all-reduced; == left_loc on one rank)
  int4* hist_items;
  int4* split_items;
  int* item_nid;
  SplitOut* split_out;
  int* tfeat;
  int* tthr;
  int* tleft;
  int* tright;
  float* tval;
  long long* root_cnt;   // [0] local, [1] global
  int* part_cnt;         // per split: rows of this rank's segment (single-pass partition)
  int* hist_first;       // per build k: first histogram item of the build's slot ([nb] = item count)
};

__device__ __forceinline__ float leaf_value(double g, double h, const LvParams& p) {
  return node_leaf_value(g, h, p.mcw, p.l1, p.l2, p.max_abs_leaf, p.lr);
}

__device__ void reset_node(DNode& n, int depth) {
  n.G = n.H = n.gl = n.hl = 0.0;
  n.cnt_global = 0;
  n.begin = n.cnt_local = 0;
  n.depth = depth;
  n.slot = -1;
  n.feat = -1;
  n.bin_a = n.bin_b = -1;
  n.left = n.right = -1;
  n.loss_chg = -INFINITY;
  n.value = 0.f;
  n.is_leaf = 1;
}

// Exclusive scan of one int per thread over the block (wave64 shuffles + one total per
// wave through LDS; 256 threads for the planner launches, 1024 in the fused split + plan
// kernel). Returns this thread's exclusive prefix; *total = sum.
// Must be called by every thread of the block. s_tmp: >= blockDim.x/64 + 1 ints.
__device__ __forceinline__ int block_scan_excl(int v, int* s_tmp, int* total) {
  const int tid = threadIdx.x, l = tid & (kWave - 1), w = tid >> 6;
  int inc = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int o = __shfl_up(inc, off, kWave);
    if (l >= off) inc += o;
  }
  if (l == kWave - 1) s_tmp[w] = inc;
  __syncthreads();
  int before = 0, all = 0;
  const int nw = (int)blockDim.x / kWave;
  for (int k = 0; k < nw; ++k) {
    const int t = s_tmp[k];
    if (k < w) before += t;
    all += t;
  }
  __syncthreads();  // s_tmp reusable afterwards
  *total = all;
  return before + inc - v;
}

// In-place exclusive scan of a[0..n) (n <= kMaxPend) by one block.
// Returns the total. Each thread owns a contiguous run of ceil(n/256) entries; the
// run totals are scanned with wave shuffles (no serial lane-0 loop: the old
// 256-step LDS chain cost ~10 us per planner launch).
__device__ int block_exclusive_scan(int* a, int n, int* s_tmp) {
  const int tid = threadIdx.x;
  const int per = (n + (int)blockDim.x - 1) / (int)blockDim.x;
  const int b = min(n, tid * per), e = min(n, b + per);
  int run = 0;
  for (int i = b; i < e; ++i) run += a[i];
  int total;
  int acc = block_scan_excl(run, s_tmp, &total);
  for (int i = b; i < e; ++i) {
    const int v = a[i];
    a[i] = acc;
    acc += v;
  }
  __syncthreads();
  return total;
}

// Parallel chunk emission: segment s (begin[s], count[s]) -> first[s] .. first[s]+nblk[s]
// items {tag(s), chunk_begin, chunk_end, j}. first[] holds the exclusive scan of nblk.
__device__ void emit_all_chunks(int4* items, int total_items, int nseg, const int* first,
                                const int* begin, const int* count, const int* tag, int ch,
                                bool blk_index) {
  for (int k = threadIdx.x; k < total_items; k += (int)blockDim.x) {
    int lo = 0, hi = nseg - 1;  // last s with first[s] <= k
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (first[mid] <= k) lo = mid; else hi = mid - 1;
    }
    const int s = lo;
    const int j = k - first[s];
    const int cb = begin[s] + j * ch;
    items[k] = make_int4(tag ? tag[s] : s, cb, min(cb + ch, begin[s] + count[s]), blk_index ? j : 0);
  }
}

// Fixed-point scales from the (all-reduced) max |g|, |h| and global row count (threads 0, 1).
__device__ __forceinline__ void lv_scales_body(const float* __restrict__ mx, const long long* __restrict__ cnt,
                                               float* __restrict__ scales, double* __restrict__ inv_scales) {
  if (threadIdx.x >= 2) return;
  const double m = (double)mx[threadIdx.x];
  double s = 1.0;
  if (m > 0.0) {
    const double n = (double)max(1LL, cnt[1]);
    int k = (int)floor(log2(4611686018427387904.0 / (m * n)));
    k = min(max(k, -120), 120);
    s = ldexp(1.0, k);
  }
  scales[threadIdx.x] = (float)s;
  inv_scales[threadIdx.x] = 1.0 / s;
}

// Root: node 0 holds all (local) rows; one build item; chunked histogram work. mx != nullptr:
// the tree's fixed-point scales too (lv_scales_kernel's work: one launch less per tree).
__global__ __launch_bounds__(kPlanThreads) void lv_init_kernel(LvParams p, LvBufs b, const float* __restrict__ mx,
                                                               float* __restrict__ scales,
                                                               double* __restrict__ inv_scales) {
  __shared__ int s_first[2], s_begin[1], s_count[1], s_tag[1];
  if (mx) lv_scales_body(mx, b.root_cnt, scales, inv_scales);
  const int n_local = (int)b.root_cnt[0];
  const int ch = max(p.min_rows, (n_local + p.hist_target - 1) / max(1, p.hist_target));
  const int nblk = (n_local + ch - 1) / ch;
  if (threadIdx.x == 0) {
    DNode& r = b.nodes[0];
    reset_node(r, 0);
    r.begin = 0;
    r.cnt_local = n_local;
    r.cnt_global = b.root_cnt[1];
    r.slot = 0;
    int* st = b.st;
    for (int i = 0; i < ST_WORDS; ++i) st[i] = 0;
    st[ST_NUM_NODES] = 1;
    st[ST_NUM_LEAF] = 1;
    b.pending[0] = 0;
    st[ST_N_PENDING] = 1;
    st[ST_N_HIST] = nblk;
    st[ST_N_BUILD] = 1;
    b.split_items[0] = make_int4(0, 0, 0, 0);
    b.item_nid[0] = 0;
    st[ST_N_SITEMS] = 1;
    s_first[0] = 0;
    s_begin[0] = 0;
    s_count[0] = n_local;
    s_tag[0] = 0;
  }
  __syncthreads();
  emit_all_chunks(b.hist_items, nblk, 1, s_first, s_begin, s_count, s_tag, ch, false);
}

// Fast path of lv_plan_split_body for levels of <= kPlanThreads pending nodes whose split
// items follow lv_plan_children_body's layout (pending [2k, 2k+1] = the children of build k;
// item k = its built child, item nb + k = the derived one; the root: one item, one node):
// ONE thread per pending node keeps that node in registers from its records to its
// partition descriptor, so the dependent global round trips are st -> (pending, item_nid)
// -> (records, node fields) instead of ~12 (node-table writes read back by other threads,
// the chunk counts and their scan in global memory). Same decisions, same outputs.
__device__ void lv_plan_split_fast(const LvParams& p, const LvBufs& b, int fused, int implicit_items, int nsi,
                                   int npend, int num_nodes0, int num_leaf0, int nprev) {
  // (256-thread planner launches and the 1024-thread fused split + plan kernel's last block)
  __shared__ int s_tmp[1024 / kWave + 1];
  __shared__ int s_cnt[kPlanThreads], s_first[kPlanThreads], s_beg[kPlanThreads];
  __shared__ long long s_total;
  int* st = b.st;
  const int tid = threadIdx.x;
  const double mcw2 = (double)p.mcw * 2.0;
  if (fused) {  // previous level's children: global counts from the all-reduced cursors
    const size_t cs = fused == 2 ? kCurStride : 1;
    for (int s = tid; s < nprev; s += (int)blockDim.x) {
      const DNode& P = b.nodes[b.split_nid[s]];
      const long long lg = b.left_glob[(size_t)s * cs] & 0xffffffffll;
      b.nodes[P.left].cnt_global = lg;
      b.nodes[P.right].cnt_global = P.cnt_global - lg;
    }
    // (nothing below reads cnt_global when counts are fused: min_split_samples <= 0 there)
  }
  if (tid == 0) s_total = 0;
  const bool mine = tid < npend;
  int nid = 0, item = 0;
  if (mine) {
    nid = b.pending[tid];
    const int k = tid >> 1;
    item = b.item_nid[k] == nid ? k : (nsi >> 1) + k;
  }
  double G = 0.0, H = 0.0, gl = 0.0, hl = 0.0;
  int feat = -1, bin_a = -1, bin_b = -1, depth = 0, beg = 0, cnt_local = 0;
  long long cnt_global = 0;
  float loss_chg = -INFINITY;
  bool cand = false;
  if (mine) {
    const int ng = p.split_groups;
    const SplitOut* rec = b.split_out + (size_t)item * ng;
    auto fkey = [](int f) { return f < 0 ? 0x7fffffff : f; };
    int bg = 0;
    for (int g = 1; g < ng; ++g)
      if (better(rec[g].loss_chg, fkey(rec[g].feat), fkey(rec[g].bin_b), rec[bg].loss_chg, fkey(rec[bg].feat),
                 fkey(rec[bg].bin_b)))
        bg = g;
    const SplitOut o = rec[bg];
    G = rec[0].g;  // node totals: identical exact sums in every group's record
    H = rec[0].h;
    gl = o.gl;
    hl = o.hl;
    feat = o.feat;
    bin_a = o.bin_a;
    bin_b = o.bin_b;
    loss_chg = o.loss_chg;
    DNode& n = b.nodes[nid];
    cnt_global = n.cnt_global;
    depth = n.depth;
    beg = n.begin;
    cnt_local = n.cnt_local;
    if (!(H >= mcw2 && cnt_global >= (long long)p.min_split_samples)) {  // canSplit
      loss_chg = -INFINITY;
      feat = -1;
    }
    n.G = G;
    n.H = H;
    n.gl = gl;
    n.hl = hl;
    n.feat = feat;
    n.bin_a = bin_a;
    n.bin_b = bin_b;
    n.loss_chg = loss_chg;
    // pop-time leaf rules that do not depend on the running leaf count
    cand = !(!(loss_chg > p.min_split_loss) || (p.max_depth >= 0 && p.max_depth == depth) ||
             (p.min_split_samples > 0 && cnt_global < p.min_split_samples));
  }
  // FIFO leaf budget: the first (max_leaf_cnt - num_leaf0) candidates split
  int ncand;
  const int rank = block_scan_excl(cand ? 1 : 0, s_tmp, &ncand);
  const int limit = (p.max_leaf_cnt > 0 && num_leaf0 <= p.max_leaf_cnt) ? p.max_leaf_cnt - num_leaf0 : 0x7fffffff;
  const int nsplit = min(ncand, limit);
  if (tid == 0) {
    st[ST_PART_DONE] = 0;
    st[ST_NUM_NODES] = num_nodes0 + 2 * nsplit;
    st[ST_NUM_LEAF] = num_leaf0 + nsplit;
    st[ST_N_SPLIT] = nsplit;
  }
  if (mine) {
    DNode& n = b.nodes[nid];
    const int s = (cand && rank < limit) ? rank : -1;
    if (s < 0) {
      n.is_leaf = 1;
      n.value = leaf_value(G, H, p);
    } else {
      n.is_leaf = 0;
      n.left = num_nodes0 + 2 * s;
      n.right = num_nodes0 + 2 * s + 1;
      b.split_nid[s] = nid;
      b.split_snap[s] = num_leaf0 + s + 1;  // leaf count after this split
      b.part_feat[s] = feat;
      const int keep = small_only_level(p.small_only, p.max_depth, depth) ? (left_small_by_hess(hl, H) ? 1 : 2) : 0;
      b.part_thr[s] = ((bin_a + bin_b) >> 1) | (keep << kKeepShift);  // bin <= floor((a+b)/2) <=> bin < (a+b)/2
      b.part_begin[s] = beg;
      b.part_cnt[s] = cnt_local;
      b.left_loc[s] = 0;
      b.left_loc[(size_t)s * kCurStride] = 0;  // the fused partition's line-spaced cursor
      s_cnt[s] = cnt_local;
      s_beg[s] = beg;
      atomicAdd(reinterpret_cast<unsigned long long*>(&s_total), (unsigned long long)cnt_local);
    }
  }
  __syncthreads();
  const long long total = s_total;
  const int ch = (int)max((long long)p.part_chunk, (total + p.part_target - 1) / max(1, p.part_target));
  const int nblk = tid < nsplit ? (s_cnt[tid] + ch - 1) / ch : 0;
  int nitems;
  const int first = block_scan_excl(nblk, s_tmp, &nitems);
  if (tid < nsplit) {
    b.part_first[tid] = first;
    b.part_nblk[tid] = nblk;
    s_first[tid] = first;
  }
  if (tid == 0) st[ST_N_PART] = nitems;
  if (!implicit_items) {
    __syncthreads();
    emit_all_chunks(b.part_items, nitems, nsplit, s_first, s_beg, s_cnt, nullptr, ch, true);
  }
}

// Apply split results, pop the level's nodes in FIFO order, emit partition chunks.
template <int KP>
__device__ void lv_plan_split_body(const LvParams& p, const LvBufs& b, int fused, int implicit_items) {
  {
    // one round trip for every state word; the fast path when the level fits one thread per
    // node (implicit_items bit 1: YTK_PLAN_FAST=0, the general path below)
    const bool fast_ok = !(implicit_items & 2);
    implicit_items &= 1;
    const int nsi = b.st[ST_N_SITEMS], npend = b.st[ST_N_PENDING];
    const int num_nodes0 = b.st[ST_NUM_NODES], num_leaf0 = b.st[ST_NUM_LEAF], nprev = b.st[ST_N_SPLIT];
    if (fast_ok && npend <= kPlanThreads && npend == nsi && (int)blockDim.x >= kPlanThreads) {
      lv_plan_split_fast(p, b, fused, implicit_items, nsi, npend, num_nodes0, num_leaf0, nprev);
      return;
    }
  }
  __shared__ int s_aux[KP];   // candidate flag, later: split index / -1
  __shared__ int s_rank[KP];  // rank among the candidates (FIFO order)
  __shared__ int s_tmp[kPlanThreads + 1];
  const int NT = (int)blockDim.x;
  __shared__ long long s_total;
  int* st = b.st;
  const int tid = threadIdx.x;
  const double mcw2 = (double)p.mcw * 2.0;
  // 0. fused counts: the children of the previous level's splits get their global row
  //    counts from the (now all-reduced) count slots
  // fused == 2: the counts were accumulated by the fused partition kernel into line-spaced
  // cursors ((right << 32) | left, kCurStride apart); fused == 1: one word per split
  if (fused) {
    const int nprev = st[ST_N_SPLIT];
    const size_t cs = fused == 2 ? kCurStride : 1;
    for (int s = tid; s < nprev; s += NT) {
      const DNode& P = b.nodes[b.split_nid[s]];
      const long long lg = b.left_glob[(size_t)s * cs] & 0xffffffffll;  // low half: left rows (see partition)
      b.nodes[P.left].cnt_global = lg;
      b.nodes[P.right].cnt_global = P.cnt_global - lg;
    }
    __syncthreads();
  }
  // 1. apply split-finder results to the node table (canSplit)
  const int nsi = st[ST_N_SITEMS];
  for (int i = tid; i < nsi; i += NT) {
    DNode& n = b.nodes[b.item_nid[i]];
    // the item's best over its feature-group records: better() order (larger gain, then
    // lower feature, then lower bin), "none" (-1) last -- the single block's argmax
    const int ng = p.split_groups;
    int bg = 0;
    auto fkey = [](int f) { return f < 0 ? 0x7fffffff : f; };
    for (int g = 1; g < ng; ++g) {
      const SplitOut& c = b.split_out[(size_t)i * ng + g];
      const SplitOut& bb = b.split_out[(size_t)i * ng + bg];
      if (better(c.loss_chg, fkey(c.feat), fkey(c.bin_b), bb.loss_chg, fkey(bb.feat), fkey(bb.bin_b))) bg = g;
    }
    SplitOut o = b.split_out[(size_t)i * ng + bg];
    if (bg != 0) {  // node totals: identical exact sums in every group's record
      o.g = b.split_out[(size_t)i * ng].g;
      o.h = b.split_out[(size_t)i * ng].h;
    }
    n.G = o.g;
    n.H = o.h;
    n.gl = o.gl;
    n.hl = o.hl;
    n.feat = o.feat;
    n.bin_a = o.bin_a;
    n.bin_b = o.bin_b;
    n.loss_chg = o.loss_chg;
    if (!(o.h >= mcw2 && n.cnt_global >= (long long)p.min_split_samples)) {
      n.loss_chg = -INFINITY;
      n.feat = -1;
    }
  }
  __syncthreads();
  // 2. pop-time leaf rules that do not depend on the running leaf count
  const int npend = st[ST_N_PENDING];
  const int num_nodes0 = st[ST_NUM_NODES], num_leaf0 = st[ST_NUM_LEAF];
  for (int i = tid; i < npend; i += NT) {
    const DNode& n = b.nodes[b.pending[i]];
    const bool leaf = !(n.loss_chg > p.min_split_loss) ||
                      (p.max_depth >= 0 && p.max_depth == n.depth) ||
                      (p.min_split_samples > 0 && n.cnt_global < p.min_split_samples);
    s_aux[i] = leaf ? 0 : 1;
    s_rank[i] = leaf ? 0 : 1;
  }
  if (tid == 0) s_total = 0;
  __syncthreads();
  // 3. FIFO leaf budget, in parallel: the running leaf count before candidate i is
  // num_leaf0 + rank(i) (each split adds one leaf) and the reference makes a node a
  // leaf once that count == max_leaf_cnt, so exactly the first
  // (max_leaf_cnt - num_leaf0) candidates split.
  const int ncand = block_exclusive_scan(s_rank, npend, s_tmp);
  const int limit = (p.max_leaf_cnt > 0 && num_leaf0 <= p.max_leaf_cnt) ? p.max_leaf_cnt - num_leaf0
                                                                         : 0x7fffffff;
  const int nsplit = min(ncand, limit);
  if (tid == 0) {
    st[ST_PART_DONE] = 0;
    st[ST_NUM_NODES] = num_nodes0 + 2 * nsplit;
    st[ST_NUM_LEAF] = num_leaf0 + nsplit;
    st[ST_N_SPLIT] = nsplit;
  }
  // 4. write decisions back; per-split partition descriptors
  for (int i = tid; i < npend; i += NT) {
    const int id = b.pending[i];
    DNode& n = b.nodes[id];
    const int s = (s_aux[i] && s_rank[i] < limit) ? s_rank[i] : -1;
    if (s < 0) {
      n.is_leaf = 1;
      n.value = leaf_value(n.G, n.H, p);
    } else {
      n.is_leaf = 0;
      n.left = num_nodes0 + 2 * s;
      n.right = num_nodes0 + 2 * s + 1;
      b.split_nid[s] = id;
      b.split_snap[s] = num_leaf0 + s + 1;  // leaf count after this split
      b.part_feat[s] = n.feat;
      const int keep = small_only_level(p.small_only, p.max_depth, n.depth)
                           ? (left_small_by_hess(n.hl, n.H) ? 1 : 2) : 0;
      b.part_thr[s] = ((n.bin_a + n.bin_b) >> 1) | (keep << kKeepShift);  // bin <= floor((a+b)/2) <=> bin < (a+b)/2
      b.part_begin[s] = n.begin;
      b.part_nblk[s] = n.cnt_local;              // temporarily: count
      b.part_cnt[s] = n.cnt_local;
      b.left_loc[s] = 0;
      b.left_loc[(size_t)s * kCurStride] = 0;  // the fused partition's line-spaced cursor
      atomicAdd(reinterpret_cast<unsigned long long*>(&s_total), (unsigned long long)n.cnt_local);
    }
  }
  __syncthreads();
  const long long total = s_total;
  const int ch = (int)max((long long)p.part_chunk, (total + p.part_target - 1) / max(1, p.part_target));
  // counts -> chunk counts (stage counts in LDS for emission)
  int* s_count = s_aux;  // reuse: per split row count
  for (int s = tid; s < nsplit; s += NT) {
    const int c = b.part_nblk[s];
    s_count[s] = c;
    b.part_first[s] = (c + ch - 1) / ch;
  }
  __syncthreads();
  const int nitems = block_exclusive_scan(b.part_first, nsplit, s_tmp);
  for (int s = tid; s < nsplit; s += NT) b.part_nblk[s] = (s + 1 < nsplit ? b.part_first[s + 1] : nitems) - b.part_first[s];
  if (tid == 0) st[ST_N_PART] = nitems;
  __syncthreads();
  // the single-pass partition maps its blocks to (split, chunk) itself from part_first
  if (!implicit_items)
    emit_all_chunks(b.part_items, nitems, nsplit, b.part_first, b.part_begin, s_count, nullptr, ch, true);
}

__global__ __launch_bounds__(kPlanThreads) void lv_plan_split_kernel(LvParams p, LvBufs b, int fused,
                                                                   int implicit_items) {
  lv_plan_split_body<kMaxPend>(p, b, fused, implicit_items);
}

// Children of this level's splits: segments, terminal check, build / derive lists,
// histogram chunks. build_base: first slot of this level, half: slots for builds,
// dgap: derived slot = built slot + dgap (half, plus the count slots when fused).
// fused (multi-GPU, min_split_samples <= 0): the left counts are still LOCAL here --
// they ride in count slots of the level's histogram all-reduce -- so the smaller child
// is chosen by the (globally identical) hessian sums and cnt_global is patched by the
// next lv_plan_split. Exact int64 histograms make the choice result-neutral.
// KP: bound on the level's splits (LDS arrays); kAtomicCursor: the cursors were just
// updated by atomics of other blocks of the same kernel (fused partition epilogue)
template <int KP, bool kAtomicCursor>
__device__ void lv_plan_children_body(const LvParams& p, const LvBufs& b, int cs, int build_base, int half, int dgap,
                                      int use_loc, int fused) {
  __shared__ int s_nb[KP];     // 1 if the split's children get histograms
  __shared__ int s_small[KP];  // small child node id
  __shared__ int s_tmp[kPlanThreads + 1];
  __shared__ long long s_total;
  __shared__ int s_hbeg[KP], s_hcnt[KP], s_hslot[KP];
  int* st = b.st;
  const int tid = threadIdx.x;
  const int nsplit = st[ST_N_SPLIT];
  const bool fast_ok = !(use_loc & 2);  // bit 1: YTK_PLAN_FAST=0 (the general path below)
  use_loc &= 1;
  const long long* lglob_arr = use_loc ? b.left_loc : b.left_glob;
  if (tid == 0) s_total = 0;
  __syncthreads();
  if (fast_ok && nsplit <= kPlanThreads && (int)blockDim.x == kPlanThreads) {
    // Fast path: one thread per split keeps the parent and its children in registers from
    // the cursors to the histogram work list -- dependent global round trips st ->
    // (split_nid, cursors, snap) -> parent fields, instead of re-reading the node table
    // (written by other threads) and a pending copy through memory. Same outputs.
    const int s = tid;
    const bool mine = s < nsplit;
    int pid = 0, snap = 0;
    long long lloc = 0, lglob = 0;
    if (mine) {
      pid = b.split_nid[s];
      snap = b.split_snap[s];
      if (kAtomicCursor) {
        lloc = __hip_atomic_load(&b.left_loc[(size_t)s * cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffll;
        lglob = __hip_atomic_load(&lglob_arr[(size_t)s * cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffll;
      } else {
        lloc = b.left_loc[(size_t)s * cs] & 0xffffffffll;
        lglob = lglob_arr[(size_t)s * cs] & 0xffffffffll;
      }
    }
    bool need = false, left_small = false;
    int lid = 0, rid = 0, pslot = 0, pbeg = 0, lcnt = 0, rcnt = 0;
    if (mine) {
      const DNode& P = b.nodes[pid];
      lid = P.left;
      rid = P.right;
      pslot = P.slot;
      pbeg = P.begin;
      const int pdepth = P.depth, pcnt = P.cnt_local;
      const long long pcg = P.cnt_global;
      const double pG = P.G, pH = P.H, pgl = P.gl, phl = P.hl;
      DNode& L = b.nodes[lid];
      DNode& R = b.nodes[rid];
      reset_node(L, pdepth + 1);
      reset_node(R, pdepth + 1);
      lcnt = (int)lloc;
      rcnt = pcnt - (int)lloc;
      const long long lcg = lglob, rcg = pcg - lglob;
      L.begin = pbeg;
      L.cnt_local = lcnt;
      L.cnt_global = lcg;
      R.begin = pbeg + lcnt;
      R.cnt_local = rcnt;
      R.cnt_global = rcg;
      const bool terminal = (p.max_depth >= 0 && p.max_depth == pdepth + 1) ||
                            (p.max_leaf_cnt > 0 && p.max_leaf_cnt == snap) ||
                            (p.min_split_samples > 0 && lcg < p.min_split_samples && rcg < p.min_split_samples);
      if (terminal) {
        L.G = pgl; L.H = phl;
        R.G = pG - pgl; R.H = pH - phl;
        L.value = leaf_value(pgl, phl, p);
        R.value = leaf_value(pG - pgl, pH - phl, p);
      } else {
        left_small = (fused || small_only_level(p.small_only, p.max_depth, pdepth)) ? left_small_by_hess(phl, pH)
                                                                                     : (lcg < rcg);
        need = true;
        atomicAdd(reinterpret_cast<unsigned long long*>(&s_total), (unsigned long long)(left_small ? lcnt : rcnt));
      }
    }
    int nb;
    const int k = block_scan_excl(need ? 1 : 0, s_tmp, &nb);  // build index (scan barriers order s_total)
    const long long total = s_total;
    const int tgt = p.hist_target > 2 * nb ? p.hist_target - nb : p.hist_target;
    const int ch = (int)max((long long)p.min_rows, (total + tgt - 1) / max(1, tgt));
    int hbeg = 0, hcnt = 0;
    if (need) {
      const int small_id = left_small ? lid : rid, large_id = left_small ? rid : lid;
      const int sslot = build_base + k, lslot = build_base + dgap + k;
      b.nodes[small_id].slot = sslot;
      b.nodes[large_id].slot = lslot;
      b.split_items[k] = make_int4(sslot, 0, 0, 0);
      b.item_nid[k] = small_id;
      b.split_items[nb + k] = make_int4(lslot, pslot, sslot, 1);
      b.item_nid[nb + k] = large_id;
      b.pending[2 * k] = lid;
      b.pending[2 * k + 1] = rid;
      hbeg = left_small ? pbeg : pbeg + lcnt;
      hcnt = left_small ? lcnt : rcnt;
    }
    int nitems;
    const int first = block_scan_excl(need ? (hcnt + ch - 1) / ch : 0, s_tmp, &nitems);
    if (need) {  // per build k (emit_all_chunks reads them by build index)
      s_small[k] = first;
      s_hbeg[k] = hbeg;
      s_hcnt[k] = hcnt;
      s_hslot[k] = build_base + k;
      if (b.hist_first) b.hist_first[k] = first;
    }
    __syncthreads();
    emit_all_chunks(b.hist_items, nitems, nb, s_small, s_hbeg, s_hcnt, s_hslot, ch, false);
    // build slots nb < k < half have no node this level: empty ranges, so the known-range
    // reduce (one y block per build slot) reads no stale items left by an earlier level
    if (b.hist_first)
      for (int k = nb + 1 + tid; k <= half; k += kPlanThreads) b.hist_first[k] = nitems;
    if (tid == 0) {
      if (b.hist_first) b.hist_first[nb] = nitems;
      const int hs = half >> 1;
      st[ST_N_HIST_A] = (hs > 0 && nb > hs) ? s_small[hs] : nitems;
      st[ST_N_PENDING] = 2 * nb;
      st[ST_N_BUILD] = nb;
      st[ST_N_SITEMS] = 2 * nb;
      st[ST_N_HIST] = nitems;
    }
    return;
  }
  for (int s = tid; s < nsplit; s += kPlanThreads) {
    DNode& P = b.nodes[b.split_nid[s]];
    DNode& L = b.nodes[P.left];
    DNode& R = b.nodes[P.right];
    // split cursors pack (right rows << 32) | left rows (single-pass partition); the
    // count-only pass accumulates the left rows alone -- either way the low half
    long long lloc, lglob;
    if (kAtomicCursor) {
      lloc = __hip_atomic_load(&b.left_loc[(size_t)s * cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffll;
      lglob = __hip_atomic_load(&lglob_arr[(size_t)s * cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffll;
    } else {
      lloc = b.left_loc[(size_t)s * cs] & 0xffffffffll;
      lglob = lglob_arr[(size_t)s * cs] & 0xffffffffll;
    }
    reset_node(L, P.depth + 1);
    reset_node(R, P.depth + 1);
    L.begin = P.begin;
    L.cnt_local = (int)lloc;
    L.cnt_global = lglob;
    R.begin = P.begin + (int)lloc;
    R.cnt_local = P.cnt_local - (int)lloc;
    R.cnt_global = P.cnt_global - lglob;
    const bool terminal = (p.max_depth >= 0 && p.max_depth == P.depth + 1) ||
                          (p.max_leaf_cnt > 0 && p.max_leaf_cnt == b.split_snap[s]) ||
                          (p.min_split_samples > 0 && L.cnt_global < p.min_split_samples &&
                           R.cnt_global < p.min_split_samples);
    if (terminal) {
      L.G = P.gl; L.H = P.hl;
      R.G = P.G - P.gl; R.H = P.H - P.hl;
      L.value = leaf_value(L.G, L.H, p);
      R.value = leaf_value(R.G, R.H, p);
      s_nb[s] = 0;
    } else {
      const bool left_small = (fused || small_only_level(p.small_only, p.max_depth, P.depth))
                                  ? left_small_by_hess(P.hl, P.H) : (L.cnt_global < R.cnt_global);
      s_small[s] = left_small ? P.left : P.right;
      s_nb[s] = 1;
      atomicAdd(reinterpret_cast<unsigned long long*>(&s_total),
                (unsigned long long)(left_small ? L.cnt_local : R.cnt_local));
    }
  }
  __syncthreads();
  // keep a copy of the flags (scan is in place)
  for (int s = tid; s < nsplit; s += kPlanThreads) s_hslot[s] = s_nb[s];
  __syncthreads();
  const int nb = block_exclusive_scan(s_nb, nsplit, s_tmp);  // s_nb = build index
  const long long total = s_total;
  // sum over the nodes of ceil(rows / ch) <= total / ch + nb: sizing the chunks for
  // hist_target - nb items keeps the launch within ONE block per CU (the 128-KiB LDS
  // histogram allows one per CU) -- hist_target + nb items left nb CUs running two
  // chunks back to back, doubling the kernel's time
  const int tgt = p.hist_target > 2 * nb ? p.hist_target - nb : p.hist_target;
  const int ch = (int)max((long long)p.min_rows, (total + tgt - 1) / max(1, tgt));
  for (int s = tid; s < nsplit; s += kPlanThreads) {
    if (!s_hslot[s]) continue;
    const int k = s_nb[s];
    DNode& P = b.nodes[b.split_nid[s]];
    const int small_id = s_small[s];
    const int large_id = (small_id == P.left) ? P.right : P.left;
    DNode& S = b.nodes[small_id];
    DNode& Lg = b.nodes[large_id];
    S.slot = build_base + k;
    Lg.slot = build_base + dgap + k;
    b.split_items[k] = make_int4(S.slot, 0, 0, 0);
    b.item_nid[k] = small_id;
    b.split_items[nb + k] = make_int4(Lg.slot, P.slot, S.slot, 1);
    b.item_nid[nb + k] = large_id;
    b.next_pending[2 * k] = P.left;
    b.next_pending[2 * k + 1] = P.right;
    s_hbeg[k] = S.begin;
    s_hcnt[k] = S.cnt_local;
  }
  __syncthreads();
  for (int i = tid; i < 2 * nb; i += kPlanThreads) b.pending[i] = b.next_pending[i];
  // histogram chunks of the build nodes
  for (int k = tid; k < nb; k += kPlanThreads) s_hslot[k] = build_base + k;
  __syncthreads();
  for (int k = tid; k < nb; k += kPlanThreads) s_small[k] = (s_hcnt[k] + ch - 1) / ch;
  __syncthreads();
  const int nitems = block_exclusive_scan(s_small, nb, s_tmp);
  emit_all_chunks(b.hist_items, nitems, nb, s_small, s_hbeg, s_hcnt, s_hslot, ch, false);
  // the items of build k are [s_small[k], s_small[k + 1]) (the fused reduce + split kernel
  // reads its slot's range from here instead of scanning the work list)
  if (b.hist_first) {
    for (int k = tid; k < nb; k += kPlanThreads) b.hist_first[k] = s_small[k];
    for (int k = nb + tid; k <= half; k += kPlanThreads) b.hist_first[k] = nitems;  // nb < k: empty
  }
  if (tid == 0) {
    // items of the first half of the build slots (k < half/2): the multi-GPU engine
    // all-reduces that half while the second half is still being built
    const int hs = half >> 1;
    st[ST_N_HIST_A] = (hs > 0 && nb > hs) ? s_small[hs] : nitems;
    st[ST_N_PENDING] = 2 * nb;
    st[ST_N_BUILD] = nb;
    st[ST_N_SITEMS] = 2 * nb;
    st[ST_N_HIST] = nitems;
  }
}

__global__ __launch_bounds__(kPlanThreads) void lv_plan_children_kernel(LvParams p, LvBufs b, int build_base,
                                                                    int half, int dgap, int use_loc,
                                                                    int fused) {
  lv_plan_children_body<kMaxPend, false>(p, b, 1, build_base, half, dgap, use_loc, fused);
}

// One-GPU levels: the partition (partition_atomic_body) and the children planning in one
// launch -- the last block to finish (device-scope counter, no fences: the split cursors
// are returning atomics, read back with atomic loads) runs lv_plan_children_body.
// kMode 3 (the first levels, the root's above all): the chunks scatter at prefix sums of the
// lv_part_count_lean_kernel counts (kMode 2: reservations lv_part_scan_kernel computed).
template <bool kScatter, int KP, int kS, bool kPrefetch, bool kPfGh = false, bool kPfCol = false,
          typename BinT = uint8_t, int kMode = 0>
__global__ __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(kS <= 8 && !kPrefetch ? 8 : 4, 8)))
void lv_partition_children_kernel(LvParams p, LvBufs b, const BinT* binsT, long long ncol, const int* rows,
                                  const float2* ghp, int* rows_out, float2* gh_out, int build_base, int half,
                                  int dgap, int use_loc, int fused, int maxp, int gh_rows,
                                  unsigned long long* chunk_io, unsigned long long* gsum) {
  if constexpr (kScatter && kPrefetch)
    partition_atomic_body_pf<BinT, kS, kPfGh, kPfCol, kMode>(binsT, ncol, rows, ghp, rows_out, gh_out, b.part_first, b.st + ST_N_SPLIT,
                                          b.st + ST_N_PART, b.part_feat, b.part_thr, b.part_begin, b.part_cnt,
                                          reinterpret_cast<unsigned long long*>(b.left_loc), nullptr, kCurStride,
                                          gh_rows, chunk_io, gsum);
  else
    partition_atomic_body<BinT, kScatter, kS>(binsT, ncol, rows, ghp, rows_out, gh_out, b.part_first, b.st + ST_N_SPLIT,
                                             b.st + ST_N_PART, b.part_feat, b.part_thr, b.part_begin, b.part_cnt,
                                             reinterpret_cast<unsigned long long*>(b.left_loc), nullptr, kCurStride);
  if (!last_block_done(reinterpret_cast<unsigned long long*>(b.left_loc) + (size_t)maxp * kCurStride)) return;
  if constexpr (kMode == 3)  // the split totals the children planning reads from the cursors
    part_split_totals<kPartThreads>(chunk_io, gsum, b.part_first, b.st + ST_N_SPLIT, b.st + ST_N_PART,
                                    reinterpret_cast<unsigned long long*>(b.left_loc), kCurStride);
  lv_plan_children_body<KP, true>(p, b, kCurStride, build_base, half, dgap, use_loc, fused);
}

// one block per chunk (part_count_lean_body)
__global__ __launch_bounds__(kPartThreads) void lv_part_count_lean_kernel(LvBufs b, const uint8_t* binsT, long long ncol,
                                                                          const int* rows, unsigned long long* chunk_io,
                                                                          unsigned long long* gsum) {
  part_count_lean_body(binsT, ncol, rows, b.part_first, b.st + ST_N_SPLIT, b.st + ST_N_PART, b.part_feat, b.part_thr,
                       b.part_begin, b.part_cnt, chunk_io, gsum);
}

// the chunk counts -> reservations + split cursor totals (part_chunk_scan_body)
__global__ __launch_bounds__(kChunkScanThreads) void lv_part_scan_kernel(LvBufs b, unsigned long long* chunk_io) {
  part_chunk_scan_body(chunk_io, b.part_first, b.st + ST_N_SPLIT, b.st + ST_N_PART,
                       reinterpret_cast<unsigned long long*>(b.left_loc), kCurStride);
}

// One GPU: the level's split search (one kNodeThreads block per node item, the node-
// resident split_node_block) and the next level's split planning in ONE launch -- the
// last block to finish runs lv_plan_split_body. Saves a launch per level (the planner's
// ~7 us, mostly launch latency). The SplitOut records are plain stores, so the storing
// thread fences (release) before its block counts itself done and the last block fences
// (acquire: its caches may hold a previous level's records) before planning. Blocks past the device item count only
// count themselves.
template <int KP>
__global__ __launch_bounds__(kNodeThreads) void lv_split_plan_kernel(
    LvParams p, LvBufs b, long long* __restrict__ hist, int B, int F, int Bp, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, GainParams gp, const double* __restrict__ inv_dev,
    unsigned long long* __restrict__ done, int implicit_items) {
  extern __shared__ __attribute__((aligned(16))) longlong2 sh_node[];
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  if ((int)blockIdx.x < b.st[ST_N_SITEMS])  // uniform per block
    split_node_block(hist, B, F, Bp, nbins_f, fmask, f0, b.split_items[blockIdx.x], b.split_out + blockIdx.x, gp,
                     sh_node);
  // release by the one thread that stored this block's record (a fence per wave measured
  // +6 us per launch), acquire by the last block's thread 0 before its barrier
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (!last_block_done(done)) return;
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  lv_plan_split_body<KP>(p, b, 0, implicit_items);
}

// One GPU, gathered levels: the staged histogram's split-K slot reduce and the split search
// in ONE launch (replaces hist_reduce_kernel + split_node_kernel: ~10 us per level, mostly two
// dependent global round trips and a launch). Block (chunk, g8) x build k x z: 256 threads =
// 32 bins x 8 features (one 128-B segment of a staged bin row per thread octet), summing the
// build's items [hist_first[k], hist_first[k + 1]) with split-K over z into the zeroed slot
// (exact int64 memory-side atomics, as hist_reduce_kernel). The LAST block to arrive for
// (k, g8) -- a self-resetting counter -- searches the 8-feature group of the built child and
// of its derived sibling (parent - built, materialised as in split_node_kernel) and writes
// the two group records the level planner combines (split_groups = ceil(F / 8)).
// Ordering: every wave waits for its own atomics (vmcnt) before the block barrier; thread 0
// then releases (agent) before counting the block in, and the last block acquires before it
// reads the slot -- the per-thread fences of a plain-store design cost +6 us per launch
// (profiles/r2_split_plan_fusion.md).
constexpr int kRsThreads = 1024;
constexpr int kRsDirect = 16;            // slots with <= this many items: one z block sums them

// Split search of a built node AND its derived sibling over one group of <= 8 features by one
// 1024-thread block: the built slot (coherent loads: accumulated by memory-side atomics in
// this launch) and the parent slot are streamed once, the derived slot (parent - built) is
// materialised, both transposed into LDS as [node][feature][B + 1]; wave w scans feature
// w & 7 of node w >> 3 (one DPP scan per wave -- the serial per-node, per-feature scans of
// split_node_block with 4 waves took ~10 us per node). Same arithmetic, totals feature and
// tie order as split_node_block, so the records are the split kernel's.
template <int GF>
__device__ __forceinline__ void split_pair_block(long long* __restrict__ hist, int B, int F, int Bp,
                                                 const int* __restrict__ nbins_f, const uint8_t* __restrict__ fmask,
                                                 int f0, int sS, int sP, int sL, SplitOut* __restrict__ outS,
                                                 SplitOut* __restrict__ outL, const GainParams& gp, longlong2* sh,
                                                 int fbeg, int fend, unsigned long long* pr) {
  const int FG = fend - fbeg;  // 1..GF
  constexpr int kW = kRsThreads / kWave;  // 16
  __shared__ float s_chg[kW];
  __shared__ int s_feat[kW], s_a[kW], s_b[kW];
  __shared__ double s_gl[kW], s_hl[kW];
  __shared__ long long s_G[2], s_H[2];
  __shared__ int s_nb[GF];
  __shared__ uint8_t s_fm[GF];
  const int t = threadIdx.x, wid = t >> 6, l = lane_id();
  if (t < FG) { s_nb[t] = nbins_f[fbeg + t]; s_fm[t] = fmask[fbeg + t]; }
  const size_t slot_sz = (size_t)B * F * 2;
  const longlong2* hS = reinterpret_cast<const longlong2*>(hist + (size_t)sS * slot_sz);
  const longlong2* hP = reinterpret_cast<const longlong2*>(hist + (size_t)sP * slot_sz);
  longlong2* hL = reinterpret_cast<longlong2*>(hist + (size_t)sL * slot_sz);
  const int total = B * FG;
  constexpr int kL = (256 * GF + kRsThreads - 1) / kRsThreads;  // entries per thread (B <= 256)
  longlong2 vs[kL], vp[kL];
#pragma unroll
  for (int j = 0; j < kL; ++j) {
    const int i = t + j * kRsThreads;
    if (i < total) {
      const int bin = i / FG, gi = bin * F + fbeg + (i - bin * FG);
      vs[j] = hist_ld2<true>(hS + gi);
      vp[j] = hP[gi];
    }
  }
#pragma unroll
  for (int j = 0; j < kL; ++j) {
    const int i = t + j * kRsThreads;
    if (i < total) {
      const int bin = i / FG, fl = i - bin * FG, gi = bin * F + fbeg + fl;
      const longlong2 d = make_longlong2(vp[j].x - vs[j].x, vp[j].y - vs[j].y);
      hL[gi] = d;  // the derived histogram (the next level subtracts from it)
      sh[fl * Bp + bin] = vs[j];
      sh[(GF + fl) * Bp + bin] = d;
    }
  }
  __syncthreads();
  if (pr && t == 0) pr[3] = wall_clock64();
  // wave w: node w / GF, feature w % GF (waves >= 2G idle in the scan)
  const int node = min(wid / GF, 1), fl = wid < 2 * GF ? wid % GF : GF;
  const longlong2* hn = sh + node * GF * Bp;
  // node totals (exact int64) from the group's copy of f0, else its first feature -- waves 0
  // and 8 compute them for their node
  if (fl == 0 && wid < 2 * GF) {
    const int ft = (f0 >= fbeg && f0 < fend) ? f0 - fbeg : 0;
    const int nb0 = s_nb[ft];
    long long sg = 0, shh = 0;
    for (int bin = l; bin < nb0; bin += kWave) {
      const longlong2 q = hn[ft * Bp + bin];
      sg += q.x;
      shh += q.y;
    }
    const long long Gq = readlane64(dpp_scan_add(sg), kWave - 1), Hq = readlane64(dpp_scan_add(shh), kWave - 1);
    if (l == 0) { s_G[node] = Gq; s_H[node] = Hq; }
  }
  __syncthreads();
  if (pr && t == 0) pr[4] = wall_clock64();
  const long long Gq = s_G[node], Hq = s_H[node];
  const double Gd = (double)Gq * gp.inv_sg, Hd = (double)Hq * gp.inv_sh;
  const float root_gain = (float)calc_gain(Gd, Hd, gp);
  float best_chg = -INFINITY;
  int best_f = 0xffff, best_a = -1, best_b = 0xffff;
  double best_gl = 0.0, best_hl = 0.0;
  if (fl < FG && s_fm[fl])  // wave-uniform
    wave_feature_scan(hn + fl * Bp, s_nb[fl], fbeg + fl, Gq, Hq, root_gain, gp, best_chg, best_f, best_a, best_b,
                      best_gl, best_hl, (pr && wid == 0) ? pr + 8 : nullptr);
  {
    const unsigned u = __float_as_uint(best_chg + 0.0f);
    const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    const unsigned long long key = ((unsigned long long)ord << 32) |
                                   ((unsigned)(0xffff - best_f) << 16) | (unsigned)(0xffff - best_b);
    const unsigned long long kmax = (unsigned long long)readlane64((long long)dpp_max_u64(key), kWave - 1);
    const unsigned long long hit = __ballot(key == kmax);
    const int src = __builtin_ctzll(hit);
    if (l == 0) {
      s_chg[wid] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best_chg), src));
      s_feat[wid] = __builtin_amdgcn_readlane(best_f, src);
      s_a[wid] = __builtin_amdgcn_readlane(best_a, src);
      s_b[wid] = __builtin_amdgcn_readlane(best_b, src);
    }
    const double gl = readlane_f64(best_gl, src), hl = readlane_f64(best_hl, src);
    if (l == 0) { s_gl[wid] = gl; s_hl[wid] = hl; }
  }
  if (pr && t == 0) pr[5] = wall_clock64();
  __syncthreads();
  if (pr && t == 0) pr[6] = wall_clock64();
  if (l == 0 && fl == 0 && wid < 2 * GF) {  // waves 0 and GF: the node's record
    const int w0 = node * GF;
    int bw = w0;
    for (int w = w0 + 1; w < w0 + GF; ++w)
      if (better(s_chg[w], s_feat[w], s_b[w], s_chg[bw], s_feat[bw], s_b[bw])) bw = w;
    SplitOut o;
    o.loss_chg = s_chg[bw];
    o.feat = (s_feat[bw] == 0xffff) ? -1 : s_feat[bw];
    o.bin_a = s_a[bw];
    o.bin_b = (s_b[bw] == 0xffff) ? -1 : s_b[bw];
    o.gl = s_gl[bw];
    o.hl = s_hl[bw];
    o.g = Gd;
    o.h = Hd;
    *(node == 0 ? outS : outL) = o;
  }
}

// One GPU, gathered levels: the staged histogram's split-K slot reduce and the split search
// in ONE launch (replaces hist_reduce_kernel + split_node_kernel). Block (chunk, g8) x build k
// x z: 1024 threads = 128 bins x 8 features (one 128-B segment of a staged bin row per thread
// octet), summing the build's items [hist_first[k], hist_first[k + 1]) with split-K over z
// into the zeroed slot (exact int64 memory-side atomics, as hist_reduce_kernel). The LAST
// block to arrive for (k, g8) -- a self-resetting counter -- searches the 8-feature group of
// the built child and of its derived sibling (split_pair_block) and writes the two group
// records the level planner combines (split_groups = ceil(F / 8)).
// Ordering without fences: every wave waits for its own atomics (vmcnt: performed at the
// memory side) before the block barrier and the counter atomic; the last block reads the
// slot with coherent atomic loads. (An agent-scope release per block -- buffer_wbl2 of the
// XCD's L2 -- cost more than the launch it saves.)
template <int G>
__global__ __launch_bounds__(kRsThreads) void lv_reduce_split_kernel(
    LvBufs b, const long long* __restrict__ staging, long long* __restrict__ hist, int B, int F, int groups32,
    int slot_base, const int* __restrict__ nbins_f, const uint8_t* __restrict__ fmask, int f0, GainParams gp,
    const double* __restrict__ inv_dev, unsigned* __restrict__ counters, int nchunks, int ng,
    unsigned long long* __restrict__ prof, int warm_twice) {
  extern __shared__ __attribute__((aligned(16))) longlong2 sh_rs[];  // tail: [2][8][B + 1]
  __shared__ int s_last;
  // prof (optional, YTK_RS_PROF): per block [entry, counted in, tail start, tail end] wall
  // clocks (100 MHz)
  unsigned long long* pr = prof ? prof + 16 * ((size_t)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x)
                                : nullptr;
  if (pr && threadIdx.x == 0) pr[0] = wall_clock64();
  const int k = (int)blockIdx.y;
  const int nb = b.st[ST_N_BUILD];
  if (k >= nb) return;  // uniform: no build in this slot
  const int lo = b.hist_first[k], cnt = b.hist_first[k + 1] - lo;
  const bool direct = cnt <= kRsDirect;
  if (direct && blockIdx.z != 0) return;  // uniform; such blocks are not counted
  const int Z = direct ? 1 : (int)gridDim.z;
  constexpr int kBins = kRsThreads / G;  // bins per block (G consecutive threads: one bin row segment)
  const int g8 = (int)blockIdx.x / nchunks, ch = (int)blockIdx.x - g8 * nchunks;
  const int t = threadIdx.x, j = t % G;
  const int bin = ch * kBins + t / G, f = g8 * G + j;
  const int slot = slot_base + k;
  if (bin < B && f < F) {
    const int E = B * 32;
    const int fg = f >> 5, l = f & 31;
    const longlong2* st = reinterpret_cast<const longlong2*>(staging) + (size_t)fg * E + bin * 32 + l;
    const size_t istride = (size_t)groups32 * E;
    long long g = 0, h = 0;
    int it = lo + (direct ? 0 : (int)blockIdx.z);
    const int end = lo + cnt;
    for (; it + 7 * Z < end; it += 8 * Z) {
      longlong2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = st[(size_t)(it + u * Z) * istride];
#pragma unroll
      for (int u = 0; u < 8; ++u) { g += v[u].x; h += v[u].y; }
    }
    for (; it < end; it += Z) {
      const longlong2 v = st[(size_t)it * istride];
      g += v.x;
      h += v.y;
    }
    if (g | h) {
      unsigned long long* o = reinterpret_cast<unsigned long long*>(hist + (((size_t)slot * B + bin) * F + f) * 2);
      atomicAdd(o, (unsigned long long)g);
      atomicAdd(o + 1, (unsigned long long)h);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // this wave's atomics have been performed (memory side)
  __syncthreads();
  if (t == 0) {
    unsigned* c = counters + (size_t)k * ng + g8;
    const unsigned target = (unsigned)(nchunks * Z);
    const bool last = atomicAdd(c, 1u) == target - 1;
    if (last) atomicExch(c, 0u);  // self-resetting for the next level / tree
    s_last = last ? 1 : 0;
    if (pr) pr[1] = wall_clock64();
  }
  __syncthreads();
  if (!s_last) return;
  if (pr && threadIdx.x == 0) pr[2] = wall_clock64();
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  const int4 d = b.split_items[nb + k];  // (derived slot, parent slot, built slot, 1)
  const int fbeg = g8 * G, fend = min(F, fbeg + G);
  if (pr && warm_twice) {  // YTK_RS_PROF_TWICE: search twice, time the warm second pass (idempotent)
    split_pair_block<G>(hist, B, F, B + 1, nbins_f, fmask, f0, slot, d.y, d.x, b.split_out + (size_t)k * ng + g8,
                        b.split_out + (size_t)(nb + k) * ng + g8, gp, sh_rs, fbeg, fend, nullptr);
    __syncthreads();
    if (threadIdx.x == 0) pr[2] = wall_clock64();
  }
  split_pair_block<G>(hist, B, F, B + 1, nbins_f, fmask, f0, slot, d.y, d.x, b.split_out + (size_t)k * ng + g8,
                      b.split_out + (size_t)(nb + k) * ng + g8, gp, sh_rs, fbeg, fend, pr);
  if (pr && threadIdx.x == 0) pr[7] = wall_clock64();
}

// Bin-threshold arrays used by the fused score/gradient kernel.
__device__ __forceinline__ void lv_finalize_body(const LvBufs& b, int max_nodes) {
  const int nn = b.st[ST_NUM_NODES];
  for (int i = threadIdx.x; i < max_nodes; i += blockDim.x) {
    if (i < nn) {
      const DNode& n = b.nodes[i];
      const bool leaf = n.is_leaf || n.left < 0;
      b.tfeat[i] = leaf ? -1 : n.feat;
      b.tthr[i] = (n.bin_a + n.bin_b) >> 1;
      b.tleft[i] = n.left;
      b.tright[i] = n.right;
      b.tval[i] = n.value;
    } else {
      b.tfeat[i] = -1;
      b.tthr[i] = 0;
      b.tleft[i] = -1;
      b.tright[i] = -1;
      b.tval[i] = 0.f;
    }
  }
}

__global__ void lv_finalize_kernel(LvBufs b, int max_nodes) { lv_finalize_body(b, max_nodes); }

// Raw-feature version of the finished tree for test-set scoring:
// cond = mean (0.5*(v_a+v_b)) or median split of the candidate values,
// default child = left iff fill < cond (Tree.java:293-309, 357-375).
__device__ __forceinline__ void lv_raw_tree_body(const LvBufs& b, int max_nodes, const float* __restrict__ cand,
                                                 const int* __restrict__ coff, const float* __restrict__ fill,
                                                 int split_median, int* __restrict__ nfeat,
                                                 float* __restrict__ nthr, int* __restrict__ nleft,
                                                 int* __restrict__ nright, uint8_t* __restrict__ ndefl,
                                                 float* __restrict__ nval) {
  const int nn = b.st[ST_NUM_NODES];
  for (int i = threadIdx.x; i < max_nodes; i += blockDim.x) {
    if (i >= nn) {
      nfeat[i] = -1; nthr[i] = 0.f; nleft[i] = -1; nright[i] = -1; ndefl[i] = 1; nval[i] = 0.f;
      continue;
    }
    const DNode& n = b.nodes[i];
    const bool leaf = n.is_leaf || n.left < 0;
    nfeat[i] = leaf ? -1 : n.feat;
    nleft[i] = n.left;
    nright[i] = n.right;
    nval[i] = n.value;
    float cond = 0.f;
    if (!leaf) {
      const float* c = cand + coff[n.feat];
      if (!split_median) {
        cond = 0.5f * (c[n.bin_a] + c[n.bin_b]);
      } else {
        const int s = n.bin_a + n.bin_b;
        cond = (s % 2 == 0) ? c[s / 2] : 0.5f * (c[(s - 1) / 2] + c[(s + 1) / 2]);
      }
    }
    nthr[i] = cond;
    ndefl[i] = leaf ? 1 : (fill ? (fill[n.feat] < cond ? 1 : 0) : 1);
  }
}

__global__ void lv_raw_tree_kernel(LvBufs b, int max_nodes, const float* __restrict__ cand,
                                   const int* __restrict__ coff, const float* __restrict__ fill,
                                   int split_median, int* __restrict__ nfeat,
                                   float* __restrict__ nthr, int* __restrict__ nleft,
                                   int* __restrict__ nright, uint8_t* __restrict__ ndefl,
                                   float* __restrict__ nval) {
  lv_raw_tree_body(b, max_nodes, cand, coff, fill, split_median, nfeat, nthr, nleft, nright, ndefl, nval);
}

struct LvRawArgs {
  const float* cand;
  const int* coff;
  const float* fill;
  int split_median;
  int* nfeat;
  float* nthr;
  int* nleft;
  int* nright;
  uint8_t* ndefl;
  float* nval;
};

// Tree tail in ONE single-block launch (each of these was its own ~5-us launch at the end of
// every tree): the deferred last level's children planning (children = 1), then the
// bin-threshold arrays (finalize) and the raw-threshold tree for the test-set pass. Same
// block, so a workgroup barrier orders the node-table writes before the reads.
__global__ __launch_bounds__(kPlanThreads) void lv_tail_kernel(LvParams p, LvBufs b, int children, int build_base,
                                                               int half, int dgap, int use_loc, int fused,
                                                               int max_nodes, LvRawArgs r) {
  if (children) {
    lv_plan_children_body<kMaxPend, false>(p, b, 1, build_base, half, dgap, use_loc, fused);
    __syncthreads();
  }
  lv_finalize_body(b, max_nodes);
  if (r.nfeat)
    lv_raw_tree_body(b, max_nodes, r.cand, r.coff, r.fill, r.split_median, r.nfeat, r.nthr, r.nleft, r.nright,
                     r.ndefl, r.nval);
}

// Fixed-point scales from the (all-reduced) max |g|, |h| and global row count.
__global__ void lv_scales_kernel(const float* __restrict__ mx, const long long* __restrict__ cnt,
                                 float* __restrict__ scales, double* __restrict__ inv_scales) {
  lv_scales_body(mx, cnt, scales, inv_scales);
}

}  // namespace ytk

using namespace ytk;

static LvBufs make_bufs(const uintptr_t* a) {
  LvBufs b;
  b.st = (int*)a[0];
  b.nodes = (DNode*)a[1];
  b.pending = (int*)a[2];
  b.next_pending = (int*)a[3];
  b.split_nid = (int*)a[4];
  b.split_snap = (int*)a[5];
  b.part_items = (int4*)a[6];
  b.part_feat = (int*)a[7];
  b.part_thr = (int*)a[8];
  b.part_begin = (int*)a[9];
  b.part_first = (int*)a[10];
  b.part_nblk = (int*)a[11];
  b.part_counts = (int*)a[12];
  b.left_loc = (long long*)a[13];
  b.left_glob = (long long*)a[14];
  b.hist_items = (int4*)a[15];
  b.split_items = (int4*)a[16];
  b.item_nid = (int*)a[17];
  b.split_out = (SplitOut*)a[18];
  b.tfeat = (int*)a[19];
  b.tthr = (int*)a[20];
  b.tleft = (int*)a[21];
  b.tright = (int*)a[22];
  b.tval = (float*)a[23];
  b.root_cnt = (long long*)a[24];
  b.part_cnt = (int*)a[25];
  b.hist_first = (int*)a[26];
  return b;
}

static LvParams make_params(const int* ip, const float* fp) {
  LvParams p;
  p.max_depth = ip[0];
  p.max_leaf_cnt = ip[1];
  p.min_split_samples = ip[2];
  p.hist_target = ip[3];
  p.part_target = ip[4];
  p.min_rows = ip[5];
  p.part_chunk = ip[6];
  p.split_groups = max(1, ip[7]);
  p.small_only = ip[8];
  p.min_split_loss = fp[0];
  p.mcw = fp[1];
  p.l1 = fp[2];
  p.l2 = fp[3];
  p.max_abs_leaf = fp[4];
  p.lr = fp[5];
  return p;
}

static int plan_fast_off() {  // YTK_PLAN_FAST=0: the planners' general paths (default: fast paths)
  const char* e = getenv("YTK_PLAN_FAST");  // read per launch (~0.1 us): tests toggle it
  return (e && e[0] == '0') ? 2 : 0;
}

extern "C" {

// which: 0 init, 1 plan_split (arg1 = fused: patch the previous level's cnt_global from
//        left_glob; 2: line-spaced cursors of the fused partition), 3 plan_children(arg0=build_base, arg1=half | ncs<<14 | fused<<29 |
//        use_loc<<30; derived slots start at build_base + half + ncs),
//        4 finalize(arg0=max_nodes)
void ytk_lv_step(int which, const uintptr_t* ptrs, const int* ip, const float* fp, int arg0,
                 int arg1, uintptr_t stream) {
  LvParams p = make_params(ip, fp);
  LvBufs b = make_bufs(ptrs);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (which) {
    case 0:
      hipLaunchKernelGGL(lv_init_kernel, dim3(1), dim3(kPlanThreads), 0, s, p, b, (const float*)nullptr,
                         (float*)nullptr, (double*)nullptr);
      break;
    case 1:  // arg0 = 1: no partition work list (single-pass partition maps blocks itself)
      hipLaunchKernelGGL(lv_plan_split_kernel, dim3(1), dim3(kPlanThreads), 0, s, p, b, arg1, arg0 | plan_fast_off());
      break;
    case 3:
      hipLaunchKernelGGL(lv_plan_children_kernel, dim3(1), dim3(kPlanThreads), 0, s, p, b, arg0,
                         arg1 & 0x3fff, (arg1 & 0x3fff) + ((arg1 >> 14) & 0x3fff), ((arg1 >> 30) & 1) | plan_fast_off(),
                         (arg1 >> 29) & 1);
      break;
    case 4: hipLaunchKernelGGL(lv_finalize_kernel, dim3(1), dim3(256), 0, s, b, arg0); break;
    default: throw std::runtime_error("bad lv step");
  }
  YTK_LAUNCH_CHECK();
}

// Fused partition + children planning (one GPU, uint8 bins): count_only = last level;
// arg0 / arg1 as ytk_lv_step(3).
void ytk_lv_partition_children(const uintptr_t* ptrs, const int* ip, const float* fp, uintptr_t binsT, long long ncol,
                               uintptr_t rows, uintptr_t ghp, uintptr_t rows_out, uintptr_t gh_out, int max_blocks,
                               int count_only, int arg0, int arg1, int maxp, uintptr_t stream, int bin_bytes,
                               int gh_rows, uintptr_t chunk_io) {
  // chunk_io (optional, >= max_blocks + max_blocks / 32 + 1 u64, the group sums zeroed once;
  // for levels of <= kChunkScanMaxSplits splits): the
  // chunks reserve through a count pass + one-block scan instead of the split cursor atomics
  // gh_rows: ghp is row-indexed (pipelined bodies only: the unpipelined ones read (g, h) by
  // position)
  LvParams p = make_params(ip, fp);
  LvBufs b = make_bufs(ptrs);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int half = arg1 & 0x3fff, dgap = (arg1 & 0x3fff) + ((arg1 >> 14) & 0x3fff);
  const int use_loc = ((arg1 >> 30) & 1) | plan_fast_off(), fused = (arg1 >> 29) & 1;
  const dim3 grid(std::max(1, std::min(max_blocks, kPartGrid)));
  if (bin_bytes == 2) {
    // uint16 bins (wide): one configuration -- 2048-row chunks, the pipelined body with the
    // next chunk's row ids and (g, h) in flight
    if (p.part_chunk != kPartThreads * kAtomSub)
      throw std::invalid_argument("lv_partition_children: uint16 bins take 2048-row chunks");
#define YTK_LVPC16(SC, KP)                                                                                   \
  hipLaunchKernelGGL((lv_partition_children_kernel<SC, KP, kAtomSub, SC, SC, false, uint16_t>), grid,        \
                     dim3(kPartThreads), 0, s, p, b, (const uint16_t*)binsT, ncol, (const int*)rows,        \
                     (const float2*)ghp, (int*)rows_out, (float2*)gh_out, arg0, half, dgap, use_loc, fused, maxp, \
                     gh_rows, nullptr, nullptr)
    if (maxp <= 64) {
      if (count_only) YTK_LVPC16(false, 64); else YTK_LVPC16(true, 64);
    } else if (maxp <= 512) {
      if (count_only) YTK_LVPC16(false, 512); else YTK_LVPC16(true, 512);
    } else {
      if (count_only) YTK_LVPC16(false, kMaxPend); else YTK_LVPC16(true, kMaxPend);
    }
#undef YTK_LVPC16
    YTK_LAUNCH_CHECK();
    return;
  }
  if (p.part_chunk != kPartThreads * kAtomSub && p.part_chunk != kPartThreads * 2 * kAtomSub &&
      p.part_chunk != kPartThreads * kAtomSub / 2)
    throw std::invalid_argument("lv_partition_children: part_chunk must be 1024, 2048 or 4096");
  const bool wide = p.part_chunk == kPartThreads * 2 * kAtomSub;
  const bool narrow = p.part_chunk == kPartThreads * kAtomSub / 2;  // small shards: 2x the blocks
  // software-pipelined partition: the next chunk's row ids and (g, h) in flight during this
  // chunk's rank / reserve / scatter. Measured (profiles/r2_partition_chunk.md): off
  // 1.474-1.496, row ids only (YTK_PART_PREFETCH=1) 1.430-1.441, row ids + (g, h) (=2,
  // 87 VGPRs) 1.393 ms/tree; YTK_PART_PREFETCH=0: off. Default (unset or 3): also the next
  // chunk's split-feature bytes, gathered once its row ids have arrived (after this chunk's
  // cursor reservation): 1.287-1.304 -> 1.245-1.250 ms/tree, 500 trees 1.146 -> 1.130
  // (profiles/r6/level_knobs/); the 1/8 shard is unchanged (0.390)
  const char* pf = getenv("YTK_PART_PREFETCH");  // read per launch (~0.1 us): tests toggle it
  const bool prefetch = !(pf && pf[0] == '0');
  const bool pf_gh = !(pf && (pf[0] == '0' || pf[0] == '1'));
  const bool pf_col = !pf || pf[0] == '3';
  if (gh_rows && (!prefetch || count_only))
    throw std::invalid_argument("lv_partition_children: row-indexed (g, h) needs the pipelined scatter body");
  if (chunk_io && !count_only && prefetch && pf_col && !wide && !narrow) {
    // count pass (same chunks, same split-feature gathers, no scatter) -> scan -> scatter
    unsigned long long* cio = reinterpret_cast<unsigned long long*>(chunk_io);
    // group sums past the counts (zero between levels: the partition's last block re-zeroes)
    unsigned long long* gsum = cio + std::max(1, max_blocks);
    // one block per chunk: max_blocks bounds the level's chunks (extra blocks return at once)
    // YTK_PART_SCAN_KERNEL=1: a one-block scan launch between the two (mode 2) instead of each
    // partition block summing its chunk's prefix (mode 3; the count pass adds the group sums)
    const char* sk = getenv("YTK_PART_SCAN_KERNEL");
    const bool scan_launch = sk && sk[0] == '1';
    hipLaunchKernelGGL(lv_part_count_lean_kernel, dim3(std::max(1, max_blocks)), dim3(kPartThreads), 0, s, b,
                       (const uint8_t*)binsT, ncol, (const int*)rows, cio, scan_launch ? nullptr : gsum);
    if (scan_launch) hipLaunchKernelGGL(lv_part_scan_kernel, dim3(1), dim3(kChunkScanThreads), 0, s, b, cio);
#define YTK_LVPC_SCAN1(KP, MODE)                                                                                \
  hipLaunchKernelGGL((lv_partition_children_kernel<true, KP, kAtomSub, true, true, true, uint8_t, MODE>), grid, \
                     dim3(kPartThreads), 0, s, p, b, (const uint8_t*)binsT, ncol, (const int*)rows,             \
                     (const float2*)ghp, (int*)rows_out, (float2*)gh_out, arg0, half, dgap, use_loc, fused, maxp, \
                     gh_rows, cio, gsum)
#define YTK_LVPC_SCAN(KP)                                                                                       \
  do {                                                                                                          \
    if (scan_launch) YTK_LVPC_SCAN1(KP, 2);                                                                     \
    else YTK_LVPC_SCAN1(KP, 3);                                                                                 \
  } while (0)
    if (maxp <= 64) YTK_LVPC_SCAN(64);
    else if (maxp <= 512) YTK_LVPC_SCAN(512);
    else YTK_LVPC_SCAN(kMaxPend);
#undef YTK_LVPC_SCAN
#undef YTK_LVPC_SCAN1
    YTK_LAUNCH_CHECK();
    return;
  }
#define YTK_LVPC4(SC, KP, S, PF, PG, PC)                                                                      \
  hipLaunchKernelGGL((lv_partition_children_kernel<SC, KP, S, PF, PG, PC>), grid, dim3(kPartThreads), 0, s, p, b,            \
                     (const uint8_t*)binsT, ncol, (const int*)rows, (const float2*)ghp, (int*)rows_out,          \
                     (float2*)gh_out, arg0, half, dgap, use_loc, fused, maxp, gh_rows, nullptr, nullptr)
#define YTK_LVPC2(SC, KP, S, PF)                                                  \
  do {                                                                            \
    if ((PF) && pf_col) YTK_LVPC4(SC, KP, S, PF, true, true);                     \
    else if ((PF) && pf_gh) YTK_LVPC4(SC, KP, S, PF, true, false);                \
    else YTK_LVPC4(SC, KP, S, PF, false, false);                                  \
  } while (0)
#define YTK_LVPC1(SC, KP, S) do { if (prefetch && (SC)) YTK_LVPC2(SC, KP, S, true); else YTK_LVPC2(SC, KP, S, false); } while (0)
#define YTK_LVPC(SC, KP)                                                          \
  do {                                                                            \
    if (wide) YTK_LVPC1(SC, KP, 2 * kAtomSub);                                    \
    else if (narrow) YTK_LVPC1(SC, KP, kAtomSub / 2);                             \
    else YTK_LVPC1(SC, KP, kAtomSub);                                             \
  } while (0)
  if (maxp <= 64) {
    if (count_only) YTK_LVPC(false, 64); else YTK_LVPC(true, 64);
  } else if (maxp <= 512) {
    if (count_only) YTK_LVPC(false, 512); else YTK_LVPC(true, 512);
  } else {
    if (count_only) YTK_LVPC(false, kMaxPend); else YTK_LVPC(true, kMaxPend);
  }
#undef YTK_LVPC
#undef YTK_LVPC1
#undef YTK_LVPC2
#undef YTK_LVPC4
  YTK_LAUNCH_CHECK();
}

// Fused split search + next-level split planning (one GPU, all-reduce-free). Falls back to
// the two launches (split_find + plan_split) when the node-resident kernel's LDS (plus
// the planner's) does not fit. fp: [6] LvParams floats; gpf: mcw, l1, l2, max_abs_leaf.
void ytk_split_find(uintptr_t hist, int B, int F, uintptr_t nbins_f, uintptr_t fmask, int f0, uintptr_t items,
                    int nitems, uintptr_t out, float mcw, float l1, float l2, float max_abs_leaf, double inv_sg,
                    double inv_sh, uintptr_t nitems_dev, uintptr_t inv_dev, uintptr_t part, uintptr_t counters,
                    uintptr_t stream);

void ytk_lv_split_plan(const uintptr_t* ptrs, const int* ip, const float* fp, uintptr_t hist, int B, int F,
                       uintptr_t nbins_f, uintptr_t fmask, int f0, int nitems, const float* gpf, uintptr_t inv_dev,
                       uintptr_t part, uintptr_t counters, int implicit_items, int maxp, uintptr_t stream) {
  LvParams p = make_params(ip, fp);
  LvBufs b = make_bufs(ptrs);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int Bp = B + 1;
  const size_t node_lds = (size_t)F * Bp * sizeof(long long) * 2;
  const size_t plan_lds = 2 * sizeof(int) * (size_t)(maxp <= 64 ? 64 : maxp <= 512 ? 512 : kMaxPend) + 4096;
  const bool fits = node_lds <= kNodeLdsMax && node_lds + plan_lds + 4096 <= 160 * 1024 && B <= 4 * kWave &&
                    B * F <= kNodeLoads * kNodeThreads && F <= kNodeMaxF && F < 0xffff;
  if (!fits) {
    ytk_split_find(hist, B, F, nbins_f, fmask, f0, (uintptr_t)b.split_items, nitems, (uintptr_t)b.split_out,
                   gpf[0], gpf[1], gpf[2], gpf[3], 1.0, 1.0, (uintptr_t)(b.st + ST_N_SITEMS), inv_dev, part,
                   counters, stream);
    hipLaunchKernelGGL(lv_plan_split_kernel, dim3(1), dim3(kPlanThreads), 0, s, p, b, 0, implicit_items);
    YTK_LAUNCH_CHECK();
    return;
  }
  GainParams gp{gpf[0], gpf[1], gpf[2], gpf[3], 1.0, 1.0};
  unsigned long long* done = reinterpret_cast<unsigned long long*>(b.left_loc) + (size_t)maxp * kCurStride;
#define YTK_LVSP(KP)                                                                                        \
  hipLaunchKernelGGL((lv_split_plan_kernel<KP>), dim3(std::max(1, nitems)), dim3(kNodeThreads), node_lds, s, p, b, \
                     (long long*)hist, B, F, Bp, (const int*)nbins_f, (const uint8_t*)fmask, f0, gp,               \
                     (const double*)inv_dev, done, implicit_items)
  if (maxp <= 64) YTK_LVSP(64);
  else if (maxp <= 512) YTK_LVSP(512);
  else YTK_LVSP(kMaxPend);
#undef YTK_LVSP
  YTK_LAUNCH_CHECK();
}

// Staged histogram reduce + split search of a gathered level (lv_reduce_split_kernel): nslots
// builds from slot_base; records [item][ceil(F / 8)]; counters: nslots * ceil(F / 8) zeroed
// (self-resetting) words; zs: split-K factor.
void ytk_lv_reduce_split(const uintptr_t* ptrs, uintptr_t staging, uintptr_t hist, int B, int F, int slot_base,
                         int nslots, uintptr_t nbins_f, uintptr_t fmask, int f0, const float* gpf, uintptr_t inv_dev,
                         uintptr_t counters, int zs, uintptr_t stream, uintptr_t prof, int group) {
  if (nslots <= 0) return;
  if (B > 256 || F > kNodeMaxF) throw std::invalid_argument("lv_reduce_split: B <= 256 and F <= 256 only");
  LvBufs b = make_bufs(ptrs);
  if (!b.hist_first) throw std::invalid_argument("lv_reduce_split: hist_first is required");
  const int groups32 = (F + 31) / 32;
  GainParams gp{gpf[0], gpf[1], gpf[2], gpf[3], 1.0, 1.0};
  const int twice = prof && getenv("YTK_RS_PROF_TWICE") ? 1 : 0;
#define YTK_RS(GS)                                                                                                \
  do {                                                                                                            \
    const int nchunks = (B + kRsThreads / GS - 1) / (kRsThreads / GS), ng = (F + GS - 1) / GS;                    \
    const size_t lds = (size_t)2 * GS * (B + 1) * sizeof(longlong2);                                             \
    hipLaunchKernelGGL((lv_reduce_split_kernel<GS>), dim3(nchunks * ng, nslots, std::max(1, zs)), dim3(kRsThreads), \
                       lds, reinterpret_cast<hipStream_t>(stream), b, (const long long*)staging, (long long*)hist, B, F, \
                       groups32, slot_base, (const int*)nbins_f, (const uint8_t*)fmask, f0, gp, (const double*)inv_dev, \
                       (unsigned*)counters, nchunks, ng, (unsigned long long*)prof, twice);                          \
  } while (0)
  if (group == 8) YTK_RS(8);
  else if (group == 4) YTK_RS(4);
  else if (group == 2) YTK_RS(2);
  else throw std::invalid_argument("lv_reduce_split: group must be 2, 4 or 8");
#undef YTK_RS
  YTK_LAUNCH_CHECK();
}

void ytk_lv_raw_tree(const uintptr_t* ptrs, int max_nodes, uintptr_t cand, uintptr_t coff,
                     uintptr_t fill, int split_median, uintptr_t nfeat, uintptr_t nthr,
                     uintptr_t nleft, uintptr_t nright, uintptr_t ndefl, uintptr_t nval,
                     uintptr_t stream) {
  LvBufs b = make_bufs(ptrs);
  hipLaunchKernelGGL(lv_raw_tree_kernel, dim3(1), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), b, max_nodes, (const float*)cand,
                     (const int*)coff, (const float*)fill, split_median, (int*)nfeat, (float*)nthr,
                     (int*)nleft, (int*)nright, (uint8_t*)ndefl, (float*)nval);
  YTK_LAUNCH_CHECK();
}


// lv_step(0) with the tree's fixed-point scales computed by the same launch
void ytk_lv_init_scales(const uintptr_t* ptrs, const int* ip, const float* fp, uintptr_t mx, uintptr_t scales,
                        uintptr_t inv_scales, uintptr_t stream) {
  LvParams p = make_params(ip, fp);
  LvBufs b = make_bufs(ptrs);
  hipLaunchKernelGGL(lv_init_kernel, dim3(1), dim3(kPlanThreads), 0, reinterpret_cast<hipStream_t>(stream), p, b,
                     (const float*)mx, (float*)scales, (double*)inv_scales);
  YTK_LAUNCH_CHECK();
}

// Tree tail (lv_tail_kernel): children = 1 runs lv_step(3)'s planning first (arg0 / arg1 as
// there); raw outputs optional (nfeat == 0: finalize only).
void ytk_lv_tail(const uintptr_t* ptrs, const int* ip, const float* fp, int children, int arg0, int arg1,
                 int max_nodes, uintptr_t cand, uintptr_t coff, uintptr_t fill, int split_median, uintptr_t nfeat,
                 uintptr_t nthr, uintptr_t nleft, uintptr_t nright, uintptr_t ndefl, uintptr_t nval,
                 uintptr_t stream) {
  LvParams p = make_params(ip, fp);
  LvBufs b = make_bufs(ptrs);
  LvRawArgs r{(const float*)cand, (const int*)coff, (const float*)fill, split_median, (int*)nfeat, (float*)nthr,
              (int*)nleft, (int*)nright, (uint8_t*)ndefl, (float*)nval};
  hipLaunchKernelGGL(lv_tail_kernel, dim3(1), dim3(kPlanThreads), 0, reinterpret_cast<hipStream_t>(stream), p, b,
                     children, arg0, arg1 & 0x3fff, (arg1 & 0x3fff) + ((arg1 >> 14) & 0x3fff),
                     ((arg1 >> 30) & 1) | plan_fast_off(), (arg1 >> 29) & 1, max_nodes, r);
  YTK_LAUNCH_CHECK();
}

void ytk_lv_scales(uintptr_t mx, uintptr_t cnt, uintptr_t scales, uintptr_t inv_scales,
                   uintptr_t stream) {
  hipLaunchKernelGGL(lv_scales_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     (const float*)mx, (const long long*)cnt, (float*)scales, (double*)inv_scales);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
