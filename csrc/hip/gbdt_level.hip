// GPU-resident level-wise tree construction (gfx950).
//
// Reference control flow: J/optimizer/gbdt/DataParallelTreeMaker.java make() :229-295
// -- FIFO expansion queue (level-wise), leaf conditions at pop time (lossChg <=
// min_split_loss, depth == max_depth, leaves == max_leaf_cnt, samples <
// min_split_samples), children made leaves right away when their depth reaches
// max_depth / the leaf budget is used / both children are below min_split_samples,
// smaller child histogram + sibling subtraction, canSplit (UpdateStrategy:50-53).
//
// MI355X design: the sequential decisions of a level (<= 2^depth nodes) run in a
// one-lane "planner" kernel that also writes the work lists (partition chunks,
// histogram chunks, split items) and their counts into device memory. The heavy
// kernels (partition / histogram / split) are launched with a FIXED maximal grid
// and read their item count from device memory (blocks past it exit at once).
// Hence a whole tree is a fixed, host-known launch sequence: no device->host
// synchronisation inside a tree (and multi-GPU all-reduces operate on fixed-size
// slabs, enqueued on the same stream).
#include "common.h"

namespace ytk {

struct SplitOut {
  float loss_chg;
  int feat;
  int bin_a;
  int bin_b;
  double gl, hl;
  double g, h;
};

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
static_assert(sizeof(DNode) == 88, "DNode layout");

enum {
  ST_NUM_NODES = 0, ST_NUM_LEAF, ST_N_PENDING, ST_N_SPLIT, ST_N_PART, ST_N_HIST,
  ST_N_SITEMS, ST_N_BUILD, ST_WORDS = 16
};

struct LvParams {
  int max_depth, max_leaf_cnt, min_split_samples;
  float min_split_loss, mcw, l1, l2, max_abs_leaf, lr;
  int hist_target, part_target, min_rows;
};

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
  long long* left_loc;   // per split
  long long* left_glob;  // per split (all-reduced)
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
};

__device__ __forceinline__ double thr_l1d(double w, double lam) {
  if (w > lam) return w - lam;
  if (w < -lam) return w + lam;
  return 0.0;
}

__device__ float leaf_value(double g, double h, const LvParams& p) {
  double v = 0.0;
  if (h >= (double)p.mcw) {
    v = (p.l1 == 0.f) ? -g / (h + p.l2) : -thr_l1d(g, p.l1) / (h + p.l2);
    if (p.max_abs_leaf > 0.f) {
      if (v > p.max_abs_leaf) v = p.max_abs_leaf;
      else if (v < -p.max_abs_leaf) v = -p.max_abs_leaf;
    }
  }
  return (float)v * p.lr;  // (float) nodeValue * learning_rate
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

__device__ void emit_chunks(int4* items, int& k, int tag, int b, int c, int ch, bool blk_index) {
  for (int j = 0; j * ch < c; ++j) {
    const int s = b + j * ch;
    items[k++] = make_int4(tag, s, min(s + ch, b + c), blk_index ? j : 0);
  }
}

// Root: node 0 holds all (local) rows; one build item; chunked histogram work.
__global__ void lv_init_kernel(LvParams p, LvBufs b) {
  if (threadIdx.x != 0) return;
  const int n_local = (int)b.root_cnt[0];
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
  const int ch = max(p.min_rows, (n_local + p.hist_target - 1) / max(1, p.hist_target));
  int k = 0;
  emit_chunks(b.hist_items, k, 0, 0, n_local, ch, false);
  st[ST_N_HIST] = k;
  st[ST_N_BUILD] = 1;
  b.split_items[0] = make_int4(0, 0, 0, 0);
  b.item_nid[0] = 0;
  st[ST_N_SITEMS] = 1;
}

// Apply split results to the node table, then pop the level's nodes in FIFO order.
__global__ void lv_plan_split_kernel(LvParams p, LvBufs b) {
  if (threadIdx.x != 0) return;
  int* st = b.st;
  const double mcw2 = (double)p.mcw * 2.0;
  for (int i = 0; i < st[ST_N_SITEMS]; ++i) {
    DNode& n = b.nodes[b.item_nid[i]];
    const SplitOut& o = b.split_out[i];
    n.G = o.g;
    n.H = o.h;
    n.gl = o.gl;
    n.hl = o.hl;
    n.feat = o.feat;
    n.bin_a = o.bin_a;
    n.bin_b = o.bin_b;
    n.loss_chg = o.loss_chg;
    if (!(n.H >= mcw2 && n.cnt_global >= (long long)p.min_split_samples)) {  // canSplit
      n.loss_chg = -INFINITY;
      n.feat = -1;
    }
  }
  int num_nodes = st[ST_NUM_NODES], num_leaf = st[ST_NUM_LEAF], nsplit = 0;
  long long total = 0;
  for (int i = 0; i < st[ST_N_PENDING]; ++i) {
    const int id = b.pending[i];
    DNode& n = b.nodes[id];
    const bool leaf = !(n.loss_chg > p.min_split_loss) ||
                      (p.max_depth >= 0 && p.max_depth == n.depth) ||
                      (p.max_leaf_cnt > 0 && p.max_leaf_cnt == num_leaf) ||
                      (p.min_split_samples > 0 && n.cnt_global < p.min_split_samples);
    if (leaf) {
      n.is_leaf = 1;
      n.value = leaf_value(n.G, n.H, p);
      continue;
    }
    n.is_leaf = 0;
    n.left = num_nodes;
    n.right = num_nodes + 1;
    num_nodes += 2;
    num_leaf += 1;
    b.split_nid[nsplit] = id;
    b.split_snap[nsplit] = num_leaf;
    ++nsplit;
    total += n.cnt_local;
  }
  st[ST_NUM_NODES] = num_nodes;
  st[ST_NUM_LEAF] = num_leaf;
  st[ST_N_SPLIT] = nsplit;
  const int ch = max((long long)p.min_rows, (total + p.part_target - 1) / max(1, p.part_target));
  int k = 0;
  for (int s = 0; s < nsplit; ++s) {
    const DNode& n = b.nodes[b.split_nid[s]];
    b.part_feat[s] = n.feat;
    b.part_thr[s] = (n.bin_a + n.bin_b) >> 1;  // bin <= floor((a+b)/2) <=> bin < (a+b)/2 rule
    b.part_begin[s] = n.begin;
    b.part_first[s] = k;
    emit_chunks(b.part_items, k, s, n.begin, n.cnt_local, ch, true);
    b.part_nblk[s] = k - b.part_first[s];
  }
  st[ST_N_PART] = k;
}

// Per-split left counts from the partition block counts (local; the host
// all-reduces left_glob across ranks when distributed).
__global__ void lv_sum_counts_kernel(LvBufs b, int copy_glob) {
  const int nsplit = b.st[ST_N_SPLIT];
  for (int s = threadIdx.x; s < nsplit; s += blockDim.x) {
    long long c = 0;
    const int f = b.part_first[s], n = b.part_nblk[s];
    for (int j = 0; j < n; ++j) c += b.part_counts[f + j];
    b.left_loc[s] = c;
    if (copy_glob) b.left_glob[s] = c;
  }
}

// Children of this level's splits: segments, terminal check, build / derive lists.
// build_base: first histogram slot of this level, half: slots reserved for builds.
__global__ void lv_plan_children_kernel(LvParams p, LvBufs b, int build_base, int half) {
  if (threadIdx.x != 0) return;
  int* st = b.st;
  const int nsplit = st[ST_N_SPLIT];
  int nb = 0, npend = 0;
  long long total = 0;
  int nd = 0;
  for (int s = 0; s < nsplit; ++s) {
    DNode& P = b.nodes[b.split_nid[s]];
    DNode& L = b.nodes[P.left];
    DNode& R = b.nodes[P.right];
    const long long lloc = b.left_loc[s], lglob = b.left_glob[s];
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
      continue;
    }
    DNode& small = (L.cnt_global < R.cnt_global) ? L : R;
    DNode& large = (L.cnt_global < R.cnt_global) ? R : L;
    const int small_id = (L.cnt_global < R.cnt_global) ? P.left : P.right;
    const int large_id = (L.cnt_global < R.cnt_global) ? P.right : P.left;
    small.slot = build_base + nb;
    large.slot = build_base + half + nd;
    b.split_items[nb] = make_int4(small.slot, 0, 0, 0);
    b.item_nid[nb] = small_id;
    // derived items are appended after all builds (indices fixed below)
    b.next_pending[npend++] = P.left;
    b.next_pending[npend++] = P.right;
    total += small.cnt_local;
    ++nb;
    ++nd;
    (void)large_id;
  }
  // derived items: second pass keeps build items contiguous
  int di = nb;
  for (int s = 0; s < nsplit; ++s) {
    const DNode& P = b.nodes[b.split_nid[s]];
    const DNode& L = b.nodes[P.left];
    const DNode& R = b.nodes[P.right];
    if (L.slot < 0 && R.slot < 0) continue;  // terminal pair
    const bool left_small = L.cnt_global < R.cnt_global;
    const DNode& small = left_small ? L : R;
    const DNode& large = left_small ? R : L;
    b.split_items[di] = make_int4(large.slot, P.slot, small.slot, 1);
    b.item_nid[di] = left_small ? P.right : P.left;
    ++di;
  }
  for (int i = 0; i < npend; ++i) b.pending[i] = b.next_pending[i];
  st[ST_N_PENDING] = npend;
  st[ST_N_BUILD] = nb;
  st[ST_N_SITEMS] = di;
  const int ch = max((long long)p.min_rows, (total + p.hist_target - 1) / max(1, p.hist_target));
  int k = 0;
  for (int i = 0; i < nb; ++i) {
    const DNode& n = b.nodes[b.item_nid[i]];
    emit_chunks(b.hist_items, k, n.slot, n.begin, n.cnt_local, ch, false);
  }
  st[ST_N_HIST] = k;
}

// Remaining pending nodes become leaves (only when the level loop stopped early)
// and the bin-threshold arrays used by the fused score/gradient kernel are built.
__global__ void lv_finalize_kernel(LvParams p, LvBufs b, int max_nodes) {
  int* st = b.st;
  if (threadIdx.x == 0) {
    for (int i = 0; i < st[ST_N_PENDING]; ++i) {
      DNode& n = b.nodes[b.pending[i]];
      if (n.is_leaf && n.left < 0) n.value = leaf_value(n.G, n.H, p);
    }
  }
  __syncthreads();
  const int nn = st[ST_NUM_NODES];
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

// Raw-feature version of the finished tree for test-set scoring:
// cond = mean (0.5*(v_a+v_b)) or median split of the candidate values,
// default child = left iff fill < cond (Tree.java:293-309, 357-375).
__global__ void lv_raw_tree_kernel(LvBufs b, int max_nodes, const float* __restrict__ cand,
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

// Fixed-point scales from the (all-reduced) max |g|, |h| and global row count.
__global__ void lv_scales_kernel(const double* __restrict__ mx, const long long* __restrict__ cnt,
                                 float* __restrict__ scales, double* __restrict__ inv_scales) {
  if (threadIdx.x >= 2) return;
  const double m = mx[threadIdx.x];
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
  return b;
}

extern "C" {

// ptrs: 25 device pointers (see make_bufs); iparams: max_depth, max_leaf_cnt,
// min_split_samples, hist_target, part_target, min_rows; fparams: min_split_loss,
// mcw, l1, l2, max_abs_leaf, lr.
void ytk_lv_step(int which, const uintptr_t* ptrs, const int* ip, const float* fp, int arg0,
                 int arg1, uintptr_t stream) {
  LvParams p;
  p.max_depth = ip[0];
  p.max_leaf_cnt = ip[1];
  p.min_split_samples = ip[2];
  p.hist_target = ip[3];
  p.part_target = ip[4];
  p.min_rows = ip[5];
  p.min_split_loss = fp[0];
  p.mcw = fp[1];
  p.l1 = fp[2];
  p.l2 = fp[3];
  p.max_abs_leaf = fp[4];
  p.lr = fp[5];
  LvBufs b = make_bufs(ptrs);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (which) {
    case 0: hipLaunchKernelGGL(lv_init_kernel, dim3(1), dim3(64), 0, s, p, b); break;
    case 1: hipLaunchKernelGGL(lv_plan_split_kernel, dim3(1), dim3(64), 0, s, p, b); break;
    case 2: hipLaunchKernelGGL(lv_sum_counts_kernel, dim3(1), dim3(256), 0, s, b, arg0); break;
    case 3: hipLaunchKernelGGL(lv_plan_children_kernel, dim3(1), dim3(64), 0, s, p, b, arg0, arg1); break;
    case 4: hipLaunchKernelGGL(lv_finalize_kernel, dim3(1), dim3(256), 0, s, p, b, arg0); break;
    default: throw std::runtime_error("bad lv step");
  }
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

void ytk_lv_scales(uintptr_t mx, uintptr_t cnt, uintptr_t scales, uintptr_t inv_scales,
                   uintptr_t stream) {
  hipLaunchKernelGGL(lv_scales_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     (const double*)mx, (const long long*)cnt, (float*)scales, (double*)inv_scales);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
