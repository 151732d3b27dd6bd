// GPU-resident leaf-wise (loss-guided) tree growth (gfx950).
//
// Reference control flow: J/optimizer/gbdt/DataParallelTreeMaker.java make() :104-115,
// 219-295 -- a priority queue of leaves ordered by lossChg; pop the best, split it, build
// its children's histograms (smaller child + sibling subtraction), search their splits,
// push them; leaf rules at pop time (lossChg <= min_split_loss, depth == max_depth,
// leaves == max_leaf_cnt, samples < min_split_samples) and at child creation
// (children_terminal). Host equivalent: csrc/native/leafwise.cpp (LeafGrower).
//
// MI355X design. The sequential pop order only depends on the split gains, so the
// order is REPLAYED from known gains and the device computes children speculatively in
// batches (an expansion that the replay never pops only permuted rows inside its own
// segment -- the tree is identical to the sequential algorithm). Everything that was a
// host round trip per batch is a device planner here, so a tree is a fixed launch
// sequence per batch that the host enqueues without waiting:
//   lw_plan      (1 workgroup) apply the last batch's split records, replay the queue
//                (wave-wide argmax over LDS keys; the sequential part never touches
//                global memory), write the tree nodes the replay finalised (all lanes,
//                from an LDS event list), choose the next batch (the unexpanded nodes the
//                growth would split within the leaf budget, ranked by bottleneck key),
//                emit the partition work (device counts).
//   partition    partition_atomic_kernel: children land in the OTHER half of a 2N-entry
//                ping-pong row buffer (out_shift), so no copy-back of the segments.
//   lw_children  child counts from the split cursors, smaller child, histogram chunks,
//                split items (built + derived), the slots to zero.
//   zero / hist / reduce / split: the existing kernels with device-resident counts.
// Histogram slots are never recycled inside a tree (slot = speculative node id; a
// 255-leaf tree uses < 600 of them, ~70 MB of the 288 GB of HBM3E).
#include "common.h"
#include "gbdt_fx.h"                 // fx_round, hist_lds_pos (subtree histograms)
#include "gbdt_partition_atomic.h"  // partition_atomic_body
#include "gbdt_split_node.h"        // SplitOut
#include "gbdt_tree_node.h"         // DNode, node_leaf_value

#include <algorithm>
#include <stdexcept>
#include <vector>

namespace ytk {

enum {
  LW_NUM_TNODES = 0,  // == ST_NUM_NODES of the level engine (finalize / raw-tree kernels)
  LW_NUM_LEAF, LW_N_SIDS, LW_N_SPLIT, LW_N_PBLK, LW_N_HIST, LW_N_SITEMS, LW_N_BUILD, LW_DONE,
  LW_SEQ, LW_N_HEAP, LW_OVERFLOW, LW_BATCHES, LW_EXPANDED, LW_N_ZERO, LW_PART_DONE, LW_WORDS = 16
};

constexpr int kLwThreads = 256;      // children body (runs in the 256-thread partition blocks)
constexpr int kLwPlanThreads = 1024;  // planner / init: 16 waves for the block-parallel phases
                                      // (the replay itself is one wave either way)
constexpr int kLwCap = 2304;     // speculative nodes per tree (LDS-staged by the planner)
constexpr int kLwLeafMax = 512;   // max_leaf_cnt of the LDS-resident planner; also the batch-size cap
// Larger trees (up to kLwLeafMaxBig leaves, kLwCapBig speculative nodes) run the same planner
// with its per-node arrays and queues in a global-memory workspace (LwPlanWs): the replay's
// dependent reads then hit L2 instead of LDS, which is slower per pop but has no size limit.
constexpr int kLwLeafMaxBig = 4096;
constexpr int kLwCapBig = 16384;
constexpr int kLwSort = 4096;     // LDS scratch (u64): replay events, then batch-choice keys
constexpr int kLwChunk = 2048;    // rows per partition block (partition_atomic_kernel CH)
constexpr int kLwReduceDirect = 16;  // == kReduceDirect (gbdt_hist.hip)

struct LwParams {
  int max_depth, max_leaf, min_split_samples, speculate;  // speculate: 0 off, else percent
  float min_split_loss, mcw, l1, l2, max_abs_leaf, lr;
  int hist_target, min_rows, cap, N;  // N: half size of the ping-pong row buffers
  int split_groups;  // split records per item (feature groups of split_node_kernel)
  int dist;  // multi-GPU: per batch the host all-reduces the built slots + split cursors
  int bin_bytes;  // 1: uint8 bins, 2: uint16 bins (B > 256)
  int batch_cap;  // > 0: at most this many splits per batch (the RCCL batch loop sizes its fixed
                  // messages by it, ytk_lw_set_batch_cap); 0: no cap
  int slow_children;  // set per partition launch: 1 = YTK_PLAN_FAST=0 (general children path)
  // small-node subtrees (single GPU): batch entries with <= sub_rows rows are grown by
  // lw_subtree_kernel, up to sub_max more splits each, expanding nodes whose path-minimum
  // gain is >= sub_alpha x the previous tree's smallest split gain; sub_rows = 0: off
  int sub_rows, sub_max;
  float sub_alpha;
};

// global-memory planner workspace (large trees): the arrays the LDS planner keeps in LDS
struct LwPlanWs {
  int4* nd;                 // [cap]
  float* loss;              // [cap]
  int* seq;                 // [cap]
  int* par;                 // [cap]
  int4* ch;                 // [cap]
  int* hsid;                // [max_leaf + 8]
  unsigned long long* akey;  // [pow2 >= max_leaf + 8]
  unsigned long long* bkey;  // [2 max_leaf + 8]
  int* uid;                 // [3 max_leaf + 16]
  unsigned long long* buf;  // events (int4) / rank keys + bottlenecks
};

struct LwBufs {
  int* st;
  DNode* tnodes;  // the tree (tree node ids, reference numbering)
  // speculative nodes, structure of arrays [cap]
  double *G, *H, *gl, *hl;
  long long* cnt;  // rows (global)
  int *begin, *cnt_local, *depth, *feat, *bin_a, *bin_b, *lc, *tid, *seq, *state;
  float* loss;
  int* heap;  // [max_leaf + 2] speculative ids of the queue
  int* batch;  // [max_leaf] parents expanded by the current batch
  int *part_feat, *part_thr, *part_begin, *part_cnt, *part_first, *part_shift;  // [max_leaf]
  unsigned long long* cursor;  // [max_leaf * kCurStride + kDoneWords] split cursors ((right << 32) | left)
                               // a cache line apart, then the done counters
  int4* hist_items;            // [hist bound]
  int* build_ids;              // [max_leaf + 1] slots built this batch
  int4* split_items;           // [2 max_leaf + 2]
  int* item_sid;               // [2 max_leaf + 2]
  SplitOut* split_out;         // [2 max_leaf + 2]
  const long long* root_cnt;   // [0] local rows, [1] global rows
  unsigned long long* prof;    // optional [32]: planner phase times (wall clock ticks), rows
  int* done_host;              // host-mapped pinned int[2]: [0] LW_DONE, [1] batches planned (optional)
  int* zero_ids;               // [max_leaf + 1] built slots with != 1 histogram item
  int2* zero_range;            // [max_leaf + 1] their items [x, x + y)
  LwPlanWs ws;                 // large trees only (max_leaf > kLwLeafMax): else all null
  int* sub;                    // [SUB_WORDS] subtree state (below)
  int2* sub_list;              // [max_leaf] (parent, first child id) of the batch's subtree roots
};

// sub words: the batch's subtree roots, the node-id limit their expansions may reach (keeps
// 2 (remaining + 1) ids free, the planner's invariant), the leaf budget left, the previous
// tree's smallest split gain (float bits), the running minimum of this tree's split gains
enum { SUB_N = 0, SUB_LIMIT, SUB_REM, SUB_LAMBDA, SUB_MIN, SUB_WORDS = 8 };

// planner phase timing (YTK_LW_PROF=1): thread 0 accumulates wall-clock ticks per phase
#define LW_TICK(slot)                                                         \
  do {                                                                        \
    if (b.prof && threadIdx.x == 0) {                                         \
      const unsigned long long t_ = wall_clock64();                           \
      atomicAdd(&b.prof[slot], t_ - t_prev);                                  \
      t_prev = t_;                                                            \
    }                                                                         \
  } while (0)

enum { EV_LEAF = 0, EV_SPLIT = 1, EV_LEAFIFY = 2 };

constexpr int kLwQueueSort = 1024;  // power of two >= kLwLeafMax + 8

// pop-time leaf rules that do not depend on the running leaf count
__device__ __forceinline__ bool lw_static_leaf(const LwParams& p, float loss, int depth, int cnt) {
  return !(loss > p.min_split_loss) || (p.max_depth >= 0 && depth == p.max_depth) ||
         (p.min_split_samples > 0 && cnt < p.min_split_samples);
}

// node id bits of a queue key: 12 for the LDS planner (ids and seqs < 4096 for max_leaf <=
// 512), 16 for the workspace planner (cap <= kLwCapBig)
template <bool kBig>
struct LwKey {
  static constexpr int kBits = kBig ? 16 : 12;
  static constexpr unsigned long long kMask = (1ull << kBits) - 1;
};

// queue key: larger lossChg first, then the earlier push (smaller seq) -- the
// priority_queue order of LeafGrower::Entry; the node id rides in the low bits (seqs are
// unique so the id never decides the order)
template <bool kBig>
__device__ __forceinline__ unsigned long long lw_qkey(float loss, int seq, int sid) {
  unsigned u = __float_as_uint(loss);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving float -> uint
  constexpr int kB = LwKey<kBig>::kBits;
  return ((unsigned long long)u << 32) | ((LwKey<kBig>::kMask - (unsigned long long)seq) << kB) |
         (unsigned long long)sid;
}

// binary max-heap of keys in LDS, one thread
__device__ __forceinline__ void lw_heap_push(unsigned long long* key, int n, unsigned long long k) {
  int i = n;
  while (i > 0) {
    const int par = (i - 1) >> 1;
    const unsigned long long kp = key[par];
    if (kp >= k) break;
    key[i] = kp;
    i = par;
  }
  key[i] = k;
}

// remove the top of a heap of n + 1 entries whose last entry k is re-inserted
__device__ __forceinline__ void lw_heap_sift_down(unsigned long long* key, int n, unsigned long long k) {
  if (n == 0) return;
  int i = 0;
  while (true) {
    const int c = 2 * i + 1;
    if (c >= n) break;
    unsigned long long kc = key[c];
    int cc = c;
    if (c + 1 < n) {
      const unsigned long long k2 = key[c + 1];
      if (k2 > kc) { kc = k2; cc = c + 1; }
    }
    if (kc <= k) break;
    key[i] = kc;
    i = cc;
  }
  key[i] = k;
}

// max of a u64 over the wave (every lane gets it)
__device__ __forceinline__ unsigned long long lw_wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

// (max key, its index) of key[0..n) by one wave, every lane gets both; (0, -1) when
// n == 0. Keys are unique (node id in the low bits), so the index follows the key.
__device__ __forceinline__ void lw_wave_argmax(const unsigned long long* key, int n, unsigned long long& kmax,
                                               int& imax) {
  const int l = threadIdx.x & (kWave - 1);
  unsigned long long best = 0ull;
  for (int i = l; i < n; i += kWave) {
    const unsigned long long k = key[i];
    best = k > best ? k : best;
  }
  best = lw_wave_max_u64(best);
  int idx = -1;
  for (int i = l; i < n; i += kWave)
    if (key[i] == best) idx = i;
  // the one lane that found it (if any) -> all lanes
  const unsigned long long hit = __ballot(idx >= 0);
  kmax = best;
  imax = hit ? __shfl(idx, __builtin_ctzll(hit), kWave) : -1;
}

// block bitonic sort (descending) of a[0..n), n a power of two
__device__ void lw_bitonic_desc(unsigned long long* a, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (n >> 1); t += (int)blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long x = a[lo], y = a[hi];
        if ((x < y) == desc) {
          a[lo] = y;
          a[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Exclusive scan of one int per thread over the block (wave shuffles + LDS totals).
__device__ __forceinline__ int lw_scan(int v, int* s_tmp, int* total) {
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
  __syncthreads();
  *total = all;
  return before + inc - v;
}

// In-place exclusive scan of a[0..n) by the block (contiguous run per thread).
__device__ int lw_scan_array(int* a, int n, int* s_tmp) {
  const int per = (n + (int)blockDim.x - 1) / (int)blockDim.x;
  const int b = min(n, (int)threadIdx.x * per), e = min(n, b + per);
  int run = 0;
  for (int i = b; i < e; ++i) run += a[i];
  int total;
  int acc = lw_scan(run, s_tmp, &total);
  for (int i = b; i < e; ++i) {
    const int v = a[i];
    a[i] = acc;
    acc += v;
  }
  __syncthreads();
  return total;
}

__device__ void lw_write_node(DNode& n, const LwBufs& b, int sid, bool leaf, double G, double H, float loss,
                              long long cnt, int left, const LwParams& p) {
  n.G = G;
  n.H = H;
  n.gl = leaf ? 0.0 : b.gl[sid];
  n.hl = leaf ? 0.0 : b.hl[sid];
  n.cnt_global = cnt;
  n.begin = 0;
  n.cnt_local = 0;
  n.depth = 0;
  n.slot = sid;
  n.feat = leaf ? -1 : b.feat[sid];
  n.bin_a = leaf ? -1 : b.bin_a[sid];
  n.bin_b = leaf ? -1 : b.bin_b[sid];
  n.left = leaf ? -1 : left;
  n.right = leaf ? -1 : left + 1;
  n.loss_chg = loss;
  n.value = leaf ? node_leaf_value(G, H, p.mcw, p.l1, p.l2, p.max_abs_leaf, p.lr) : 0.f;
  n.is_leaf = leaf ? 1 : 0;
}

// Root: node 0 holds every (local) row; histogram chunks of slot 0; the root is queued.
__global__ __launch_bounds__(kLwPlanThreads) void lw_init_kernel(LwParams p, LwBufs b) {
  const int n_local = (int)b.root_cnt[0];
  const int ch = max(p.min_rows, (n_local + p.hist_target - 1) / max(1, p.hist_target));
  const int nblk = (n_local + ch - 1) / ch;
  int* st = b.st;
  if (threadIdx.x == 0) {
    for (int i = 0; i < LW_WORDS; ++i) st[i] = 0;
    st[LW_NUM_TNODES] = 1;
    st[LW_NUM_LEAF] = 1;
    st[LW_N_SIDS] = 1;
    st[LW_SEQ] = 1;
    st[LW_N_HEAP] = 1;
    st[LW_N_HIST] = nblk;
    st[LW_N_BUILD] = 1;
    st[LW_N_SITEMS] = 1;
    b.heap[0] = 0;
    b.G[0] = b.H[0] = b.gl[0] = b.hl[0] = 0.0;
    b.cnt[0] = b.root_cnt[1];
    b.begin[0] = 0;
    b.cnt_local[0] = n_local;
    b.depth[0] = 0;
    b.feat[0] = -1;
    b.bin_a[0] = b.bin_b[0] = -1;
    b.lc[0] = -1;
    b.tid[0] = 0;
    b.seq[0] = 0;
    b.state[0] = 0;
    b.loss[0] = -INFINITY;
    b.build_ids[0] = 0;
    st[LW_N_ZERO] = 1;
    b.zero_ids[0] = 0;
    b.zero_range[0] = make_int2(0, nblk);
    b.split_items[0] = make_int4(0, 0, 0, 0);
    b.item_sid[0] = 0;
    if (b.sub) {  // the last tree's smallest split gain becomes this tree's expansion floor
      const unsigned m = (unsigned)b.sub[SUB_MIN];
      if (m != 0x7f800000u) b.sub[SUB_LAMBDA] = (int)m;
      b.sub[SUB_MIN] = 0x7f800000;  // +inf
      b.sub[SUB_N] = 0;
    }
  }
  for (int k = threadIdx.x; k < nblk; k += kLwPlanThreads)
    b.hist_items[k] = make_int4(0, k * ch, min((k + 1) * ch, n_local), (k == 0 && nblk > kLwReduceDirect) ? 2 : 0);
}

// Start of every planning step (planner or auto-expansion): multi-GPU, the previous
// batch's split cursors ((right << 32) | left rows) were all-reduced with its built
// histograms, so the children's GLOBAL row counts replace the local ones the partition
// epilogue wrote (DataParallelTreeMaker.java:518,538); then the previous batch's split
// records are applied (canSplit: UpdateStrategy.java:50-53). Ends without a barrier.
__device__ void lw_apply_splits(const LwParams& p, const LwBufs& b) {
  int* st = b.st;
  const int tid = threadIdx.x;
  if (p.dist) {
    const int kprev = st[LW_N_SPLIT];
    for (int j = tid; j < kprev; j += (int)blockDim.x) {
      const int P = b.batch[j];
      const int L = b.lc[P];
      const long long lg = (long long)(b.cursor[(size_t)j * kCurStride] & 0xffffffffull);
      b.cnt[L] = lg;
      b.cnt[L + 1] = b.cnt[P] - lg;
    }
    __syncthreads();
  }
  const double mcw2 = (double)p.mcw * 2.0;
  const int nsi = st[LW_N_SITEMS];
  for (int i = tid; i < nsi; i += (int)blockDim.x) {
    const int sid = b.item_sid[i];
    // best of the item's feature-group records (split_node_kernel order: larger gain, then
    // lower feature, then lower bin; none last); node totals are equal in every record
    const int ng = p.split_groups;
    auto fkey = [](int f) { return f < 0 ? 0x7fffffff : f; };
    int bg = 0;
    for (int g = 1; g < ng; ++g) {
      const SplitOut& c = b.split_out[(size_t)i * ng + g];
      const SplitOut& bb = b.split_out[(size_t)i * ng + bg];
      if (better(c.loss_chg, fkey(c.feat), fkey(c.bin_b), bb.loss_chg, fkey(bb.feat), fkey(bb.bin_b))) bg = g;
    }
    SplitOut o = b.split_out[(size_t)i * ng + bg];
    if (bg != 0) {
      o.g = b.split_out[(size_t)i * ng].g;
      o.h = b.split_out[(size_t)i * ng].h;
    }
    b.G[sid] = o.g;
    b.H[sid] = o.h;
    b.gl[sid] = o.gl;
    b.hl[sid] = o.hl;
    int feat = o.feat;
    float chg = o.loss_chg;
    if (!(o.h >= mcw2 && b.cnt[sid] >= (long long)p.min_split_samples)) {
      chg = -INFINITY;
      feat = -1;
    }
    b.feat[sid] = feat;
    b.bin_a[sid] = o.bin_a;
    b.bin_b[sid] = o.bin_b;
    b.loss[sid] = chg;
    b.state[sid] = 1;
  }
}

// Phase F for batch entry j (parent P): children ids lc, lc + 1, their fresh node state, the
// partition descriptor (chunks of kLwChunk rows), the split cursor reset.
// Returns the entry's partition chunk count (also stored in part_first[j] for the general scan).
__device__ __forceinline__ int lw_expand_one(const LwParams& p, const LwBufs& b, int j, int P, int lc) {
  b.batch[j] = P;
  const int dep = b.depth[P] + 1;
  for (int c = lc; c <= lc + 1; ++c) {
    b.G[c] = b.H[c] = b.gl[c] = b.hl[c] = 0.0;
    b.cnt[c] = 0;
    b.begin[c] = 0;
    b.cnt_local[c] = 0;
    b.depth[c] = dep;
    b.feat[c] = -1;
    b.bin_a[c] = b.bin_b[c] = -1;
    b.lc[c] = -1;
    b.tid[c] = -1;
    b.seq[c] = 0;
    b.state[c] = 0;
    b.loss[c] = -INFINITY;
  }
  const int beg = b.begin[P], cnt = b.cnt_local[P];
  b.part_feat[j] = b.feat[P];
  b.part_thr[j] = (b.bin_a[P] + b.bin_b[P]) >> 1;  // bin <= floor((a+b)/2) <=> bin < (a+b)/2
  b.part_begin[j] = beg;
  b.part_cnt[j] = cnt;
  b.part_shift[j] = beg < p.N ? p.N : -p.N;
  const int nch = (cnt + kLwChunk - 1) / kLwChunk;
  b.part_first[j] = nch;
  b.cursor[(size_t)j * kCurStride] = 0ull;
  return nch;
}

// kBig: the per-node arrays and queues live in the global workspace b.ws (large trees)
template <bool kBig>
__global__ __launch_bounds__(kLwPlanThreads) void lw_plan_kernel(LwParams p, LwBufs b) {
  constexpr int kC = kBig ? 1 : kLwCap, kL = kBig ? 1 : kLwLeafMax;
  // node fields the replay reads, packed: {lc, tid, depth | state << 16 | static_leaf << 24, cnt}
  __shared__ int4 l_nd[kC];
  __shared__ float l_loss[kC];
  __shared__ int l_seq[kC];
  __shared__ int l_hsid[kL + 8];
  __shared__ int l_par[kC];  // batch choice: forest parents (pointer jumping)
  // children of an expanded node, as the replay needs them (one LDS round trip per pop):
  // {loss_l bits, loss_r bits, terminal-by-static-rules | poppable_l << 1 | poppable_r << 2, 0}
  __shared__ int4 l_ch[kC];
  __shared__ unsigned long long l_akey[kBig ? 1 : kLwQueueSort];  // poppable queue entries, sorted
  __shared__ unsigned long long l_bkey[2 * kL + 8];               // children heap
  __shared__ int l_uid[3 * kL + 16];                              // blocking entries
  __shared__ int s_na, s_nu;
  // replay events (then reused by the batch choice: rank keys + bottlenecks, 27 KiB)
  __shared__ unsigned long long l_buf[kBig ? 1 : kLwSort];
  int4* s_nd = kBig ? b.ws.nd : l_nd;
  float* s_loss = kBig ? b.ws.loss : l_loss;
  int* s_seq = kBig ? b.ws.seq : l_seq;
  int* s_hsid = kBig ? b.ws.hsid : l_hsid;
  int* s_par = kBig ? b.ws.par : l_par;
  int4* s_ch = kBig ? b.ws.ch : l_ch;
  unsigned long long* s_akey = kBig ? b.ws.akey : l_akey;
  unsigned long long* s_bkey = kBig ? b.ws.bkey : l_bkey;
  int* s_uid = kBig ? b.ws.uid : l_uid;
  unsigned long long* s_buf = kBig ? b.ws.buf : l_buf;
  const int capr = kBig ? (p.cap + 127) & ~127 : kLwCap;  // rank-key entries (a multiple of 128)
  const int leaf_max = kBig ? p.max_leaf : kLwLeafMax;
  __shared__ int s_tmp[kLwPlanThreads / kWave + 1];
  __shared__ int s_nev, s_blocked, s_nh, s_num_leaf, s_ntree, s_seqc, s_k, s_ncand;
  int* st = b.st;
  const int tid = threadIdx.x;
  if (st[LW_DONE]) {
    if (tid == 0) st[LW_PART_DONE] = 0;
    return;
  }
  unsigned long long t_prev = b.prof && tid == 0 ? wall_clock64() : 0ull;
  lw_apply_splits(p, b);
  const int nsid = st[LW_N_SIDS];
  __syncthreads();
  LW_TICK(0);
  // B. stage what the replay reads
  for (int i = tid; i < nsid; i += kLwPlanThreads) {
    const float loss = b.loss[i];
    const int cnt = (int)b.cnt[i], depth = b.depth[i];
    const int sl = lw_static_leaf(p, loss, depth, cnt) ? 1 : 0;
    s_loss[i] = loss;
    s_seq[i] = b.seq[i];
    const int lc = b.lc[i];
    s_nd[i] = make_int4(lc, b.tid[i], depth | (b.state[i] << 16) | (sl << 24), cnt);
    if (lc >= 0) {
      const float ll = b.loss[lc], lr = b.loss[lc + 1];
      const int dc = b.depth[lc], cl = (int)b.cnt[lc], cr = (int)b.cnt[lc + 1];
      const bool popl = lw_static_leaf(p, ll, dc, cl) || b.lc[lc] >= 0;
      const bool popr = lw_static_leaf(p, lr, dc, cr) || b.lc[lc + 1] >= 0;
      const bool tstat = (p.max_depth >= 0 && p.max_depth == dc) ||
                         (p.min_split_samples > 0 && cl < p.min_split_samples && cr < p.min_split_samples);
      s_ch[i] = make_int4(__float_as_int(ll), __float_as_int(lr), (tstat ? 1 : 0) | (popl ? 2 : 0) | (popr ? 4 : 0), 0);
    }
  }
  int nh = st[LW_N_HEAP];
  for (int i = tid; i < nh; i += kLwPlanThreads) s_hsid[i] = b.heap[i];
  if (tid == 0) { s_na = 0; s_nu = 0; }
  __syncthreads();
  LW_TICK(1);
  // C. replay the queue as far as the known gains allow. Queue entries are either
  //    POPPABLE (expanded, or a leaf by the static rules) or BLOCKING (neither): the
  //    replay stops exactly when the best remaining entry is blocking, so blocking
  //    entries only need their running max key (u). The poppable entries are sorted
  //    once (block bitonic); poppable children pushed during the replay go to a small
  //    binary heap; one lane merges the two. Keys carry the node id, node fields are
  //    packed: a pop is three dependent LDS round trips.
  int4* s_ev = reinterpret_cast<int4*>(s_buf);  // kLwSort / 2 events
  {
    for (int i = tid; i < nh; i += kLwPlanThreads) {
      const int sid = s_hsid[i];
      const int4 nd = s_nd[sid];
      if ((nd.z >> 24) || nd.x >= 0) s_akey[atomicAdd(&s_na, 1)] = lw_qkey<kBig>(s_loss[sid], s_seq[sid], sid);
      else s_uid[atomicAdd(&s_nu, 1)] = sid;
    }
    __syncthreads();
    const int na = s_na;
    int n2 = 1;
    while (n2 < na) n2 <<= 1;
    for (int i = na + tid; i < n2; i += kLwPlanThreads) s_akey[i] = 0ull;
    __syncthreads();
    lw_bitonic_desc(s_akey, n2);
  }
  LW_TICK(7);
  if (tid < kWave) {
    // Wave 0 runs the replay in lockstep: every lane holds the same scalar state and
    // issues the same (same-address, conflict-free) LDS writes, so no lane ever reads a
    // value another lane wrote; the lanes split only the scans (blocking max, children
    // max after a B pop, the queue copy-out). The children of the replayed splits go to
    // an UNSORTED array B with its running max (push: one store; pop: one wave max scan)
    // -- a binary heap here cost ~log2(n) dependent LDS round trips per push and pop,
    // about 1 us per replayed split.
    const int lane = tid;
    const int na = s_na;
    int nu = s_nu;
    unsigned long long u = 0ull;
    for (int i = lane; i < nu; i += kWave) {
      const int sid = s_uid[i];
      const unsigned long long k = lw_qkey<kBig>(s_loss[sid], s_seq[sid], sid);
      u = k > u ? k : u;
    }
    u = lw_wave_max_u64(u);
    int num_leaf = st[LW_NUM_LEAF], ntree = st[LW_NUM_TNODES], seqc = st[LW_SEQ];
    int nev = 0, blocked = -1, pa = 0, nbh = 0, bidx = -1;
    unsigned long long bmax = 0ull;
    bool bulk = false;
    unsigned long long ka = na > 0 ? s_akey[0] : 0ull;  // the next A key, loaded ahead
    while (true) {
      if (p.max_leaf > 0 && num_leaf == p.max_leaf) { bulk = true; break; }
      const unsigned long long top = ka > bmax ? ka : bmax;
      if (u > top) { blocked = (int)(u & LwKey<kBig>::kMask); break; }
      if (top == 0ull) break;  // queue empty
      const int sid = (int)(top & LwKey<kBig>::kMask);
      const int4 nd = s_nd[sid];
      const int4 ch = s_ch[sid];
      if (ka > bmax) {
        ++pa;
        ka = pa < na ? s_akey[pa] : 0ull;
      } else {
        --nbh;
        const unsigned long long last = s_bkey[nbh];
        if (bidx != nbh) s_bkey[bidx] = last;
        lw_wave_argmax(s_bkey, nbh, bmax, bidx);
      }
      if (nd.z >> 24) {  // leaf by the static rules
        s_ev[nev++] = make_int4(EV_LEAF, sid, nd.y, 0);
        s_nd[sid].z = (nd.z & 0xff00ffff) | (2 << 16);
        continue;
      }
      const int t = nd.y, lt = ntree;
      ntree += 2;
      ++num_leaf;
      const int l = nd.x, r = l + 1;
      const bool term = (ch.z & 1) || (p.max_leaf > 0 && p.max_leaf == num_leaf);
      s_nd[sid].z = (nd.z & 0xff00ffff) | (2 << 16);
      s_ev[nev++] = make_int4(EV_SPLIT, sid, t, lt);
      if (term) {
        const int4 ndl = s_nd[l], ndr = s_nd[r];
        s_ev[nev++] = make_int4(EV_LEAFIFY, sid, lt, 0);
        s_nd[l] = make_int4(ndl.x, lt, (ndl.z & 0xff00ffff) | (2 << 16), ndl.w);
        s_nd[r] = make_int4(ndr.x, lt + 1, (ndr.z & 0xff00ffff) | (2 << 16), ndr.w);
        continue;
      }
      s_nd[l].y = lt;
      s_nd[r].y = lt + 1;
      s_seq[l] = seqc;
      s_seq[r] = seqc + 1;
      const unsigned long long kl = lw_qkey<kBig>(__int_as_float(ch.x), seqc, l);
      const unsigned long long kr = lw_qkey<kBig>(__int_as_float(ch.y), seqc + 1, r);
      seqc += 2;
      if (ch.z & 2) {
        s_bkey[nbh] = kl;
        if (kl > bmax) { bmax = kl; bidx = nbh; }
        ++nbh;
      } else {
        s_uid[nu++] = l;
        u = kl > u ? kl : u;
      }
      if (ch.z & 4) {
        s_bkey[nbh] = kr;
        if (kr > bmax) { bmax = kr; bidx = nbh; }
        ++nbh;
      } else {
        s_uid[nu++] = r;
        u = kr > u ? kr : u;
      }
    }
    // the remaining queue: A tail, the children array, the blocking entries (a set)
    const int ra = na - pa;
    for (int i = lane; i < ra; i += kWave) s_hsid[i] = (int)(s_akey[pa + i] & LwKey<kBig>::kMask);
    for (int i = lane; i < nbh; i += kWave) s_hsid[ra + i] = (int)(s_bkey[i] & LwKey<kBig>::kMask);
    for (int i = lane; i < nu; i += kWave) s_hsid[ra + nbh + i] = s_uid[i];
    int nr = ra + nbh + nu;
    if (bulk) {  // leaf budget used: every queued node pops as a leaf (order-independent)
      for (int i = lane; i < nr; i += kWave) {
        const int sid = s_hsid[i];
        const int4 nd = s_nd[sid];
        s_ev[nev + i] = make_int4(EV_LEAF, sid, nd.y, 0);
        s_nd[sid].z = (nd.z & 0xff00ffff) | (2 << 16);
      }
      nev += nr;
      nr = 0;
    }
    if (lane == 0) {
      s_nev = nev;
      s_blocked = blocked;
      s_nh = nr;
      s_num_leaf = num_leaf;
      s_ntree = ntree;
      s_seqc = seqc;
      if (b.prof) atomicAdd(&b.prof[21], (unsigned long long)(pa));
    }
  }
  __syncthreads();
  LW_TICK(2);
  // D. tree nodes finalised by the replay (independent writes, all lanes)
  const int nev = s_nev;
  for (int e = tid; e < nev; e += kLwPlanThreads) {
    const int4 ev = s_ev[e];
    const int sid = ev.y;
    if (ev.x == EV_LEAF) {
      lw_write_node(b.tnodes[ev.z], b, sid, true, b.G[sid], b.H[sid], b.loss[sid], b.cnt[sid], -1, p);
    } else if (ev.x == EV_SPLIT) {
      const float ls = b.loss[sid];
      lw_write_node(b.tnodes[ev.z], b, sid, false, b.G[sid], b.H[sid], ls, b.cnt[sid], ev.w, p);
      if (b.sub && ls >= 0.f) atomicMin(reinterpret_cast<unsigned*>(&b.sub[SUB_MIN]), __float_as_uint(ls));
    } else {  // children made leaves right away: sums from the parent's best split
      const int l = s_nd[sid].x;
      const double gl = b.gl[sid], hl = b.hl[sid];
      lw_write_node(b.tnodes[ev.z], b, l, true, gl, hl, -INFINITY, b.cnt[l], -1, p);
      lw_write_node(b.tnodes[ev.z + 1], b, l + 1, true, b.G[sid] - gl, b.H[sid] - hl, -INFINITY, b.cnt[l + 1],
                    -1, p);
    }
  }
  __syncthreads();  // s_buf is reused below
  LW_TICK(3);
  const int blocked = s_blocked;
  const int num_leaf = s_num_leaf;
  nh = s_nh;
  // E. next batch: the blocked node + the best other candidates
  int k = 0;
  const int remaining = p.max_leaf > 0 ? p.max_leaf - num_leaf : 1;
  if (blocked >= 0) {
    const int fr = p.cap - nsid;
    // keep a node pair per future split free (2 (remaining + 1) ids): speculative expansions
    // the replay never splits can then never starve the forced expansion of a blocked node,
    // which the next replay always splits (so it pays for its pair); cap >= 2 max_leaf + 3
    // holds the invariant from the root on
    k = p.speculate ? max(1, min(min(remaining, kLwLeafMax), (fr - 2 * remaining - 2) >> 1)) : 1;
    // host-chosen cap (RCCL batch loop): the batch is then the best-ranked prefix of the
    // candidates -- the replay still splits exactly the sequential growth's nodes
    if (p.batch_cap > 0) k = min(k, p.batch_cap);
    if (fr < 2) k = 0;
  }
  int* s_batch = reinterpret_cast<int*>(s_akey);  // the batch, in pop order (A is consumed)
  if (k > 0) {
    // Which unexpanded nodes would the sequential growth split within the leaf budget?
    // (the host planner's virtual replay, builder.py _grow_loss_guided). A priority queue
    // over a forest pops nodes in decreasing order of their BOTTLENECK key (the minimum
    // key on the path from the queue entry that roots them), so with the not-yet-computed
    // children treated as absent, the nodes popped as splits before the budget runs out
    // are the top `remaining` splittable known nodes by bottleneck; the batch is the
    // unexpanded ones among them, best first. Pointer jumping gives the bottlenecks in
    // log(depth) block steps; each candidate's rank is a count over the splittable set.
    // (Top-k by the node's own gain expanded ~1.6x as many nodes: docs/performance.md.)
    unsigned long long* s_rk = s_buf;                                 // [capr] splittable rank keys
    unsigned* s_m = reinterpret_cast<unsigned*>(s_buf + capr);        // [capr] bottleneck ord(loss)
    constexpr int kPer = ((kBig ? kLwCapBig : kLwCap) + kLwPlanThreads - 1) / kLwPlanThreads;
    auto ord = [](float f) {
      const unsigned u = __float_as_uint(f);
      return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    };
    auto live = [&](int i) { return ((s_nd[i].z >> 16) & 0xff) == 1; };  // known gain, not final
    // the splittable live nodes (each pops as a split) and the unexpanded ones among them
    auto splittable = [&](int i) { return live(i) && (s_nd[i].z >> 24) == 0; };
    const int per = (nsid + kLwPlanThreads - 1) / kLwPlanThreads;
    const int i0 = min(nsid, tid * per), i1 = min(nsid, i0 + per);
    int c = 0, cc = 0;
    for (int i = i0; i < i1; ++i) {
      const bool sp = splittable(i);
      c += sp ? 1 : 0;
      cc += (sp && s_nd[i].x < 0) ? 1 : 0;
    }
    int ns, ncand;
    int pos = lw_scan(c, s_tmp, &ns);
    int pc = lw_scan(cc, s_tmp, &ncand);
    // rank window: speculate percent of the leaf budget (s_uid holds 3 leaf_max ranks)
    const int rem = min(3 * leaf_max, max(1, remaining * p.speculate / 100));
    if (ns <= rem && ncand <= k) {
      // every splittable node ranks inside the window and the batch has room for every
      // candidate: the batch is all of them, and no bottleneck / rank is needed (the order
      // only numbers the speculative nodes: the replay orders pops by (gain, push seq), so
      // the tree is the same). Most batches of a 255-leaf tree take this path.
      for (int i = i0; i < i1; ++i)
        if (splittable(i) && s_nd[i].x < 0) s_batch[pc++] = i;
      if (tid == 0) {
        s_k = ncand;
        s_ncand = ncand;
      }
      __syncthreads();
      k = s_k;
    } else {
    for (int i = tid; i < nsid; i += kLwPlanThreads) {
      s_par[i] = -1;
      s_m[i] = ord(s_loss[i]);
    }
    __syncthreads();
    for (int i = tid; i < nsid; i += kLwPlanThreads) {
      const int4 nd = s_nd[i];
      if (((nd.z >> 16) & 0xff) == 1 && nd.x >= 0) s_par[nd.x] = s_par[nd.x + 1] = i;
    }
    __syncthreads();
    while (true) {
      unsigned nm[kPer];
      int np[kPer];
      int any = 0;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int i = tid + j * kLwPlanThreads;
        np[j] = -1;
        if (i < nsid) {
          const int pp = s_par[i];
          nm[j] = s_m[i];
          if (pp >= 0) {
            nm[j] = min(nm[j], s_m[pp]);
            np[j] = s_par[pp];
            any = 1;
          }
        }
      }
      if (!__syncthreads_or(any)) break;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int i = tid + j * kLwPlanThreads;
        if (i < nsid) {
          s_m[i] = nm[j];
          s_par[i] = np[j];
        }
      }
      __syncthreads();
    }
    LW_TICK(22);
    // rank keys of the splittable nodes, compacted
    auto rkey = [&](int i) {
      return i == blocked ? ~0ull
                          : (((unsigned long long)s_m[i] << 32) |
                             (unsigned long long)((ord(s_loss[i]) >> LwKey<kBig>::kBits) << LwKey<kBig>::kBits) |
                             (unsigned long long)i);
    };
    int* s_cand = s_par;  // all -1 after the pointer jumping: reused as the candidate list
    for (int i = i0; i < i1; ++i) {
      if (!splittable(i)) continue;
      s_rk[pos++] = rkey(i);
      if (s_nd[i].x < 0) s_cand[pc++] = i;
    }
    const int ns_pad = (ns + 2 * kWave - 1) & ~(2 * kWave - 1);  // <= capr (a multiple of 128)
    for (int z = ns + tid; z < ns_pad; z += kLwPlanThreads) s_rk[z] = 0ull;  // never ranks above a key
    for (int r = tid; r < rem; r += kLwPlanThreads) s_uid[r] = -1;
    __syncthreads();
    LW_TICK(23);
    // rank of each candidate among the splittable set: a wave takes 4 candidates, every
    // key it loads is compared with all 4 (ballot + popcount: wave-uniform counts)
    const int lane = tid & (kWave - 1);
    for (int g = (tid >> 6) * 4; g < ncand; g += kLwPlanThreads / kWave * 4) {
      unsigned long long me[4];
      int rank[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        me[j] = g + j < ncand ? rkey(s_cand[g + j]) : ~0ull;
        rank[j] = 0;
      }
      for (int z0 = 0; z0 < ns_pad; z0 += 2 * kWave) {
        const unsigned long long a0 = s_rk[z0 + lane], a1 = s_rk[z0 + kWave + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j) rank[j] += __popcll(__ballot(a0 > me[j])) + __popcll(__ballot(a1 > me[j]));
      }
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (g + j < ncand && rank[j] < rem) s_uid[rank[j]] = s_cand[g + j];
      }
    }
    __syncthreads();
    LW_TICK(24);
    // compact the chosen ones in rank order
    const int pr = (rem + kLwPlanThreads - 1) / kLwPlanThreads;
    const int r0 = min(rem, tid * pr), r1 = min(rem, r0 + pr);
    int nc = 0;
    for (int r = r0; r < r1; ++r) nc += s_uid[r] >= 0 ? 1 : 0;
    int nsel;
    int q = lw_scan(nc, s_tmp, &nsel);
    for (int r = r0; r < r1; ++r)
      if (s_uid[r] >= 0) s_batch[q++] = s_uid[r];
    if (tid == 0) {
      s_k = min(k, nsel);
      s_ncand = ncand;
    }
    __syncthreads();
    k = s_k;
    }  // ranked batch choice
  }
  LW_TICK(4);
  // F. expand the batch: children ids, partition descriptors (chunks of kLwChunk rows)
  // (k <= kLwLeafMax < kLwPlanThreads: one entry per thread.) Entries with <= sub_rows rows
  // go to the subtree kernel (sub_list); the others, compacted, to the partition pipeline.
  // Child ids follow the batch order either way.
  static_assert(kLwLeafMax <= kLwPlanThreads, "one batch entry per planner thread");
  int nblocks = 0, kn = k, ks = 0;
  if (k > 0) {
    const int j = tid;
    const bool mine = j < k;
    const int P = mine ? s_batch[j] : 0;
    const bool sub = mine && p.sub_rows > 0 && s_nd[P].w <= p.sub_rows;
    const int jn = lw_scan(mine && !sub ? 1 : 0, s_tmp, &kn);
    const int js = lw_scan(sub ? 1 : 0, s_tmp, &ks);
    int nch = 0;
    if (mine) {
      const int lc = nsid + 2 * j;
      s_nd[P].x = lc;
      if (sub) b.sub_list[js] = make_int2(P, lc);
      else nch = lw_expand_one(p, b, jn, P, lc);
    }
    // exclusive scan of the chunk counts in registers (no read-back of part_first)
    const int first = lw_scan(nch, s_tmp, &nblocks);
    if (mine && !sub) b.part_first[jn] = first;
  }
  LW_TICK(5);
  // G. write back the replay state
  for (int i = tid; i < nsid; i += kLwPlanThreads) {
    const int4 nd = s_nd[i];
    b.lc[i] = nd.x;
    b.tid[i] = nd.y;
    b.seq[i] = s_seq[i];
    b.state[i] = (nd.z >> 16) & 0xff;
  }
  for (int i = tid; i < nh; i += kLwPlanThreads) b.heap[i] = s_hsid[i];
  if (tid == 0) {
    st[LW_PART_DONE] = 0;
    st[LW_NUM_LEAF] = num_leaf;
    st[LW_NUM_TNODES] = s_ntree;
    st[LW_SEQ] = s_seqc;
    st[LW_N_HEAP] = nh;
    st[LW_N_SPLIT] = kn;
    st[LW_N_PBLK] = nblocks;
    st[LW_N_SIDS] = nsid + 2 * k;
    if (b.sub) {
      b.sub[SUB_N] = ks;
      b.sub[SUB_LIMIT] = p.cap - 2 * remaining - 2;
      b.sub[SUB_REM] = remaining;
    }
    if (k == 0) {
      st[LW_DONE] = 1;
      if (b.done_host) *(volatile int*)b.done_host = 1;  // polled by the host: no copy launch
      if (blocked >= 0) st[LW_OVERFLOW] = 1;  // cannot happen with cap >= max_leaf + 2
    } else {
      const int nb = st[LW_BATCHES] + 1;
      st[LW_BATCHES] = nb;
      st[LW_EXPANDED] += k;
      // planner progress for the host's launch throttle (reads pinned memory, no events);
      // [2] = the batch's split count (multi-GPU: sizes the batch's all-reduce), written
      // before the count the host polls
      if (b.done_host) {
        ((volatile int*)b.done_host)[2] = k;
        ((volatile int*)b.done_host)[1] = nb;
      }
    }
  }
  LW_TICK(6);
  if (b.prof && tid == 0) {
    atomicAdd(&b.prof[8], 1ull);                      // planner calls
    atomicAdd(&b.prof[9], (unsigned long long)nblocks);  // partition blocks
    atomicAdd(&b.prof[10], (unsigned long long)s_nev);   // replay events
    if (k > 0) atomicAdd(&b.prof[11], (unsigned long long)s_ncand);  // candidates
  }
}

// Children of the batch: counts from the partition cursors, smaller child, histogram
// chunks of the built children, split items (built, then derived = parent - built).
__device__ void lw_children_body(const LwParams& p, const LwBufs& b) {
  // three LDS arrays only: this body also runs as the fused partition kernel's epilogue,
  // whose occupancy its LDS footprint sets
  __shared__ int s_need[kLwLeafMax], s_small[kLwLeafMax], s_first[kLwLeafMax];
  __shared__ int s_tmp[kLwThreads / kWave + 1];
  __shared__ unsigned long long s_total;
  int* st = b.st;
  const int tid = threadIdx.x;
  const int k = st[LW_N_SPLIT];
  if (k == 0) {
    if (tid == 0) {
      st[LW_N_HIST] = 0;
      st[LW_N_SITEMS] = 0;
      st[LW_N_BUILD] = 0;
      st[LW_N_ZERO] = 0;
    }
    return;
  }
  if (tid == 0) s_total = 0ull;
  __syncthreads();
  if (!p.slow_children && k <= kLwThreads && (int)blockDim.x == kLwThreads) {
    // Fast path (<= 256 splits): one thread per split keeps the parent, its children and the
    // built child's segment in registers from the cursor to the histogram work list --
    // dependent global round trips st -> (batch, cursor, part_*) -> lc -> depth instead of
    // re-reading the node arrays other threads wrote (build ids, begins, counts). Same
    // outputs as the general path below.
    __shared__ int s_cntb[kLwThreads];
    const int j = tid;
    const bool mine = j < k;
    int P = 0, lloc = 0, lb = 0, rcnt = 0;
    if (mine) {
      P = b.batch[j];
      const unsigned long long cur =
          __hip_atomic_load(&b.cursor[(size_t)j * kCurStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lloc = (int)(cur & 0xffffffffull);
      lb = b.part_begin[j] + b.part_shift[j];
      rcnt = b.part_cnt[j] - lloc;
    }
    bool need = false, left_small = false;
    int L = 0;
    if (mine) {
      L = b.lc[P];
      const int R = L + 1;
      const bool ls = p.dist ? (b.hl[P] < b.H[P] - b.hl[P]) : (lloc < rcnt);
      b.begin[L] = lb;
      b.cnt_local[L] = lloc;
      b.cnt[L] = lloc;
      b.begin[R] = lb + lloc;
      b.cnt_local[R] = rcnt;
      b.cnt[R] = rcnt;
      const int dep = b.depth[L];
      need = !(p.max_depth >= 0 && dep == p.max_depth) &&
             !(p.min_split_samples > 0 && lloc < p.min_split_samples && rcnt < p.min_split_samples);
      left_small = ls;
      if (need) atomicAdd(&s_total, (unsigned long long)(left_small ? lloc : rcnt));
    }
    int nb;
    const int kb = lw_scan(need ? 1 : 0, s_tmp, &nb);  // build index (the scan's barriers order s_total)
    const long long total = (long long)s_total;
    const int ch = (int)max((long long)p.min_rows, (total + p.hist_target - 1) / max(1, p.hist_target));
    int S = 0, cntS = 0, begS = 0, nfirst = 0;
    if (need) {
      S = left_small ? L : L + 1;
      const int G = left_small ? L + 1 : L;
      b.build_ids[kb] = S;
      b.split_items[kb] = make_int4(S, 0, 0, 0);
      b.item_sid[kb] = S;
      b.split_items[nb + kb] = make_int4(G, P, S, 1);
      b.item_sid[nb + kb] = G;
      cntS = left_small ? lloc : rcnt;
      begS = left_small ? lb : lb + lloc;
      nfirst = cntS == 0 ? 0 : max(1, cntS / ch);
    }
    int nitems, nzero;
    const int first = lw_scan(nfirst, s_tmp, &nitems);
    const bool multi = need && nfirst != 1;  // slots the split-K reduce adds into (zeroed)
    const int z = lw_scan(multi ? 1 : 0, s_tmp, &nzero);
    if (multi) {
      b.zero_ids[z] = S;
      b.zero_range[z] = make_int2(first, nfirst);
    }
    if (need) {
      s_first[kb] = first;
      s_small[kb] = S;
      s_need[kb] = begS;
      s_cntb[kb] = cntS;
    }
    __syncthreads();
    for (int q = tid; q < nitems; q += kLwThreads) {
      int lo = 0, hi = nb - 1;  // last build with s_first <= q
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_first[mid] <= q) lo = mid; else hi = mid - 1;
      }
      const int jq = q - s_first[lo];
      const int nc = (lo + 1 < nb ? s_first[lo + 1] : nitems) - s_first[lo];
      const int beg = s_need[lo];
      const long long cnt = s_cntb[lo];
      const int cb = beg + (int)(cnt * jq / nc);
      const int ce = beg + (int)(cnt * (jq + 1) / nc);
      b.hist_items[q] = make_int4(s_small[lo], cb, ce, nc == 1 ? 1 : (nc > kLwReduceDirect && jq == 0 ? 2 : 0));
    }
    if (tid == 0) {
      st[LW_N_HIST] = nitems;
      st[LW_N_BUILD] = nb;
      st[LW_N_ZERO] = nzero;
      st[LW_N_SITEMS] = 2 * nb;
      if (b.prof) {
        atomicAdd(&b.prof[12], (unsigned long long)total);
        atomicAdd(&b.prof[13], (unsigned long long)nb);
        atomicAdd(&b.prof[14], (unsigned long long)nitems);
      }
    }
    return;
  }
  for (int j = tid; j < k; j += kLwThreads) {
    const int P = b.batch[j];
    const int L = b.lc[P], R = L + 1;
    const unsigned long long cur = __hip_atomic_load(&b.cursor[(size_t)j * kCurStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int lloc = (int)(cur & 0xffffffffull);
    const int lb = b.part_begin[j] + b.part_shift[j];
    const int rcnt = b.part_cnt[j] - lloc;
    b.begin[L] = lb;
    b.cnt_local[L] = lloc;
    b.cnt[L] = lloc;
    b.begin[R] = lb + lloc;
    b.cnt_local[R] = rcnt;
    b.cnt[R] = rcnt;
    const int dep = b.depth[L];
    // children that are terminal whatever the replay does get no histograms
    const bool need = !(p.max_depth >= 0 && dep == p.max_depth) &&
                      !(p.min_split_samples > 0 && lloc < p.min_split_samples && rcnt < p.min_split_samples);
    // multi-GPU: the counts are still local here, so the built (smaller) child is chosen by
    // the globally identical hessian sums -- every rank builds the same slot (exact int64
    // histograms make the choice result-neutral)
    const bool left_small = p.dist ? (b.hl[P] < b.H[P] - b.hl[P]) : (lloc < rcnt);
    s_need[j] = need ? 1 : 0;
    s_small[j] = need ? (left_small ? L : R) : -1;
    if (need) atomicAdd(&s_total, (unsigned long long)(left_small ? lloc : rcnt));
  }
  __syncthreads();
  const int nb = lw_scan_array(s_need, k, s_tmp);  // s_need = build index
  const long long total = (long long)s_total;
  // (the level engine sizes its chunks for hist_target - nb items, one block per CU; here
  // that measured slower: a batch's many small built nodes are one item each anyway, and
  // the larger chunks of its big nodes lengthened the critical path: 3.53 -> 3.63 ms/tree)
  const int ch = (int)max((long long)p.min_rows, (total + p.hist_target - 1) / max(1, p.hist_target));
  for (int j = tid; j < k; j += kLwThreads) {
    const int S = s_small[j];
    if (S < 0) continue;
    const int kb = s_need[j];
    const int P = b.batch[j];
    const int L = b.lc[P];
    const int G = (S == L) ? L + 1 : L;
    b.build_ids[kb] = S;
    b.split_items[kb] = make_int4(S, 0, 0, 0);
    b.item_sid[kb] = S;
    b.split_items[nb + kb] = make_int4(G, P, S, 1);
    b.item_sid[nb + kb] = G;
    // floor(rows / ch) equal chunks (between ch and 2 ch rows each): no short tail
    // chunk paying a whole 128-KiB LDS clear + flush for a few rows
    const int cnt = b.cnt_local[S];
    s_first[kb] = cnt == 0 ? 0 : max(1, cnt / ch);
  }
  __syncthreads();
  for (int kb = tid; kb < nb; kb += kLwThreads) s_need[kb] = s_first[kb] != 1 ? 1 : 0;  // multi-item slots
  __syncthreads();
  const int nitems = lw_scan_array(s_first, nb, s_tmp);
  const int nzero = lw_scan_array(s_need, nb, s_tmp);  // s_need = index among the multi-item slots
  auto nch = [&](int kb) { return (kb + 1 < nb ? s_first[kb + 1] : nitems) - s_first[kb]; };
  for (int kb = tid; kb < nb; kb += kLwThreads) {
    const int c = nch(kb);
    if (c != 1) {
      const int z = s_need[kb];
      b.zero_ids[z] = b.build_ids[kb];
      b.zero_range[z] = make_int2(s_first[kb], c);
    }
  }
  for (int q = tid; q < nitems; q += kLwThreads) {
    int lo = 0, hi = nb - 1;  // last build with s_first <= q
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_first[mid] <= q) lo = mid; else hi = mid - 1;
    }
    const int jq = q - s_first[lo];
    const int nc = nch(lo);
    const int S = b.build_ids[lo];
    const int beg = b.begin[S];
    const long long cnt = b.cnt_local[S];
    const int cb = beg + (int)(cnt * jq / nc);
    const int ce = beg + (int)(cnt * (jq + 1) / nc);
    // w: 1 = the slot's only item (stored directly), 2 = first item of a split-K slot
    // (zeroes it), 0 otherwise
    b.hist_items[q] = make_int4(S, cb, ce, nc == 1 ? 1 : (nc > kLwReduceDirect && jq == 0 ? 2 : 0));
  }
  if (tid == 0) {
    st[LW_N_HIST] = nitems;
    st[LW_N_BUILD] = nb;
    st[LW_N_ZERO] = nzero;
    st[LW_N_SITEMS] = 2 * nb;
    if (b.prof) {
      atomicAdd(&b.prof[12], (unsigned long long)total);  // histogram rows
      atomicAdd(&b.prof[13], (unsigned long long)nb);     // built slots
      atomicAdd(&b.prof[14], (unsigned long long)nitems);  // histogram items
    }
  }
}

// Partition of the batch's segments (partition_atomic_body; children written into the
// other half of the ping-pong buffers) + the children planning, run by the LAST block to
// finish (device-scope counter): one launch and no launch gap between the two.
// kPrefetch: the software-pipelined body (partition_atomic_body_pf).
// kMode 3 (the first batches: one or two splits of thousands of chunks): the chunks scatter at
// prefix sums of the lw_part_count_lean_kernel counts (kMode 2: reservations lw_part_scan_kernel
// computed)
template <bool kPrefetch, bool kPfGh = false, typename BinT = uint8_t, bool kPfCol = false, int kMode = 0>
__global__ __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(kPrefetch ? 4 : 8, 8)))
void lw_partition_kernel(LwParams p, LwBufs b, const BinT* binsT,
                                                                   long long ncol, const int* rows,
                                                                   const float2* ghp, int* rows_out,
                                                                   float2* gh_out, unsigned long long* chunk_io,
                                                                   unsigned long long* gsum) {
  if constexpr (kPrefetch)
    partition_atomic_body_pf<BinT, kAtomSub, kPfGh, kPfCol, kMode>(binsT, ncol, rows, ghp, rows_out, gh_out, b.part_first,
                                                    b.st + LW_N_SPLIT,
                                      b.st + LW_N_PBLK, b.part_feat, b.part_thr, b.part_begin, b.part_cnt,
                                      b.cursor, b.part_shift, kCurStride, 0, chunk_io, gsum);
  else
    partition_atomic_body<BinT, true>(binsT, ncol, rows, ghp, rows_out, gh_out, b.part_first, b.st + LW_N_SPLIT,
                                      b.st + LW_N_PBLK, b.part_feat, b.part_thr, b.part_begin, b.part_cnt,
                                      b.cursor, b.part_shift, kCurStride);
  // No fences: the only cross-block data the last block reads are the split cursors,
  // updated by RETURNING device-scope atomics (complete before this block counts itself)
  // and read back with atomic loads. (An agent-scope release fence per block writes back
  // the XCD's L2 on MI355X and doubled this kernel's time.)
  if (!last_block_done(b.cursor + (size_t)p.max_leaf * kCurStride)) return;
  if constexpr (kMode == 3)  // the split totals the children planning reads from the cursors
    part_split_totals<kPartThreads>(chunk_io, gsum, b.part_first, b.st + LW_N_SPLIT, b.st + LW_N_PBLK, b.cursor,
                                    kCurStride);
  lw_children_body(p, b);
}

// one block per chunk (part_count_lean_body); no chunks once the tree is done (N_PBLK = 0)
__global__ __launch_bounds__(kPartThreads) void lw_part_count_lean_kernel(LwBufs b, const uint8_t* binsT, long long ncol,
                                                                          const int* rows, unsigned long long* chunk_io,
                                                                          unsigned long long* gsum) {
  part_count_lean_body(binsT, ncol, rows, b.part_first, b.st + LW_N_SPLIT, b.st + LW_N_PBLK, b.part_feat, b.part_thr,
                       b.part_begin, b.part_cnt, chunk_io, gsum);
}

// the chunk counts -> reservations + split cursor totals (part_chunk_scan_body)
__global__ __launch_bounds__(kChunkScanThreads) void lw_part_scan_kernel(LwBufs b, unsigned long long* chunk_io) {
  if (b.st[LW_DONE]) return;
  part_chunk_scan_body(chunk_io, b.part_first, b.st + LW_N_SPLIT, b.st + LW_N_PBLK, b.cursor, kCurStride);
}

// ---------------------------------------------------------------------------------
// Small-node subtrees (single GPU). A late 255-leaf Higgs tree is ~20 levels deep, but most
// of its splits sit in nodes of <= 32K rows (tools/lw_tree_shape.py): on the batch pipeline
// each of those levels costs a planner call + four launches (~90 us) for a few thousand
// rows. Here one 1024-thread workgroup per small batch entry P partitions P, builds the
// smaller child's exact int64 histogram in LDS (hist_fx_kernel's layout and rounding),
// derives the sibling and searches both children with the split kernels' own block search
// (split_node_block: bit-identical records), then keeps growing P's subtree best-first --
// up to sub_max more splits, only nodes whose path-minimum gain reaches sub_alpha x the
// previous tree's smallest split gain, child ids taken under the planner's id limit. Every
// expansion is speculative: the next planner's replay pops exactly the sequential growth's
// nodes (an expansion it never pops only permuted rows inside its own segment), so trees
// are identical to the batch path's (reference: DataParallelTreeMaker.java:219-295).
constexpr int kSubThreads = 1024;
constexpr int kSubU = 4;        // partition: rows per thread per step (kSubU x 16 wave counts)
constexpr int kSubFront = 160;  // local frontier entries (<= sub_max + 2 live)
constexpr int kSubHistU = 8;    // histogram: gathered rows in flight per lane
constexpr int kSubMaxSplits = 128;

struct SubArgs {
  const uint8_t* bins;   // row-major bins [N][stride]
  long long stride;
  const uint8_t* binsT;  // column-major bins [F][ncol]
  long long ncol;
  const int* rows_in;    // the batch input's row ids by position (nullptr: identity)
  const float2* gh_in;   // the batch input's (g, h) by position
  int* rows2;            // 2N ping-pong row ids
  float2* gh2;           // 2N ping-pong (g, h) (unused when ghr is set)
  const float2* ghr;     // (g, h) by ROW id (YTK_LW_GH_ROWS=1), else nullptr
  long long* hist;
  int B, F, Bp;
  const int* nbins_f;
  const uint8_t* fmask;
  int f0;
  const float* scales;       // fixed-point scales (g, h) of the tree
  const double* inv_scales;  // their inverses
};

// Rows [xb, xb + n) of rin (nullptr: identity) / ghin into the other half of the ping-pong
// buffers: left rows from the front, right rows from the back (the order inside a child is
// free: every downstream sum is exact). Returns the left count. s_c: 2 * 64 + 2 ints.
__device__ int sub_partition(const SubArgs& a, const int* rin, const float2* ghin, int xb, int n, int feat, int thr,
                             int N, int* s_c) {
  constexpr int NW = kSubThreads / kWave;
  constexpr int NE = kSubU * NW;
  static_assert(NE == kWave, "one lane of wave 0 per (step row, wave) count");
  const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
  const int sh = xb < N ? N : -N;
  const int lstart = xb + sh, rend = xb + sh + n, end = xb + n;
  const uint8_t* col = a.binsT + (size_t)feat * a.ncol;
  const unsigned long long lt = l == 0 ? 0ull : (~0ull >> (64 - l));
  int nl = 0, nr = 0;
  for (int base = xb; base < end; base += kSubU * kSubThreads) {
    int r[kSubU];
    float2 g[kSubU];
    bool ok[kSubU], lf[kSubU];
#pragma unroll
    for (int j = 0; j < kSubU; ++j) {
      const int pos = base + j * kSubThreads + tid;
      ok[j] = pos < end;
      r[j] = ok[j] ? (rin ? rin[pos] : pos) : 0;
      g[j] = (ok[j] && !a.ghr) ? ghin[pos] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < kSubU; ++j) lf[j] = ok[j] && (int)col[(unsigned)r[j]] <= thr;
    int lr[kSubU], rr[kSubU];
#pragma unroll
    for (int j = 0; j < kSubU; ++j) {
      const unsigned long long lm = __ballot(lf[j]), rm = __ballot(ok[j] && !lf[j]);
      lr[j] = __popcll(lm & lt);
      rr[j] = __popcll(rm & lt);
      if (l == 0) {
        s_c[j * NW + w] = __popcll(lm);
        s_c[NE + j * NW + w] = __popcll(rm);
      }
    }
    __syncthreads();
    if (w == 0) {  // exclusive scans of the 64 left and 64 right counts
      const int x = s_c[l], y = s_c[NE + l];
      int ix = x, iy = y;
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        const int ux = __shfl_up(ix, off, kWave), uy = __shfl_up(iy, off, kWave);
        if (l >= off) {
          ix += ux;
          iy += uy;
        }
      }
      s_c[l] = ix - x;
      s_c[NE + l] = iy - y;
      if (l == kWave - 1) {
        s_c[2 * NE] = ix;
        s_c[2 * NE + 1] = iy;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSubU; ++j) {
      if (!ok[j]) continue;
      const int dst = lf[j] ? lstart + nl + s_c[j * NW + w] + lr[j]
                            : rend - 1 - (nr + s_c[NE + j * NW + w] + rr[j]);
      a.rows2[dst] = r[j];
      if (!a.ghr) a.gh2[dst] = g[j];
    }
    nl += s_c[2 * NE];
    nr += s_c[2 * NE + 1];
    __syncthreads();  // s_c is rewritten by the next step
  }
  return nl;
}

// Exact histogram of the rows at positions [cb, cb + cn) of rows2 in LDS (hist_fx_kernel's
// bin rows of [32 g | 32 h] words at hist_lds_pos, the same fx_round), stored to `slot`.
__device__ void sub_hist(const SubArgs& a, unsigned long long* sm64, int cb, int cn, int slot, float sg, float sh) {
  constexpr int kRow = 64;
  const int tid = threadIdx.x;
  for (int i = tid; i < a.B * kRow; i += kSubThreads) sm64[i] = 0ull;
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, wr = lane >> 3, q = lane & 7;
  constexpr int RW = (kSubThreads / kWave) * 8;  // rows per block step (8 per wave instruction)
  const uint8_t* bseg = a.bins + 4 * q;
  int lpos[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) lpos[c] = hist_lds_pos(4 * q + c);
  const int end = cb + cn;
  for (int base = cb + wave * 8; base < end; base += RW * kSubHistU) {
    int r[kSubHistU];
    bool ok[kSubHistU];
#pragma unroll
    for (int j = 0; j < kSubHistU; ++j) {
      const int pos = base + j * RW + wr;
      ok[j] = pos < end;
      r[j] = a.rows2[ok[j] ? pos : cb];
    }
    unsigned d[kSubHistU];
    float2 v[kSubHistU];
#pragma unroll
    for (int j = 0; j < kSubHistU; ++j) {
      const int pos = base + j * RW + wr;
      d[j] = *reinterpret_cast<const unsigned*>(bseg + (size_t)(unsigned)r[j] * a.stride);
      const float2 t = a.ghr ? a.ghr[r[j]] : a.gh2[ok[j] ? pos : cb];
      v[j] = ok[j] ? t : make_float2(0.f, 0.f);  // rows past the end add 0
    }
#pragma unroll
    for (int j = 0; j < kSubHistU; ++j) {
      const unsigned long long gi = fx_round(v[j].x * sg), hi = fx_round(v[j].y * sh);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = (k + wr) & 3;
        const unsigned bin = __builtin_amdgcn_ubfe(d[j], 8 * c, 8);
        unsigned long long* e = sm64 + (bin * kRow + lpos[c]);
        atomicAdd(e, gi);
        atomicAdd(e + 32, hi);
      }
    }
  }
  __syncthreads();
  longlong2* out = reinterpret_cast<longlong2*>(a.hist + (size_t)slot * a.B * a.F * 2);
  for (int i = tid; i < a.B * 32; i += kSubThreads) {
    const int bin = i >> 5, fl = i & 31;
    if (fl < a.F) {
      const int li = bin * kRow + hist_lds_pos(fl);
      out[(size_t)bin * a.F + fl] = make_longlong2((long long)sm64[li], (long long)sm64[li + 32]);
    }
  }
  __syncthreads();  // the slot is read back (split search) and the LDS reused
}

// a child's split record -> its node fields (lw_apply_splits; canSplit: UpdateStrategy.java:50-53)
__device__ void sub_apply(const LwParams& p, const LwBufs& b, int sid, long long cnt, const SplitOut& o) {
  b.G[sid] = o.g;
  b.H[sid] = o.h;
  b.gl[sid] = o.gl;
  b.hl[sid] = o.hl;
  int feat = o.feat;
  float chg = o.loss_chg;
  if (!(o.h >= (double)p.mcw * 2.0 && cnt >= (long long)p.min_split_samples)) {
    chg = -INFINITY;
    feat = -1;
  }
  b.feat[sid] = feat;
  b.bin_a[sid] = o.bin_a;
  b.bin_b[sid] = o.bin_b;
  b.loss[sid] = chg;
  b.state[sid] = 1;
}

__global__ __launch_bounds__(kSubThreads) void lw_subtree_kernel(LwParams p, LwBufs b, SubArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm64[];  // histogram / split LDS
  __shared__ int s_c[2 * kSubU * (kSubThreads / kWave) + 2];
  __shared__ SplitOut s_rec[2];
  __shared__ int f_sid[kSubFront];
  __shared__ float f_loss[kSubFront], f_bl[kSubFront];
  __shared__ int s_nf, s_x, s_lc, s_splits;
  __shared__ float s_bl;
  if (b.st[LW_DONE]) return;
  const int nsub = b.sub[SUB_N];
  if ((int)blockIdx.x >= nsub) return;  // block-uniform
  const int tid = threadIdx.x;
  const int limit = b.sub[SUB_LIMIT];
  const int smax = min(p.sub_max, b.sub[SUB_REM] - 1);
  const float floor_gain = p.sub_alpha * __int_as_float(b.sub[SUB_LAMBDA]);
  const float sg = a.scales[0], sh = a.scales[1];
  const GainParams gp{p.mcw, p.l1, p.l2, p.max_abs_leaf, a.inv_scales[0], a.inv_scales[1]};
  longlong2* sh_hist = reinterpret_cast<longlong2*>(sm64);
  unsigned long long n_splits = 0, n_roots = 0;
  for (int e = blockIdx.x; e < nsub; e += gridDim.x) {
    ++n_roots;
    const int2 ent = b.sub_list[e];
    int X = ent.x, L = ent.y;
    bool root = true;
    float bl = b.loss[X];  // minimum gain on the path from P (P's own)
    if (tid == 0) {
      s_nf = 0;
      s_splits = 0;
    }
    __syncthreads();
    while (true) {
      // ---- split X into L, L + 1 (X's fields: written by earlier launches or by thread 0)
      const int xb = b.begin[X], n = b.cnt_local[X];
      const int feat = b.feat[X], thr = (b.bin_a[X] + b.bin_b[X]) >> 1;
      const int dep = b.depth[X] + 1;
      const int nl = sub_partition(a, root ? a.rows_in : a.rows2, root ? a.gh_in : a.gh2, xb, n, feat, thr, p.N, s_c);
      const int nr = n - nl;
      const int lb = xb + (xb < p.N ? p.N : -p.N);
      ++n_splits;
      // children that are terminal whatever the replay does get no histograms (lw_children_body)
      const bool need = !(p.max_depth >= 0 && dep == p.max_depth) &&
                        !(p.min_split_samples > 0 && nl < p.min_split_samples && nr < p.min_split_samples);
      if (tid == 0) {  // fresh children (lw_expand_one) with their segments (lw_children_body)
        for (int c = 0; c < 2; ++c) {
          const int sid = L + c;
          b.G[sid] = b.H[sid] = b.gl[sid] = b.hl[sid] = 0.0;
          b.cnt[sid] = c ? nr : nl;
          b.begin[sid] = c ? lb + nl : lb;
          b.cnt_local[sid] = c ? nr : nl;
          b.depth[sid] = dep;
          b.feat[sid] = -1;
          b.bin_a[sid] = b.bin_b[sid] = -1;
          b.lc[sid] = -1;
          b.tid[sid] = -1;
          b.seq[sid] = 0;
          b.state[sid] = 0;
          b.loss[sid] = -INFINITY;
        }
        b.lc[X] = L;
      }
      if (need) {
        const bool ls = nl < nr;  // build the smaller child, derive the other
        const int S = ls ? L : L + 1, G = ls ? L + 1 : L;
        sub_hist(a, sm64, ls ? lb : lb + nl, ls ? nl : nr, S, sg, sh);
        split_node_block<kSubThreads>(a.hist, a.B, a.F, a.Bp, a.nbins_f, a.fmask, a.f0, make_int4(S, 0, 0, 0),
                                      &s_rec[0], gp, sh_hist);
        __syncthreads();
        split_node_block<kSubThreads>(a.hist, a.B, a.F, a.Bp, a.nbins_f, a.fmask, a.f0, make_int4(G, X, S, 1),
                                      &s_rec[1], gp, sh_hist);
        __syncthreads();
        if (tid == 0) {
          sub_apply(p, b, S, ls ? nl : nr, s_rec[0]);
          sub_apply(p, b, G, ls ? nr : nl, s_rec[1]);
          for (int c = 0; c < 2; ++c) {  // frontier: splittable children above the gain floor
            const int sid = L + c;
            const float lc_loss = b.loss[sid];
            const float blc = fminf(bl, lc_loss);
            if (!lw_static_leaf(p, lc_loss, dep, c ? nr : nl) && blc >= floor_gain && s_nf < kSubFront) {
              f_sid[s_nf] = sid;
              f_loss[s_nf] = lc_loss;
              f_bl[s_nf] = blc;
              ++s_nf;
            }
          }
        }
      }
      // ---- next: the frontier's best gain (the subtree's own best-first order), if the
      // split budget and a child id pair under the planner's limit allow
      if (tid == 0) {
        int nx = -1;
        if (s_splits < smax && s_nf > 0) {
          int bi = 0;
          for (int i = 1; i < s_nf; ++i)
            if (f_loss[i] > f_loss[bi]) bi = i;
          int cur = __hip_atomic_load(&b.st[LW_N_SIDS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          int got = -1;
          while (cur + 2 <= limit) {
            const int old = atomicCAS(&b.st[LW_N_SIDS], cur, cur + 2);
            if (old == cur) {
              got = cur;
              break;
            }
            cur = old;
          }
          if (got >= 0) {
            nx = f_sid[bi];
            s_lc = got;
            s_bl = f_bl[bi];
            --s_nf;
            f_sid[bi] = f_sid[s_nf];
            f_loss[bi] = f_loss[s_nf];
            f_bl[bi] = f_bl[s_nf];
            ++s_splits;
          }
        }
        s_x = nx;
      }
      __syncthreads();
      const int nx = s_x;
      if (nx < 0) break;
      X = nx;
      L = s_lc;
      bl = s_bl;
      root = false;
      __syncthreads();  // s_x / s_lc / s_bl are rewritten by the next step
    }
  }
  if (b.prof && tid == 0) {
    atomicAdd(&b.prof[16], n_roots);   // subtree roots
    atomicAdd(&b.prof[17], n_splits);  // splits computed by subtrees (roots included)
  }
}

// hist[ids[i]] = 0 for the *n_dev listed slots (grid-stride over all their 16-B words).
// Slots listed with more than min_items items (the split-K reduce adds into them with
// atomics) are zeroed; the others are stored whole by the reduce / histogram kernels.
__global__ __launch_bounds__(256) void lw_zero_slots_kernel(longlong2* __restrict__ hist, long long slot_v2,
                                                            const int* __restrict__ ids, const int* __restrict__ n_dev,
                                                            const int2* __restrict__ range, int min_items) {
  const long long total = (long long)(*n_dev) * slot_v2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long s = i / slot_v2;
    if (range && range[s].y <= min_items) continue;
    hist[(size_t)ids[s] * slot_v2 + (i - s * slot_v2)] = make_longlong2(0, 0);
  }
}

// Multi-GPU batch message: msg = [kcap slots: the batch's built histograms in build order]
// [kcap * kCurStride words: the batch's split cursors]; one all-reduce per batch carries both
// (HistogramBuilder.java:95 + the child-count allreduce). Every rank plans the same batch, so
// build_ids / nb are identical; slots past nb are never read.
__global__ __launch_bounds__(256) void lw_msg_kernel(long long* __restrict__ hist, long long slot_elems,
                                                     const int* __restrict__ build_ids, const int* __restrict__ nb_dev,
                                                     unsigned long long* __restrict__ cursor, long long* __restrict__ msg,
                                                     int kcap, int unpack, const int* __restrict__ skip) {
  if (*skip) return;  // the tree is done: batches a host queued past its end move nothing
  const int nb = min(*nb_dev, kcap);
  const long long nh = (long long)nb * slot_elems;
  const long long ncur = (long long)kcap * kCurStride;
  const long long cur0 = (long long)kcap * slot_elems;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nh + ncur; i += (long long)gridDim.x * 256) {
    if (i < nh) {
      const long long kb = i / slot_elems, e = i - kb * slot_elems;
      long long* hs = hist + (size_t)build_ids[kb] * slot_elems + e;
      if (unpack) *hs = msg[i]; else msg[i] = *hs;
    } else {
      const long long j = i - nh;
      if (unpack) cursor[j] = (unsigned long long)msg[cur0 + j];
      else msg[cur0 + j] = (long long)cursor[j];
    }
  }
}

// Owner-computes batch sync (hist_sync = owner): rank r owns features [r fr, (r + 1) fr).
// Pack: x = P segments, segment r = the feature-r-block columns of the batch's built slots
// ([slot][bin][fl][2], zero padded to fr) then the batch's split cursors (replicated into
// every segment, so every rank gets their sums). Unpack: this rank's reduced segment (x)
// back into the slots' owned columns and the cursors (unpack 1: x is that segment; 2: x is
// the whole message, the segment at rank * its device-counted size). kcap >= 0: host-sized
// segments of kcap slot entries (zero beyond the built count) and kcap cursors (the RCCL
// loop, which knows the batch's split count); kcap < 0: sized by the device counts (peer).
__global__ __launch_bounds__(256) void lw_owner_kernel(long long* __restrict__ hist, long long slot_elems, int B,
                                                       int F, int fr, int P, int rank, const int* __restrict__ build_ids,
                                                       const int* __restrict__ nb_dev,
                                                       unsigned long long* __restrict__ cursor,
                                                       const int* __restrict__ k_dev, long long* __restrict__ x,
                                                       int kcap, int unpack, const int* __restrict__ skip) {
  if (kcap >= 0 && *skip) return;  // RCCL loop: batches queued past the tree's end move nothing
  const int nb = kcap >= 0 ? min(*nb_dev, kcap) : *nb_dev;
  const int ns = kcap >= 0 ? kcap : nb;
  const int kc = kcap >= 0 ? kcap : *k_dev;
  const long long sl = (long long)B * fr * 2;
  const long long nbe = (long long)ns * sl;
  const long long per = nbe + (long long)kc * kCurStride;
  const long long total = unpack ? per : per * P;
  if (unpack == 2) x += (long long)rank * per;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int r = unpack ? rank : (int)(i / per);
    const long long j = unpack ? i : i - (long long)r * per;
    long long* xi = x + i;
    if (j < nbe) {
      const long long kb = j / sl, e = j - kb * sl;
      const int c = (int)(e & 1);
      const long long q = e >> 1;
      const int fl = (int)(q % fr);
      const long long bin = q / fr;
      const int f = r * fr + fl;
      if (kb < nb && f < F) {
        long long* hs = hist + (size_t)build_ids[kb] * slot_elems + (bin * F + f) * 2 + c;
        if (unpack) *hs = *xi; else *xi = *hs;
      } else if (!unpack) {
        *xi = 0;
      }
    } else {
      const long long cj = j - nbe;
      if (unpack) cursor[cj] = (unsigned long long)*xi; else *xi = (long long)cursor[cj];
    }
  }
}

}  // namespace ytk

using namespace ytk;

namespace {
struct LwEngine {
  LwParams p;
  LwBufs b;
};
std::vector<LwEngine> g_lw;

// the workspace planner runs above the LDS planner's limits, or everywhere with
// YTK_LW_PLAN_GLOBAL=1 (tests: both planners must build the same trees)
bool lw_plan_global(int cap, int max_leaf) {
  const char* g = getenv("YTK_LW_PLAN_GLOBAL");
  return max_leaf > kLwLeafMax || cap > kLwCap || (g && g[0] == '1');
}

// planner workspace layout (16-B aligned arrays); base == nullptr: size only
size_t lw_carve_ws(char* base, int cap, int max_leaf, LwPlanWs& w) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off += (bytes + 15) & ~size_t(15);
    return q;
  };
  int q2 = 1;
  while (q2 < max_leaf + 8) q2 <<= 1;
  const size_t capr = ((size_t)cap + 127) & ~size_t(127);
  const size_t buf_u64 = std::max<size_t>(2 * (3 * (size_t)max_leaf + 8), capr + capr / 2 + 1);
  w.nd = (int4*)take(sizeof(int4) * cap);
  w.loss = (float*)take(sizeof(float) * cap);
  w.seq = (int*)take(sizeof(int) * cap);
  w.par = (int*)take(sizeof(int) * cap);
  w.ch = (int4*)take(sizeof(int4) * cap);
  w.hsid = (int*)take(sizeof(int) * (max_leaf + 8));
  w.akey = (unsigned long long*)take(8 * (size_t)q2);
  w.bkey = (unsigned long long*)take(8 * (2 * (size_t)max_leaf + 8));
  w.uid = (int*)take(sizeof(int) * (3 * (size_t)max_leaf + 16));
  w.buf = (unsigned long long*)take(8 * buf_u64);
  return off;
}
}  // namespace

extern "C" {

// ptrs: st, tnodes, G, H, gl, hl, cnt, begin, cnt_local, depth, feat, bin_a, bin_b, lc, tid, seq,
//       state, loss, heap, batch, part_feat, part_thr, part_begin, part_cnt, part_first,
//       part_shift, cursor, hist_items, build_ids, split_items, item_sid, split_out, root_cnt,
//       prof (0 = off), done_host (device pointer of a pinned int, 0 = off), zero_ids, zero_range,
//       plan workspace (ytk_lw_ws_bytes bytes; 0 when that is 0), sub words (int[8], zeroed),
//       sub_list (int2[max_leaf])
// ip: max_depth, max_leaf, min_split_samples, speculate, hist_target, min_rows, cap, N, split_groups, dist,
//     bin_bytes, sub_rows (0: no subtrees), sub_max
// fp: min_split_loss, mcw, l1, l2, max_abs_leaf, lr, sub_alpha. Returns an engine handle.
int ytk_lw_create(const uintptr_t* a, const int* ip, const float* fp) {
  LwEngine e;
  LwParams& p = e.p;
  p.max_depth = ip[0];
  p.max_leaf = ip[1];
  p.min_split_samples = ip[2];
  p.speculate = ip[3];
  if (p.speculate < 0 || p.speculate > 300) throw std::invalid_argument("lw_create: speculate percent must be in [0, 300]");
  p.hist_target = ip[4];
  p.min_rows = ip[5];
  p.cap = ip[6];
  p.N = ip[7];
  p.split_groups = ip[8] > 0 ? ip[8] : 1;
  p.dist = ip[9];
  p.bin_bytes = ip[10] == 2 ? 2 : 1;
  p.batch_cap = 0;
  p.slow_children = 0;
  // subtrees: single GPU, byte bins (multi-GPU batches all-reduce every built histogram)
  p.sub_rows = (p.dist || p.bin_bytes != 1) ? 0 : std::max(0, ip[11]);
  p.sub_max = std::min(std::max(0, ip[12]), kSubMaxSplits);
  p.sub_alpha = fp[6];
  p.min_split_loss = fp[0];
  p.mcw = fp[1];
  p.l1 = fp[2];
  p.l2 = fp[3];
  p.max_abs_leaf = fp[4];
  p.lr = fp[5];
  const bool big = lw_plan_global(p.cap, p.max_leaf);
  if (p.max_leaf < 2 || p.max_leaf > kLwLeafMaxBig || p.cap > kLwCapBig || p.cap < 2 * p.max_leaf + 3)
    throw std::invalid_argument("lw_create: need 2 <= max_leaf <= 4096 and 2 max_leaf + 3 <= cap <= 16384");
  LwBufs& b = e.b;
  int i = 0;
  b.st = (int*)a[i++];
  b.tnodes = (DNode*)a[i++];
  b.G = (double*)a[i++];
  b.H = (double*)a[i++];
  b.gl = (double*)a[i++];
  b.hl = (double*)a[i++];
  b.cnt = (long long*)a[i++];
  b.begin = (int*)a[i++];
  b.cnt_local = (int*)a[i++];
  b.depth = (int*)a[i++];
  b.feat = (int*)a[i++];
  b.bin_a = (int*)a[i++];
  b.bin_b = (int*)a[i++];
  b.lc = (int*)a[i++];
  b.tid = (int*)a[i++];
  b.seq = (int*)a[i++];
  b.state = (int*)a[i++];
  b.loss = (float*)a[i++];
  b.heap = (int*)a[i++];
  b.batch = (int*)a[i++];
  b.part_feat = (int*)a[i++];
  b.part_thr = (int*)a[i++];
  b.part_begin = (int*)a[i++];
  b.part_cnt = (int*)a[i++];
  b.part_first = (int*)a[i++];
  b.part_shift = (int*)a[i++];
  b.cursor = (unsigned long long*)a[i++];
  b.hist_items = (int4*)a[i++];
  b.build_ids = (int*)a[i++];
  b.split_items = (int4*)a[i++];
  b.item_sid = (int*)a[i++];
  b.split_out = (SplitOut*)a[i++];
  b.root_cnt = (const long long*)a[i++];
  b.prof = (unsigned long long*)a[i++];
  b.done_host = (int*)a[i++];
  b.zero_ids = (int*)a[i++];
  b.zero_range = (int2*)a[i++];
  char* ws = (char*)a[i++];  // planner workspace (ytk_lw_ws_bytes), large trees only
  if (big && !ws) throw std::invalid_argument("lw_create: the workspace planner (max_leaf > 512) needs its workspace");
  b.ws = LwPlanWs{};
  if (big) lw_carve_ws(ws, p.cap, p.max_leaf, b.ws);
  b.sub = (int*)a[i++];
  b.sub_list = (int2*)a[i++];
  if (p.sub_rows > 0 && (!b.sub || !b.sub_list)) throw std::invalid_argument("lw_create: subtrees need their buffers");
  g_lw.push_back(e);
  return (int)g_lw.size() - 1;
}

void ytk_lw_set_lr(int h, float lr) { g_lw.at(h).p.lr = lr; }
// splits per batch of the following planner launches (0: no cap)
void ytk_lw_set_batch_cap(int h, int cap) { g_lw.at(h).p.batch_cap = std::max(0, cap); }

// bytes of the planner workspace a (cap, max_leaf) engine needs (0: the LDS planner fits)
long long ytk_lw_ws_bytes(int cap, int max_leaf) {
  if (!lw_plan_global(cap, max_leaf)) return 0;
  LwPlanWs w;
  return (long long)lw_carve_ws(nullptr, cap, max_leaf, w);
}

// device address of pinned host memory (hipHostMalloc'ed by the caller's allocator)
uintptr_t ytk_host_device_ptr(uintptr_t host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(host), 0) != hipSuccess)
    throw std::runtime_error("hipHostGetDevicePointer failed (memory not pinned?)");
  return reinterpret_cast<uintptr_t>(d);
}

// which: 0 init (root), 1 plan
void ytk_lw_step(int h, int which, uintptr_t stream) {
  const LwEngine& e = g_lw.at(h);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (which) {
    case 0: hipLaunchKernelGGL(lw_init_kernel, dim3(1), dim3(kLwPlanThreads), 0, s, e.p, e.b); break;
    case 1:
      if (e.b.ws.nd)
        hipLaunchKernelGGL(lw_plan_kernel<true>, dim3(1), dim3(kLwPlanThreads), 0, s, e.p, e.b);
      else
        hipLaunchKernelGGL(lw_plan_kernel<false>, dim3(1), dim3(kLwPlanThreads), 0, s, e.p, e.b);
      break;
    default: throw std::runtime_error("bad lw step");
  }
  YTK_LAUNCH_CHECK();
}

// partition of the current batch (+ children planning in the last block); rows == 0:
// identity permutation (the root batch of an unsampled tree)
void ytk_lw_partition(int h, uintptr_t binsT, long long ncol, uintptr_t rows, uintptr_t ghp, uintptr_t rows_out,
                      uintptr_t gh_out, int max_blocks, uintptr_t stream, uintptr_t chunk_io) {
  // chunk_io (optional, >= max_blocks + max_blocks / 32 + 1 u64, the group sums zeroed once;
  // batches of <= kChunkScanMaxSplits splits): count
  // pass + one-block scan instead of the split cursor atomics (the root batch's chunks all
  // reserve on one cursor line)
  const LwEngine& e = g_lw.at(h);
  LwParams pp = e.p;  // YTK_PLAN_FAST=0: the children planning's general path (read per launch)
  {
    const char* pf = getenv("YTK_PLAN_FAST");
    pp.slow_children = (pf && pf[0] == '0') ? 1 : 0;
  }
  if (e.p.bin_bytes == 2) {  // uint16 bins (B > 256): the pipelined body with (g, h) prefetch
    const dim3 grid(std::max(1, std::min(max_blocks, kPartGrid)));
    hipLaunchKernelGGL((lw_partition_kernel<true, true, uint16_t>), grid, dim3(kPartThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), pp, e.b, (const uint16_t*)binsT, ncol,
                       (const int*)rows, (const float2*)ghp, (int*)rows_out, (float2*)gh_out, nullptr, nullptr);
    YTK_LAUNCH_CHECK();
    return;
  }
  // software-pipelined partition body, next chunk's row ids + (g, h) in flight (=2:
  // 3.41 -> 3.28-3.35 ms/tree, profiles/r2_partition_chunk.md); default (unset or 3): also the
  // next chunk's split-feature bytes, gathered once its row ids have arrived (500 trees
  // 4.013-4.023 -> 3.962-3.970 ms/tree, same trees; profiles/r6/fin/lwpf_*.json);
  // YTK_LW_PART_PREFETCH=1: row ids only (measured slower), 0: unpipelined -- ghp == 0 ((g, h)
  // row-indexed, only row ids move): row ids only
  const char* pf = getenv("YTK_LW_PART_PREFETCH");  // read per launch (~0.1 us): tests toggle it
  const bool prefetch = !(pf && pf[0] == '0');
  const dim3 grid(std::max(1, std::min(max_blocks, kPartGrid)));
  if (chunk_io && prefetch && ghp) {
    unsigned long long* cio = reinterpret_cast<unsigned long long*>(chunk_io);
    unsigned long long* gsum = cio + std::max(1, max_blocks);  // group sums past the counts
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const char* sk = getenv("YTK_PART_SCAN_KERNEL");  // 1: the separate scan launch (mode 2)
    const bool scan_launch = sk && sk[0] == '1';
    hipLaunchKernelGGL(lw_part_count_lean_kernel, dim3(std::max(1, max_blocks)), dim3(kPartThreads), 0, s, e.b,
                       (const uint8_t*)binsT, ncol, (const int*)rows, cio, scan_launch ? nullptr : gsum);
    if (scan_launch) {
      hipLaunchKernelGGL(lw_part_scan_kernel, dim3(1), dim3(kChunkScanThreads), 0, s, e.b, cio);
      hipLaunchKernelGGL((lw_partition_kernel<true, true, uint8_t, false, 2>), grid, dim3(kPartThreads), 0, s, pp,
                         e.b, (const uint8_t*)binsT, ncol, (const int*)rows, (const float2*)ghp, (int*)rows_out,
                         (float2*)gh_out, cio, gsum);
    } else {
      hipLaunchKernelGGL((lw_partition_kernel<true, true, uint8_t, false, 3>), grid, dim3(kPartThreads), 0, s, pp,
                         e.b, (const uint8_t*)binsT, ncol, (const int*)rows, (const float2*)ghp, (int*)rows_out,
                         (float2*)gh_out, cio, gsum);
    }
    YTK_LAUNCH_CHECK();
    return;
  }
  if (prefetch && (!pf || pf[0] == '3') && ghp)  // + the next chunk's split-feature bytes
    hipLaunchKernelGGL((lw_partition_kernel<true, true, uint8_t, true>), grid, dim3(kPartThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), pp, e.b, (const uint8_t*)binsT, ncol,
                       (const int*)rows, (const float2*)ghp, (int*)rows_out, (float2*)gh_out, nullptr, nullptr);
  else if (prefetch && !(pf && pf[0] == '1') && ghp)  // next chunk's (g, h) as well
    hipLaunchKernelGGL((lw_partition_kernel<true, true>), grid, dim3(kPartThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), pp, e.b, (const uint8_t*)binsT, ncol,
                       (const int*)rows, (const float2*)ghp, (int*)rows_out, (float2*)gh_out, nullptr, nullptr);
  else if (prefetch)
    hipLaunchKernelGGL(lw_partition_kernel<true>, grid, dim3(kPartThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       pp, e.b, (const uint8_t*)binsT, ncol, (const int*)rows, (const float2*)ghp, (int*)rows_out,
                       (float2*)gh_out, nullptr, nullptr);
  else
    hipLaunchKernelGGL(lw_partition_kernel<false>, grid, dim3(kPartThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       pp, e.b, (const uint8_t*)binsT, ncol, (const int*)rows, (const float2*)ghp, (int*)rows_out,
                       (float2*)gh_out, nullptr, nullptr);
  YTK_LAUNCH_CHECK();
}

// pack (unpack = 0) / unpack (1) the batch message of at most kcap splits (see lw_msg_kernel)
void ytk_lw_msg(int h, uintptr_t hist, long long slot_elems, uintptr_t msg, int kcap, int unpack, uintptr_t stream) {
  const LwEngine& e = g_lw.at(h);
  if (kcap <= 0) return;
  const long long n = (long long)kcap * (slot_elems + kCurStride);
  const int grid = (int)std::min<long long>((n + 255) / 256, 256 * 8);
  hipLaunchKernelGGL(lw_msg_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), (long long*)hist,
                     slot_elems, e.b.build_ids, e.b.st + LW_N_BUILD, e.b.cursor, (long long*)msg, kcap, unpack,
                     e.b.st + LW_DONE);
  YTK_LAUNCH_CHECK();
}

// owner-computes pack (unpack = 0: x = P segments) / unpack (1: x = this rank's segment) of
// the batch's built slots + split cursors; kcap < 0: sized by the device counts
void ytk_lw_owner(int h, uintptr_t hist, long long slot_elems, int B, int F, int fr, int P, int rank, uintptr_t x,
                  int kcap, int unpack, uintptr_t stream) {
  const LwEngine& e = g_lw.at(h);
  const int kmax = kcap >= 0 ? kcap : std::min(e.p.max_leaf, kLwLeafMax);
  const long long n = (long long)kmax * ((long long)B * fr * 2 + kCurStride) * (unpack ? 1 : P);
  if (n <= 0) return;
  const int grid = (int)std::min<long long>((n + 255) / 256, 256 * 8);
  hipLaunchKernelGGL(lw_owner_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), (long long*)hist,
                     slot_elems, B, F, fr, P, rank, e.b.build_ids, e.b.st + LW_N_BUILD, e.b.cursor,
                     e.b.st + LW_N_SPLIT, (long long*)x, kcap, unpack, e.b.st + LW_DONE);
  YTK_LAUNCH_CHECK();
}

// small-node subtrees of the current batch (after its split search; no-op when the
// engine has none). bins / binsT: uint8 row- / column-major; rows_in / gh_in: the batch's input
// (as ytk_lw_partition); ghr: row-indexed (g, h) (YTK_LW_GH_ROWS=1) or 0.
void ytk_lw_subtree(int h, uintptr_t bins, long long stride, uintptr_t binsT, long long ncol, uintptr_t rows_in,
                    uintptr_t gh_in, uintptr_t rows2, uintptr_t gh2, uintptr_t ghr, uintptr_t hist, int B, int F,
                    uintptr_t nbins_f, uintptr_t fmask, int f0, uintptr_t scales, uintptr_t inv_scales,
                    uintptr_t stream) {
  const LwEngine& e = g_lw.at(h);
  if (e.p.sub_rows <= 0) return;
  const int Bp = B + 1;
  if (F > 32 || B > 4 * kWave || stride % 32 != 0 || (size_t)F * Bp * 16 > kNodeLdsMax ||
      B * F > kNodeLoads * kNodeThreads)
    throw std::invalid_argument("lw_subtree: needs F <= 32, B <= 256, a 32-aligned bin stride");
  SubArgs a{(const uint8_t*)bins, stride, (const uint8_t*)binsT, ncol, (const int*)rows_in, (const float2*)gh_in,
            (int*)rows2, (float2*)gh2, (const float2*)ghr, (long long*)hist, B, F, Bp, (const int*)nbins_f,
            (const uint8_t*)fmask, f0, (const float*)scales, (const double*)inv_scales};
  const size_t lds = std::max((size_t)B * 64 * 8, (size_t)F * Bp * 16);
  const int grid = std::min(e.p.max_leaf, 256);
  hipLaunchKernelGGL(lw_subtree_kernel, dim3(grid), dim3(kSubThreads), lds, reinterpret_cast<hipStream_t>(stream),
                     e.p, e.b, a);
  YTK_LAUNCH_CHECK();
}

void ytk_lw_zero_slots(uintptr_t hist, long long slot_bytes, uintptr_t ids, uintptr_t n_dev, uintptr_t range,
                       int min_items, int grid, uintptr_t stream) {
  hipLaunchKernelGGL(lw_zero_slots_kernel, dim3(std::max(1, grid)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (longlong2*)hist, slot_bytes / 16, (const int*)ids,
                     (const int*)n_dev, (const int2*)range, min_items);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
