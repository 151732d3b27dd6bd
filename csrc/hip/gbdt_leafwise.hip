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
//                from an LDS event list), choose the next batch (top-k candidates by gain,
//                LDS bitonic sort), emit the partition work (device counts).
//   partition    partition_atomic_kernel: children land in the OTHER half of a 2N-entry
//                ping-pong row buffer (out_shift), so no copy-back of the segments.
//   lw_children  child counts from the split cursors, smaller child, histogram chunks,
//                split items (built + derived), the slots to zero.
//   zero / hist / reduce / split: the existing kernels with device-resident counts.
// Histogram slots are never recycled inside a tree (slot = speculative node id; a
// 255-leaf tree uses < 600 of them, ~70 MB of the 288 GB of HBM3E).
#include "common.h"
#include "gbdt_split_node.h"  // SplitOut
#include "gbdt_tree_node.h"   // DNode, node_leaf_value

#include <stdexcept>
#include <vector>

namespace ytk {

enum {
  LW_NUM_TNODES = 0,  // == ST_NUM_NODES of the level engine (finalize / raw-tree kernels)
  LW_NUM_LEAF, LW_N_SIDS, LW_N_SPLIT, LW_N_PBLK, LW_N_HIST, LW_N_SITEMS, LW_N_BUILD, LW_DONE,
  LW_SEQ, LW_N_HEAP, LW_OVERFLOW, LW_BATCHES, LW_EXPANDED, LW_N_ZERO, LW_WORDS = 16
};

constexpr int kLwThreads = 256;
constexpr int kLwCap = 2304;     // speculative nodes per tree (LDS-staged by the planner)
constexpr int kLwLeafMax = 512;   // max_leaf_cnt supported by the device engine
constexpr int kLwSort = 4096;     // candidate sort width (power of two >= kLwCap)
constexpr int kLwChunk = 2048;    // rows per partition block (partition_atomic_kernel CH)

struct LwParams {
  int max_depth, max_leaf, min_split_samples, speculate;
  float min_split_loss, mcw, l1, l2, max_abs_leaf, lr;
  int hist_target, min_rows, cap, N;  // N: half size of the ping-pong row buffers
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
  unsigned long long* cursor;  // [max_leaf] partition cursors ((right << 32) | left)
  int4* hist_items;            // [hist bound]
  int* build_ids;              // [max_leaf + 1] slots built this batch
  int4* split_items;           // [2 max_leaf + 2]
  int* item_sid;               // [2 max_leaf + 2]
  SplitOut* split_out;         // [2 max_leaf + 2]
  const long long* root_cnt;   // [0] local rows, [1] global rows
  unsigned long long* prof;    // optional [32]: planner phase times (wall clock ticks), rows
  int* zero_ids;               // [max_leaf + 1] built slots with != 1 histogram item
  int2* zero_range;            // [max_leaf + 1] their items [x, x + y)
};

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

// queue key: larger lossChg first, then the earlier push (seq) -- priority_queue order of
// LeafGrower::Entry (keys are unique: every push has its own seq)
__device__ __forceinline__ unsigned long long lw_key(float loss, int seq) {
  unsigned u = __float_as_uint(loss);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving float -> uint
  return ((unsigned long long)u << 32) | (unsigned long long)(0xffffffffu - (unsigned)seq);
}

constexpr int kQ = (kLwLeafMax + 8 + kWave - 1) / kWave;  // queue entries per lane (registers)

// one DPP step of a 64-bit max (lanes without a source keep their value)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void lw_dpp_max(unsigned& lo, unsigned& hi) {
  const unsigned olo = (unsigned)__builtin_amdgcn_update_dpp((int)lo, (int)lo, kCtrl, kRowMask, 0xf, false);
  const unsigned ohi = (unsigned)__builtin_amdgcn_update_dpp((int)hi, (int)hi, kCtrl, kRowMask, 0xf, false);
  const bool gt = ohi > hi || (ohi == hi && olo > lo);
  lo = gt ? olo : lo;
  hi = gt ? ohi : hi;
}

// wave-wide max of a u64 (row_shr 1/2/4/8 -> row maxima in lane 15 of each row,
// row_bcast 15/31 -> lane 63), broadcast with readlane
__device__ __forceinline__ unsigned long long lw_wave_max(unsigned long long v) {
  unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  lw_dpp_max<0x111, 0xf>(lo, hi);
  lw_dpp_max<0x112, 0xf>(lo, hi);
  lw_dpp_max<0x114, 0xf>(lo, hi);
  lw_dpp_max<0x118, 0xf>(lo, hi);
  lw_dpp_max<0x142, 0xa>(lo, hi);
  lw_dpp_max<0x143, 0xc>(lo, hi);
  lo = __builtin_amdgcn_readlane(lo, 63);
  hi = __builtin_amdgcn_readlane(hi, 63);
  return ((unsigned long long)hi << 32) | lo;
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
#pragma unroll
  for (int k = 0; k < kLwThreads / kWave; ++k) {
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
  const int per = (n + kLwThreads - 1) / kLwThreads;
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
__global__ __launch_bounds__(kLwThreads) void lw_init_kernel(LwParams p, LwBufs b) {
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
  }
  for (int k = threadIdx.x; k < nblk; k += kLwThreads)
    b.hist_items[k] = make_int4(0, k * ch, min((k + 1) * ch, n_local), 0);
}

__global__ __launch_bounds__(kLwThreads) void lw_plan_kernel(LwParams p, LwBufs b) {
  __shared__ float s_loss[kLwCap];
  __shared__ int s_cnt[kLwCap];
  __shared__ int s_lc[kLwCap];
  __shared__ int s_tid[kLwCap];
  __shared__ int s_seq[kLwCap];
  __shared__ short s_depth[kLwCap];
  __shared__ unsigned char s_state[kLwCap];
  __shared__ int s_hsid[kLwLeafMax + 8];
  // replay events (then reused as the candidate sort buffer: kLwSort u64 = 32 KiB)
  __shared__ unsigned long long s_buf[kLwSort];
  __shared__ int s_tmp[kLwThreads / kWave + 1];
  __shared__ int s_nev, s_blocked, s_nh, s_num_leaf, s_ntree, s_seqc, s_k, s_ncand;
  int* st = b.st;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid >> 6;
  if (st[LW_DONE]) return;
  unsigned long long t_prev = b.prof && tid == 0 ? wall_clock64() : 0ull;
  const int nsid = st[LW_N_SIDS];
  const double mcw2 = (double)p.mcw * 2.0;
  // A. split records of the previous batch (canSplit: UpdateStrategy.java:50-53)
  const int nsi = st[LW_N_SITEMS];
  for (int i = tid; i < nsi; i += kLwThreads) {
    const int sid = b.item_sid[i];
    const SplitOut o = b.split_out[i];
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
  __syncthreads();
  LW_TICK(0);
  // B. stage what the replay reads
  for (int i = tid; i < nsid; i += kLwThreads) {
    s_loss[i] = b.loss[i];
    s_cnt[i] = (int)b.cnt[i];
    s_lc[i] = b.lc[i];
    s_tid[i] = b.tid[i];
    s_seq[i] = b.seq[i];
    s_depth[i] = (short)b.depth[i];
    s_state[i] = (unsigned char)b.state[i];
  }
  int nh = st[LW_N_HEAP];
  for (int i = tid; i < nh; i += kLwThreads) s_hsid[i] = b.heap[i];
  __syncthreads();
  LW_TICK(1);
  // C. replay the queue as far as the known gains allow (wave 0). The queue lives in
  //    registers (entry i = slot i / 64 of lane i % 64); a pop is a register-local max,
  //    a DPP wave max and two readlanes -- no LDS round trip on the argmax path.
  int4* s_ev = reinterpret_cast<int4*>(s_buf);  // kLwSort / 2 events
  if (wid == 0) {
    unsigned long long qk[kQ];
    int qs[kQ];
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
      const int i = j * kWave + lane;
      qs[j] = i < nh ? s_hsid[i] : -1;
      qk[j] = i < nh ? lw_key(s_loss[qs[j]], s_seq[qs[j]]) : 0ull;
    }
    int num_leaf = st[LW_NUM_LEAF], ntree = st[LW_NUM_TNODES], seqc = st[LW_SEQ];
    int nev = 0, blocked = -1;
    unsigned long long r_prev = b.prof ? wall_clock64() : 0ull;
#define LW_RTICK(slot)                                                  \
  do {                                                                  \
    if (b.prof) {                                                       \
      const unsigned long long t_ = wall_clock64();                     \
      if (lane == 0) atomicAdd(&b.prof[slot], t_ - r_prev);             \
      r_prev = t_;                                                      \
    }                                                                   \
  } while (0)
    while (nh > 0) {
      const int used = (nh + kWave - 1) / kWave;
      if (p.max_leaf > 0 && num_leaf == p.max_leaf) {
        // leaf budget used: every queued node pops as a leaf (independent of the order)
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
          const int i = j * kWave + lane;
          if (j < used && i < nh) {
            const int sid = qs[j];
            s_ev[nev + i] = make_int4(EV_LEAF, sid, s_tid[sid], 0);
            s_state[sid] = 2;
          }
        }
        nev += nh;
        nh = 0;
        break;
      }
      unsigned long long mine = 0ull;
#pragma unroll
      for (int j = 0; j < kQ; ++j)
        if (j < used && qk[j] > mine) mine = qk[j];
      LW_RTICK(16);
      const unsigned long long best = lw_wave_max(mine);
      LW_RTICK(17);
      int myj = -1;
#pragma unroll
      for (int j = 0; j < kQ; ++j)
        if (j < used && qk[j] == best) myj = j;
      const int lb = (int)__ffsll((long long)__ballot(myj >= 0)) - 1;  // keys are unique
      const int jb = __builtin_amdgcn_readlane(myj, lb);
      int sv = 0;
#pragma unroll
      for (int j = 0; j < kQ; ++j)
        if (j == jb) sv = qs[j];
      const int sid = __builtin_amdgcn_readlane(sv, lb);
      LW_RTICK(18);
      const float chg = s_loss[sid];
      const bool leaf = !(chg > p.min_split_loss) || (p.max_depth >= 0 && (int)s_depth[sid] == p.max_depth) ||
                        (p.min_split_samples > 0 && s_cnt[sid] < p.min_split_samples);
      const int lcs = s_lc[sid];
      if (!leaf && lcs < 0) { blocked = sid; break; }
      {  // remove entry (jb, lb): the last entry moves into its place
        const int il = nh - 1, jl = il / kWave, ll = il % kWave;
        unsigned long long kl = 0ull;
        int sl = 0;
#pragma unroll
        for (int j = 0; j < kQ; ++j)
          if (j == jl) { kl = qk[j]; sl = qs[j]; }
        const unsigned klo = __builtin_amdgcn_readlane((unsigned)kl, ll);
        const unsigned khi = __builtin_amdgcn_readlane((unsigned)(kl >> 32), ll);
        const int sls = __builtin_amdgcn_readlane(sl, ll);
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
          if (lane == lb && j == jb) { qk[j] = ((unsigned long long)khi << 32) | klo; qs[j] = sls; }
          if (lane == ll && j == jl) { qk[j] = 0ull; qs[j] = -1; }
        }
      }
      --nh;
      LW_RTICK(19);
      if (leaf) {
        if (lane == 0) {
          s_ev[nev] = make_int4(EV_LEAF, sid, s_tid[sid], 0);
          s_state[sid] = 2;
        }
        ++nev;
      } else {
        const int t = s_tid[sid], lt = ntree;
        ntree += 2;
        ++num_leaf;
        const int l = lcs, r = lcs + 1;
        const float loss_l = s_loss[l], loss_r = s_loss[r];
        const bool term = (p.max_depth >= 0 && p.max_depth == (int)s_depth[l]) ||
                          (p.max_leaf > 0 && p.max_leaf == num_leaf) ||
                          (p.min_split_samples > 0 && s_cnt[l] < p.min_split_samples &&
                           s_cnt[r] < p.min_split_samples);
        if (lane == 0) {
          s_tid[l] = lt;
          s_tid[r] = lt + 1;
          s_state[sid] = 2;
          s_ev[nev] = make_int4(EV_SPLIT, sid, t, lt);
          if (term) {
            s_ev[nev + 1] = make_int4(EV_LEAFIFY, sid, lt, 0);
            s_state[l] = s_state[r] = 2;
          } else {
            s_seq[l] = seqc;
            s_seq[r] = seqc + 1;
          }
        }
        nev += term ? 2 : 1;
        if (!term) {  // push both children at entries nh, nh + 1
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int ip = nh + c, jp = ip / kWave, lp = ip % kWave;
            const unsigned long long kc = lw_key(c == 0 ? loss_l : loss_r, seqc + c);
#pragma unroll
            for (int j = 0; j < kQ; ++j)
              if (lane == lp && j == jp) { qk[j] = kc; qs[j] = c == 0 ? l : r; }
          }
          nh += 2;
          seqc += 2;
        }
      }
      __builtin_amdgcn_wave_barrier();
      LW_RTICK(20);
      if (b.prof && lane == 0) atomicAdd(&b.prof[21], 1ull);
    }
#undef LW_RTICK
    // the remaining queue, compact in [0, nh)
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
      const int i = j * kWave + lane;
      if (i < nh) s_hsid[i] = qs[j];
    }
    if (lane == 0) {
      s_nev = nev;
      s_blocked = blocked;
      s_nh = nh;
      s_num_leaf = num_leaf;
      s_ntree = ntree;
      s_seqc = seqc;
    }
  }
  __syncthreads();
  LW_TICK(2);
  // D. tree nodes finalised by the replay (independent writes, all lanes)
  const int nev = s_nev;
  for (int e = tid; e < nev; e += kLwThreads) {
    const int4 ev = s_ev[e];
    const int sid = ev.y;
    if (ev.x == EV_LEAF) {
      lw_write_node(b.tnodes[ev.z], b, sid, true, b.G[sid], b.H[sid], b.loss[sid], b.cnt[sid], -1, p);
    } else if (ev.x == EV_SPLIT) {
      lw_write_node(b.tnodes[ev.z], b, sid, false, b.G[sid], b.H[sid], b.loss[sid], b.cnt[sid], ev.w, p);
    } else {  // children made leaves right away: sums from the parent's best split
      const int l = s_lc[sid];
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
  if (blocked >= 0) {
    const int remaining = p.max_leaf > 0 ? p.max_leaf - num_leaf : 1;
    const int fr = p.cap - nsid;
    // keep one net node pair per future split (LeafGrower slack rule): never runs dry
    k = p.speculate ? max(1, min(remaining, (fr - remaining - 1) >> 1)) : 1;
    if (fr < 2) k = 0;
  }
  if (k > 0) {
    // candidates: known gain, not expanded, not final, splittable by the static rules
    const int per = (nsid + kLwThreads - 1) / kLwThreads;
    const int i0 = min(nsid, tid * per), i1 = min(nsid, i0 + per);
    int c = 0;
    for (int i = i0; i < i1; ++i)
      c += (s_state[i] == 1 && s_lc[i] < 0 && s_loss[i] > p.min_split_loss &&
            (p.max_depth < 0 || (int)s_depth[i] < p.max_depth) &&
            (p.min_split_samples <= 0 || s_cnt[i] >= p.min_split_samples)) ? 1 : 0;
    int ncand;
    int pos = lw_scan(c, s_tmp, &ncand);
    for (int i = i0; i < i1; ++i) {
      if (s_state[i] == 1 && s_lc[i] < 0 && s_loss[i] > p.min_split_loss &&
          (p.max_depth < 0 || (int)s_depth[i] < p.max_depth) &&
          (p.min_split_samples <= 0 || s_cnt[i] >= p.min_split_samples)) {
        unsigned u = __float_as_uint(s_loss[i]);
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        s_buf[pos++] = (i == blocked) ? ~0ull
                                      : (((unsigned long long)u << 32) | (unsigned long long)(0xffffffffu - (unsigned)i));
      }
    }
    __syncthreads();
    if (ncand > k) {
      // top-k: bitonic sort (descending) of the candidate keys, zero padded
      int n2 = 1;
      while (n2 < ncand) n2 <<= 1;
      for (int i = ncand + tid; i < n2; i += kLwThreads) s_buf[i] = 0ull;
      __syncthreads();
      for (int size = 2; size <= n2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int t = tid; t < (n2 >> 1); t += kLwThreads) {
            const int lo = 2 * t - (t & (stride - 1));
            const int hi = lo + stride;
            const bool desc = (lo & size) == 0;
            const unsigned long long a = s_buf[lo], c2 = s_buf[hi];
            if ((a < c2) == desc) {
              s_buf[lo] = c2;
              s_buf[hi] = a;
            }
          }
          __syncthreads();
        }
      }
    }
    if (tid == 0) {
      s_k = min(k, ncand);
      s_ncand = ncand;
    }
    __syncthreads();
    k = s_k;
  }
  LW_TICK(4);
  // F. expand the batch: children ids, partition descriptors (chunks of kLwChunk rows)
  for (int j = tid; j < k; j += kLwThreads) {
    const unsigned long long key = s_buf[j];
    const int P = (key == ~0ull) ? blocked : (int)(0xffffffffu - (unsigned)(key & 0xffffffffull));
    const int lc = nsid + 2 * j;
    s_lc[P] = lc;
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
    b.part_first[j] = (cnt + kLwChunk - 1) / kLwChunk;
    b.cursor[j] = 0ull;
  }
  __syncthreads();
  const int nblocks = k > 0 ? lw_scan_array(b.part_first, k, s_tmp) : 0;
  LW_TICK(5);
  // G. write back the replay state
  for (int i = tid; i < nsid; i += kLwThreads) {
    b.lc[i] = s_lc[i];
    b.tid[i] = s_tid[i];
    b.seq[i] = s_seq[i];
    b.state[i] = s_state[i];
  }
  for (int i = tid; i < nh; i += kLwThreads) b.heap[i] = s_hsid[i];
  if (tid == 0) {
    st[LW_NUM_LEAF] = num_leaf;
    st[LW_NUM_TNODES] = s_ntree;
    st[LW_SEQ] = s_seqc;
    st[LW_N_HEAP] = nh;
    st[LW_N_SPLIT] = k;
    st[LW_N_PBLK] = nblocks;
    st[LW_N_SIDS] = nsid + 2 * k;
    if (k == 0) {
      st[LW_DONE] = 1;
      if (blocked >= 0) st[LW_OVERFLOW] = 1;  // cannot happen with cap >= max_leaf + 2
    } else {
      st[LW_BATCHES] += 1;
      st[LW_EXPANDED] += k;
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
__global__ __launch_bounds__(kLwThreads) void lw_children_kernel(LwParams p, LwBufs b) {
  __shared__ int s_need[kLwLeafMax], s_flag[kLwLeafMax];
  __shared__ int s_small[kLwLeafMax], s_first[kLwLeafMax], s_beg[kLwLeafMax], s_cntb[kLwLeafMax];
  __shared__ int s_nch[kLwLeafMax], s_zflag[kLwLeafMax];
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
  for (int j = tid; j < k; j += kLwThreads) {
    const int P = b.batch[j];
    const int L = b.lc[P], R = L + 1;
    const int lloc = (int)(b.cursor[j] & 0xffffffffull);
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
    const bool left_small = lloc < rcnt;
    s_need[j] = need ? 1 : 0;
    s_flag[j] = need ? 1 : 0;
    s_small[j] = left_small ? L : R;
    if (need) atomicAdd(&s_total, (unsigned long long)(left_small ? lloc : rcnt));
  }
  __syncthreads();
  const int nb = lw_scan_array(s_need, k, s_tmp);  // s_need = build index
  const long long total = (long long)s_total;
  const int ch = (int)max((long long)p.min_rows, (total + p.hist_target - 1) / max(1, p.hist_target));
  for (int j = tid; j < k; j += kLwThreads) {
    if (!s_flag[j]) continue;
    const int kb = s_need[j];
    const int P = b.batch[j];
    const int S = s_small[j];
    const int L = b.lc[P];
    const int G = (S == L) ? L + 1 : L;
    b.build_ids[kb] = S;
    b.split_items[kb] = make_int4(S, 0, 0, 0);
    b.item_sid[kb] = S;
    b.split_items[nb + kb] = make_int4(G, P, S, 1);
    b.item_sid[nb + kb] = G;
    s_beg[kb] = b.begin[S];
    s_cntb[kb] = b.cnt_local[S];
  }
  __syncthreads();
  for (int kb = tid; kb < nb; kb += kLwThreads) {
    // floor(rows / ch) equal chunks (between ch and 2 ch rows each): no short tail
    // chunk paying a whole 128-KiB LDS clear + flush for a few rows
    const int c = s_cntb[kb] == 0 ? 0 : max(1, s_cntb[kb] / ch);
    s_first[kb] = c;
    s_nch[kb] = c;
    s_zflag[kb] = c != 1 ? 1 : 0;  // sole-item slots are stored directly by the hist kernel
  }
  __syncthreads();
  const int nitems = lw_scan_array(s_first, nb, s_tmp);
  const int nzero = lw_scan_array(s_zflag, nb, s_tmp);  // s_zflag = index among the multi-item slots
  for (int kb = tid; kb < nb; kb += kLwThreads) {
    if (s_nch[kb] != 1) {
      const int z = s_zflag[kb];
      b.zero_ids[z] = b.build_ids[kb];
      b.zero_range[z] = make_int2(s_first[kb], s_nch[kb]);
    }
  }
  for (int q = tid; q < nitems; q += kLwThreads) {
    int lo = 0, hi = nb - 1;  // last build with s_first <= q
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_first[mid] <= q) lo = mid; else hi = mid - 1;
    }
    const int jq = q - s_first[lo];
    const int nc = s_nch[lo];
    const long long cnt = s_cntb[lo];
    const int cb = s_beg[lo] + (int)(cnt * jq / nc);
    const int ce = s_beg[lo] + (int)(cnt * (jq + 1) / nc);
    b.hist_items[q] = make_int4(b.build_ids[lo], cb, ce, nc == 1 ? 1 : 0);
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

}  // namespace ytk

using namespace ytk;

namespace {
struct LwEngine {
  LwParams p;
  LwBufs b;
};
std::vector<LwEngine> g_lw;
}  // namespace

extern "C" {

// ptrs: st, tnodes, G, H, gl, hl, cnt, begin, cnt_local, depth, feat, bin_a, bin_b, lc, tid, seq,
//       state, loss, heap, batch, part_feat, part_thr, part_begin, part_cnt, part_first,
//       part_shift, cursor, hist_items, build_ids, split_items, item_sid, split_out, root_cnt,
//       prof (0 = off), zero_ids, zero_range
// ip: max_depth, max_leaf, min_split_samples, speculate, hist_target, min_rows, cap, N
// fp: min_split_loss, mcw, l1, l2, max_abs_leaf, lr. Returns an engine handle.
int ytk_lw_create(const uintptr_t* a, const int* ip, const float* fp) {
  LwEngine e;
  LwParams& p = e.p;
  p.max_depth = ip[0];
  p.max_leaf = ip[1];
  p.min_split_samples = ip[2];
  p.speculate = ip[3];
  p.hist_target = ip[4];
  p.min_rows = ip[5];
  p.cap = ip[6];
  p.N = ip[7];
  p.min_split_loss = fp[0];
  p.mcw = fp[1];
  p.l1 = fp[2];
  p.l2 = fp[3];
  p.max_abs_leaf = fp[4];
  p.lr = fp[5];
  if (p.max_leaf < 2 || p.max_leaf > kLwLeafMax || p.cap > kLwCap || p.cap < p.max_leaf + 2)
    throw std::invalid_argument("lw_create: need 2 <= max_leaf <= 512 and max_leaf + 2 <= cap <= 2304");
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
  b.zero_ids = (int*)a[i++];
  b.zero_range = (int2*)a[i++];
  g_lw.push_back(e);
  return (int)g_lw.size() - 1;
}

void ytk_lw_set_lr(int h, float lr) { g_lw.at(h).p.lr = lr; }

// which: 0 init (root), 1 plan, 2 children
void ytk_lw_step(int h, int which, uintptr_t stream) {
  const LwEngine& e = g_lw.at(h);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (which) {
    case 0: hipLaunchKernelGGL(lw_init_kernel, dim3(1), dim3(kLwThreads), 0, s, e.p, e.b); break;
    case 1: hipLaunchKernelGGL(lw_plan_kernel, dim3(1), dim3(kLwThreads), 0, s, e.p, e.b); break;
    case 2: hipLaunchKernelGGL(lw_children_kernel, dim3(1), dim3(kLwThreads), 0, s, e.p, e.b); break;
    default: throw std::runtime_error("bad lw step");
  }
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
