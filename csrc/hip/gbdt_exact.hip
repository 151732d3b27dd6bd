// Exact-greedy (feature-parallel) tree maker kernels (gfx950).
//
// Reference: J/optimizer/gbdt/FeatureParallelTreeMakerByLevel.java -- initNodeStats
// :277-312, findSplit :315-343, enumerateSplit :346-398 (every distinct value of a presorted
// column is a candidate: midpoint threshold, MIN_FEA_SPLIT_GAP = 1e-16f (Constants.java:34),
// min_child_hessian_sum on both sides, strictly-greater replacement in the scan order),
// resetPosition :424-444 (value < threshold goes left) -- over J/data/gbdt/FeatureColData.java
// :38-58 (every column sorted once by value).
//
// Layout: for each searched feature slot j, ord[j][0..n) are the row ids grouped into the
// level's node segments (one contiguous range per expanding node, the same ranges for every
// feature) and sorted by value inside each segment; val[j][i] is the row's value. A level is
// cut into TILES of at most kExTile positions that never straddle a node, so every per-tile
// result belongs to one node. A tree is one host call that enqueues, per level, eight
// fixed-grid launches (work counts in device words, no host round trip until the tree's
// records are read back):
//   sums<0>  per (feature, tile): exact int64 (g, h) sums of the tile's rows
//   scan<0>  per feature: exclusive tile prefixes inside each node (+ node totals, slot 0)
//   eval     per (feature, tile): in-tile exclusive scan -> left sums at every position, gap
//            test, both children's hessians, lossChg in double exactly as the reference, per
//            tile the best key (lossChg bits, lowest position), atomicMax per (feature, node)
//   decide   one block: best feature per node (strictly greater: lowest feature on ties),
//            split iff lossChg > min_split_loss within the leaf budget (a prefix count over
//            the level's nodes in expand order), node records, split feature / threshold
//   flag     per tile of slot 0: row -> left (value < threshold) / right / dropped
//   sums<1>  per (feature, tile): left rows of the tile
//   scan<1>  per feature: left offsets inside each node; slot 0's block also lays out the
//            children's segments and the next level's tile table
//   part     per (feature, tile): stable partition into the children's segments
// The last level (max_depth) runs sums<0> + scan<0> + decide only (its nodes are leaves).
#include "common.h"
#include "gbdt_split_node.h"

#include <algorithm>
#include <stdexcept>
#include <vector>

namespace ytk {

constexpr int kExThreads = 256;
constexpr int kExPer = 8;
constexpr int kExTile = kExThreads * kExPer;  // positions per tile
constexpr int kExScanThreads = 1024;

struct ExRec {  // one expanding node of a level (48 B)
  double G, H;
  long long cnt;
  float chg, thr, value;
  int feat, split, pad;
};
static_assert(sizeof(ExRec) == 48, "ExRec layout");

enum { EX_NT0 = 0, EX_NT1 = 1, EX_K0 = 2, EX_K1 = 3, EX_LEAF = 4, EX_ERR = 5, EX_WORDS = 8 };

struct ExArgs {
  const int* ord0;
  const float* val0;
  long long ld0;  // presorted columns [F][ld0]
  int* ordw[2];
  float* valw[2];
  long long ldw;  // work ping-pong [nf][ldw]
  int sampled;    // level 0 reads ordw[0] / valw[0] (the tree's kept rows) instead of ord0
  const int* fidx;  // feature of slot j, ascending
  int nf;
  const float* XT;
  long long ldx;  // raw values [F][ldx]
  const long long* q;  // [N][2] fixed-point (g, h)
  int4* tiles[2];  // (node, p0, p1, 0) per level parity
  int* nbeg[2];    // [Kmax + 1] node begins
  int* ftile[2];   // [Kmax + 1] first tile of each node
  int max_tiles, Kmax;
  int* ctl;
  long long* tsum;  // [nf][max_tiles][2]
  long long* tpre;  // [nf][max_tiles][2]
  long long* nbase;  // [nf][Kmax][2]
  unsigned long long* nkey;  // [nf][Kmax] (zero between levels: decide resets)
  long long* ntot;   // [Kmax][2]
  int* go_feat;
  float* go_thr;
  int* csplit;  // child index (2 * split rank) or -1
  int* cbeg;    // [Kmax][2]
  unsigned char* left_row;  // [N]
  ExRec* rec;
  const long long* rec_off;  // [levels] record offset of each level
  int* rec_k;
  GainParams gp;
  int min_split_samples, max_leaf;
  float msl, lr;
};

__device__ __forceinline__ const int* ex_src_ord(const ExArgs& a, int d, int j) {
  if (d == 0 && !a.sampled) return a.ord0 + (size_t)a.fidx[j] * a.ld0;
  return a.ordw[d & 1] + (size_t)j * a.ldw;
}
__device__ __forceinline__ const float* ex_src_val(const ExArgs& a, int d, int j) {
  if (d == 0 && !a.sampled) return a.val0 + (size_t)a.fidx[j] * a.ld0;
  return a.valw[d & 1] + (size_t)j * a.ldw;
}

__device__ __forceinline__ long long ld_agent(const long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// order-preserving unsigned image of a float (bits as exact.py's key: -0 below +0)
__device__ __forceinline__ unsigned f2ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// sum of (a, b) over the 256-thread block, returned to every thread
__device__ __forceinline__ void ex_block_sum2(long long& a, long long& b) {
  __shared__ long long s[2][kExThreads / kWave];
  const long long wa = readlane64(dpp_scan_add(a), kWave - 1), wb = readlane64(dpp_scan_add(b), kWave - 1);
  const int w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    s[0][w] = wa;
    s[1][w] = wb;
  }
  __syncthreads();
  a = b = 0;
#pragma unroll
  for (int k = 0; k < kExThreads / kWave; ++k) {
    a += s[0][k];
    b += s[1][k];
  }
}

// exclusive prefix of (a, b) over the block's threads in thread order (in place)
__device__ __forceinline__ void ex_block_excl2(long long& a, long long& b) {
  __shared__ long long s[2][kExThreads / kWave];
  const long long ia = dpp_scan_add(a), ib = dpp_scan_add(b);
  const int w = threadIdx.x / kWave;
  if (lane_id() == kWave - 1) {
    s[0][w] = ia;
    s[1][w] = ib;
  }
  __syncthreads();
  long long oa = 0, ob = 0;
#pragma unroll
  for (int k = 0; k < kExThreads / kWave; ++k)
    if (k < w) {
      oa += s[0][k];
      ob += s[1][k];
    }
  a = oa + ia - a;
  b = ob + ib - b;
}

__global__ __launch_bounds__(kExScanThreads) void ex_init_kernel(ExArgs a, int n) {
  const int nt = n > 0 ? (n + kExTile - 1) / kExTile : 0;
  for (int t = threadIdx.x; t < nt; t += kExScanThreads)
    a.tiles[0][t] = make_int4(0, t * kExTile, min(n, (t + 1) * kExTile), 0);
  if (threadIdx.x == 0) {
    if (nt > a.max_tiles) a.ctl[EX_ERR] = 1;
    a.ctl[EX_NT0] = min(nt, a.max_tiles);
    a.ctl[EX_NT1] = 0;
    a.ctl[EX_K0] = n > 0 ? 1 : 0;
    a.ctl[EX_K1] = 0;
    a.ctl[EX_LEAF] = 1;
    a.nbeg[0][0] = 0;
    a.nbeg[0][1] = n;
    a.ftile[0][0] = 0;
    a.ftile[0][1] = nt;
  }
}

// kMode 0: (g, h) sums of the tile's rows; 1: left rows of a split node's tile
template <int kMode>
__global__ __launch_bounds__(kExThreads) void ex_sums_kernel(ExArgs a, int d) {
  const int par = d & 1, t = blockIdx.x, j = blockIdx.y;
  if (t >= a.ctl[EX_NT0 + par]) return;
  const int4 tl = a.tiles[par][t];
  const int* ord = ex_src_ord(a, d, j);
  long long s0 = 0, s1 = 0;
  if (kMode == 0) {
    const longlong2* q2 = reinterpret_cast<const longlong2*>(a.q);
    for (int i = tl.y + threadIdx.x; i < tl.z; i += kExThreads) {
      const longlong2 v = q2[ord[i]];
      s0 += v.x;
      s1 += v.y;
    }
  } else if (a.csplit[tl.x] >= 0) {
    for (int i = tl.y + threadIdx.x; i < tl.z; i += kExThreads) s0 += a.left_row[ord[i]] == 1;
  }
  ex_block_sum2(s0, s1);
  if (threadIdx.x == 0) {
    long long* o = a.tsum + ((size_t)j * a.max_tiles + t) * 2;
    o[0] = s0;
    o[1] = s1;
  }
}

// Exclusive prefixes of the tiles inside their node, per feature (one block each). Slot 0's
// block then derives per node: mode 0 the totals, mode 1 the children's layout.
template <int kMode>
__global__ __launch_bounds__(kExScanThreads) void ex_scan_kernel(ExArgs a, int d) {
  const int par = d & 1, j = blockIdx.x, tid = threadIdx.x;
  const int nt = a.ctl[EX_NT0 + par], K = a.ctl[EX_K0 + par];
  const int4* tiles = a.tiles[par];
  const int* ftile = a.ftile[par];
  const long long* ts = a.tsum + (size_t)j * a.max_tiles * 2;
  long long* tp = a.tpre + (size_t)j * a.max_tiles * 2;
  long long* nb = a.nbase + (size_t)j * a.Kmax * 2;
  constexpr int kW = kExScanThreads / kWave;
  __shared__ long long s0[kW], s1[kW];
  __shared__ int si[kW];
  const int w = tid / kWave, l = lane_id();
  long long c0 = 0, c1 = 0;
  for (int base = 0; base < nt; base += kExScanThreads) {
    const int t = base + tid;
    long long x0 = 0, x1 = 0;
    int node = 0;
    if (t < nt) {
      x0 = ts[2 * t];
      x1 = ts[2 * t + 1];
      node = tiles[t].x;
    }
    const long long i0 = dpp_scan_add(x0), i1 = dpp_scan_add(x1);
    if (l == kWave - 1) {
      s0[w] = i0;
      s1[w] = i1;
    }
    __syncthreads();
    long long o0 = c0, o1 = c1, T0 = 0, T1 = 0;
    for (int k = 0; k < kW; ++k) {
      if (k < w) {
        o0 += s0[k];
        o1 += s1[k];
      }
      T0 += s0[k];
      T1 += s1[k];
    }
    const long long e0 = o0 + i0 - x0, e1 = o1 + i1 - x1;  // column prefix before tile t
    if (t < nt && ftile[node] == t) {
      nb[2 * node] = e0;
      nb[2 * node + 1] = e1;
    }
    __builtin_amdgcn_s_waitcnt(0);  // the node bases are in L2 before any wave reads them
    __syncthreads();
    if (t < nt) {
      tp[2 * t] = e0 - ld_agent(nb + 2 * node);
      tp[2 * t + 1] = e1 - ld_agent(nb + 2 * node + 1);
    }
    c0 += T0;
    c1 += T1;
    __syncthreads();
  }
  if (j != 0) return;
  // per-node sums (slot 0): node k's rows are its tiles, prefix difference
  auto node_sum = [&](int k, int c) -> long long {
    const long long b = ld_agent(nb + 2 * k + c);
    const long long e = (k + 1 < K) ? ld_agent(nb + 2 * (k + 1) + c) : (c == 0 ? c0 : c1);
    return e - b;
  };
  if (kMode == 0) {
    for (int k = tid; k < K; k += kExScanThreads) {
      a.ntot[2 * k] = node_sum(k, 0);
      a.ntot[2 * k + 1] = node_sum(k, 1);
    }
    return;
  }
  // children layout: split node k (child index c = csplit[k]) keeps its rows, left child
  // first: begins S_k and S_k + left_k, S_k = rows of the split nodes before k
  const int npar = par ^ 1;
  const int* nbg = a.nbeg[par];
  const int Kn = a.ctl[EX_K0 + npar];
  int carry = 0, tcarry = 0;
  for (int base = 0; base < K; base += kExScanThreads) {
    const int k = base + tid;
    int rows = 0, ntl = 0, left = 0, c = -1;
    if (k < K) {
      c = a.csplit[k];
      if (c >= 0) {
        rows = nbg[k + 1] - nbg[k];
        left = (int)node_sum(k, 0);
        ntl = (left + kExTile - 1) / kExTile + (rows - left + kExTile - 1) / kExTile;
      }
    }
    // block exclusive scans of rows and tile counts
    int ir = rows, it = ntl;
    for (int off = 1; off < kWave; off <<= 1) {
      const int vr = __shfl_up(ir, off, kWave), vt = __shfl_up(it, off, kWave);
      if (l >= off) {
        ir += vr;
        it += vt;
      }
    }
    if (l == kWave - 1) {
      s0[w] = ir;
      si[w] = it;
    }
    __syncthreads();
    int orr = carry, ot = tcarry, Tr = 0, Tt = 0;
    for (int q = 0; q < kW; ++q) {
      if (q < w) {
        orr += (int)s0[q];
        ot += si[q];
      }
      Tr += (int)s0[q];
      Tt += si[q];
    }
    if (c >= 0) {
      const int S = orr + ir - rows, ft = ot + it - ntl;
      a.cbeg[2 * k] = S;
      a.cbeg[2 * k + 1] = S + left;
      a.nbeg[npar][c] = S;
      a.nbeg[npar][c + 1] = S + left;
      a.ftile[npar][c] = ft;
      a.ftile[npar][c + 1] = ft + (left + kExTile - 1) / kExTile;
    }
    carry += Tr;
    tcarry += Tt;
    __syncthreads();
  }
  if (tid == 0) {
    a.nbeg[npar][Kn] = carry;
    a.ftile[npar][Kn] = tcarry;
    if (tcarry > a.max_tiles) a.ctl[EX_ERR] = 1;
    a.ctl[EX_NT0 + npar] = min(tcarry, a.max_tiles);
  }
  __builtin_amdgcn_s_waitcnt(0);  // the children's begins / first tiles are in L2
  __syncthreads();
  // the next level's tile table: tile t' of child c (binary search over the children's first tiles)
  const int ntn = min(tcarry, a.max_tiles);
  const int* ftn = a.ftile[npar];
  const int* nbn = a.nbeg[npar];
  for (int t = tid; t < ntn; t += kExScanThreads) {
    int lo = 0, hi = Kn - 1;  // last child with ftile <= t (children are non-empty: >= 1 tile)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (__hip_atomic_load(ftn + mid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= t) lo = mid;
      else hi = mid - 1;
    }
    const int c = lo;
    const int f0 = __hip_atomic_load(ftn + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int b0 = __hip_atomic_load(nbn + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int b1 = __hip_atomic_load(nbn + c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int p0 = b0 + (t - f0) * kExTile;
    a.tiles[npar][t] = make_int4(c, p0, min(b1, p0 + kExTile), 0);
  }
}

// this thread's kExPer consecutive positions of the tile
struct ExSpan {
  int i0;
  int n;
};
__device__ __forceinline__ ExSpan ex_span(int4 tl) {
  const int i0 = tl.y + threadIdx.x * kExPer;
  return {i0, max(0, min(kExPer, tl.z - i0))};
}

__global__ __launch_bounds__(kExThreads) void ex_eval_kernel(ExArgs a, int d) {
  const int par = d & 1, t = blockIdx.x, j = blockIdx.y;
  if (t >= a.ctl[EX_NT0 + par]) return;
  const int4 tl = a.tiles[par][t];
  const int k = tl.x;
  const int nb0 = a.nbeg[par][k], nb1 = a.nbeg[par][k + 1];
  const long long NG = a.ntot[2 * k], NH = a.ntot[2 * k + 1];
  const GainParams& gp = a.gp;
  const double G = (double)NG * gp.inv_sg, H = (double)NH * gp.inv_sh;
  // canSplit (UpdateStrategy.java:50-53): block-uniform
  if (!(H >= 2.0 * (double)gp.mcw && (nb1 - nb0) >= max(a.min_split_samples, 0))) return;
  const float root_gain = (float)calc_gain(G, H, gp);
  const int* ord = ex_src_ord(a, d, j);
  const float* val = ex_src_val(a, d, j);
  const longlong2* q2 = reinterpret_cast<const longlong2*>(a.q);
  const ExSpan sp = ex_span(tl);
  long long g[kExPer], h[kExPer];
  float v[kExPer];
  long long tg = 0, th = 0;
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    g[e] = h[e] = 0;
    v[e] = 0.f;
    if (e < sp.n) {
      const longlong2 x = q2[ord[sp.i0 + e]];
      g[e] = x.x;
      h[e] = x.y;
      v[e] = val[sp.i0 + e];
    }
    tg += g[e];
    th += h[e];
  }
  __shared__ float s_last[kExThreads];
  s_last[threadIdx.x] = sp.n > 0 ? v[sp.n - 1] : 0.f;
  long long lg = tg, lh = th;
  ex_block_excl2(lg, lh);  // includes a __syncthreads (s_last visible)
  const long long* tp = a.tpre + ((size_t)j * a.max_tiles + t) * 2;
  lg += tp[0];
  lh += tp[1];
  float vp = 0.f;
  if (sp.n > 0 && sp.i0 > nb0) vp = threadIdx.x > 0 ? s_last[threadIdx.x - 1] : val[sp.i0 - 1];
  unsigned long long best = 0;
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    if (e < sp.n) {
      const int i = sp.i0 + e;
      const float prev = e == 0 ? vp : v[e - 1];
      if (i > nb0 && fabsf(v[e] - prev) > 1e-16f && lh != 0) {
        const double Lg = (double)lg * gp.inv_sg, Lh = (double)lh * gp.inv_sh;
        const double Rg = (double)(NG - lg) * gp.inv_sg, Rh = (double)(NH - lh) * gp.inv_sh;
        if (Lh >= (double)gp.mcw && Rh >= (double)gp.mcw) {
          const float chg = (float)(calc_gain(Lg, Lh, gp) + calc_gain(Rg, Rh, gp) - (double)root_gain);
          if (!isnan(chg) && chg != -INFINITY) {
            const unsigned long long key = ((unsigned long long)f2ord(chg) << 32) | (0xffffffffu - (unsigned)i);
            best = key > best ? key : best;
          }
        }
      }
      lg += g[e];
      lh += h[e];
    }
  }
  // block max -> one atomic per tile
  __shared__ unsigned long long s_best[kExThreads / kWave];
  const unsigned long long wm = (unsigned long long)readlane64((long long)dpp_max_u64(best), kWave - 1);
  if (lane_id() == 0) s_best[threadIdx.x / kWave] = wm;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0;
    for (int q = 0; q < kExThreads / kWave; ++q) m = s_best[q] > m ? s_best[q] : m;
    if (m) atomicMax(a.nkey + (size_t)j * a.Kmax + k, m);
  }
}

__global__ __launch_bounds__(kExScanThreads) void ex_decide_kernel(ExArgs a, int d, int final_level) {
  const int par = d & 1, tid = threadIdx.x;
  const int K = a.ctl[EX_K0 + par];
  const int leaf0 = a.ctl[EX_LEAF];
  const bool budget = !final_level && (a.max_leaf <= 0 || leaf0 < a.max_leaf);
  const int room = a.max_leaf > 0 ? a.max_leaf - leaf0 : 0x7fffffff;
  ExRec* rec = a.rec + a.rec_off[d];
  const GainParams& gp = a.gp;
  constexpr int kW = kExScanThreads / kWave;
  __shared__ int s_w[kW];
  const int w = tid / kWave, l = lane_id();
  int carry = 0;
  for (int base = 0; base < K; base += kExScanThreads) {
    const int k = base + tid;
    float bchg = -INFINITY;
    int bj = -1;
    unsigned pos = 0;
    if (k < K) {
      for (int jj = 0; jj < a.nf; ++jj) {
        unsigned long long* kp = a.nkey + (size_t)jj * a.Kmax + k;
        const unsigned long long key = *kp;
        if (key) {
          *kp = 0;  // ready for the next level
          const float c = ord2f((unsigned)(key >> 32));
          if (budget && c > bchg) {
            bchg = c;
            bj = jj;
            pos = 0xffffffffu - (unsigned)key;
          }
        }
      }
    }
    const int elig = (k < K && budget && bchg > a.msl) ? 1 : 0;
    int inc = elig;
    for (int off = 1; off < kWave; off <<= 1) {
      const int v = __shfl_up(inc, off, kWave);
      if (l >= off) inc += v;
    }
    if (l == kWave - 1) s_w[w] = inc;
    __syncthreads();
    int rank = carry, tot = 0;
    for (int q = 0; q < kW; ++q) {
      if (q < w) rank += s_w[q];
      tot += s_w[q];
    }
    rank += inc - elig;  // eligible nodes before k in expand order
    if (k < K) {
      const double G = (double)a.ntot[2 * k] * gp.inv_sg, H = (double)a.ntot[2 * k + 1] * gp.inv_sh;
      const int split = elig && rank < room;
      ExRec r;
      r.G = G;
      r.H = H;
      r.cnt = a.nbeg[par][k + 1] - a.nbeg[par][k];
      r.chg = bchg;
      r.value = (float)node_value(G, H, gp) * a.lr;
      r.thr = 0.f;
      r.feat = -1;
      r.split = split;
      r.pad = 0;
      if (split) {
        const float* vv = ex_src_val(a, d, bj);
        r.thr = (vv[pos] + vv[pos - 1]) * 0.5f;
        r.feat = a.fidx[bj];
      }
      a.go_feat[k] = r.feat;
      a.go_thr[k] = r.thr;
      a.csplit[k] = split ? 2 * rank : -1;
      rec[k] = r;
    }
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) {
    const int nsplit = min(carry, room);
    const int Kn = 2 * nsplit;
    if (Kn > a.Kmax) a.ctl[EX_ERR] = 2;
    a.ctl[EX_LEAF] = leaf0 + nsplit;
    a.ctl[EX_K0 + (par ^ 1)] = min(Kn, a.Kmax);
    a.rec_k[d] = K;
  }
}

__global__ __launch_bounds__(kExThreads) void ex_flag_kernel(ExArgs a, int d) {
  const int par = d & 1, t = blockIdx.x;
  if (t >= a.ctl[EX_NT0 + par]) return;
  const int4 tl = a.tiles[par][t];
  const int f = a.go_feat[tl.x];
  const float thr = a.go_thr[tl.x];
  const int* ord = ex_src_ord(a, d, 0);
  for (int i = tl.y + threadIdx.x; i < tl.z; i += kExThreads) {
    const int r = ord[i];
    a.left_row[r] = f < 0 ? 2 : (a.XT[(size_t)f * a.ldx + r] < thr ? 1 : 0);
  }
}

__global__ __launch_bounds__(kExThreads) void ex_part_kernel(ExArgs a, int d) {
  const int par = d & 1, t = blockIdx.x, j = blockIdx.y;
  if (t >= a.ctl[EX_NT0 + par]) return;
  const int4 tl = a.tiles[par][t];
  const int k = tl.x;
  if (a.csplit[k] < 0) return;  // a leaf: its rows leave the order
  const int* ord = ex_src_ord(a, d, j);
  const float* val = ex_src_val(a, d, j);
  int* ordo = a.ordw[(d + 1) & 1] + (size_t)j * a.ldw;
  float* valo = a.valw[(d + 1) & 1] + (size_t)j * a.ldw;
  const ExSpan sp = ex_span(tl);
  int r[kExPer];
  float v[kExPer];
  unsigned lmask = 0;
  long long nl = 0, np = sp.n;
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    if (e < sp.n) {
      r[e] = ord[sp.i0 + e];
      v[e] = val[sp.i0 + e];
      if (a.left_row[r[e]] == 1) {
        lmask |= 1u << e;
        ++nl;
      }
    }
  }
  ex_block_excl2(nl, np);  // lefts / positions of the tile before this thread
  const long long* tp = a.tpre + ((size_t)j * a.max_tiles + t) * 2;
  const int lt = (int)tp[0];                   // lefts of the node before this tile
  const int before = tl.y - a.nbeg[par][k];    // node positions before this tile
  int li = a.cbeg[2 * k] + lt + (int)nl;
  int ri = a.cbeg[2 * k + 1] + (before - lt) + (int)(np - nl);
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    if (e < sp.n) {
      const int dst = (lmask >> e) & 1 ? li++ : ri++;
      ordo[dst] = r[e];
      valo[dst] = v[e];
    }
  }
}

struct ExEngine {
  ExArgs a;
};

}  // namespace ytk

using namespace ytk;

namespace {
std::vector<ExEngine> g_ex;
}

extern "C" {

// ptrs: ord0, val0, ordw0, ordw1, valw0, valw1, XT, tiles0, tiles1, nbeg0, nbeg1, ftile0,
//       ftile1, ctl, tsum, tpre, nbase, nkey, ntot, go_feat, go_thr, csplit, cbeg, left_row,
//       rec, rec_off, rec_k
// ip:   ld0, ldw, ldx, max_tiles, Kmax, min_split_samples, max_leaf
// fp:   mcw, l1, l2, max_abs_leaf, min_split_loss, lr
int ytk_ex_create(const uintptr_t* p, const long long* ip, const float* fp) {
  ExEngine e{};
  ExArgs& a = e.a;
  int i = 0;
  a.ord0 = (const int*)p[i++];
  a.val0 = (const float*)p[i++];
  a.ordw[0] = (int*)p[i++];
  a.ordw[1] = (int*)p[i++];
  a.valw[0] = (float*)p[i++];
  a.valw[1] = (float*)p[i++];
  a.XT = (const float*)p[i++];
  a.tiles[0] = (int4*)p[i++];
  a.tiles[1] = (int4*)p[i++];
  a.nbeg[0] = (int*)p[i++];
  a.nbeg[1] = (int*)p[i++];
  a.ftile[0] = (int*)p[i++];
  a.ftile[1] = (int*)p[i++];
  a.ctl = (int*)p[i++];
  a.tsum = (long long*)p[i++];
  a.tpre = (long long*)p[i++];
  a.nbase = (long long*)p[i++];
  a.nkey = (unsigned long long*)p[i++];
  a.ntot = (long long*)p[i++];
  a.go_feat = (int*)p[i++];
  a.go_thr = (float*)p[i++];
  a.csplit = (int*)p[i++];
  a.cbeg = (int*)p[i++];
  a.left_row = (unsigned char*)p[i++];
  a.rec = (ExRec*)p[i++];
  a.rec_off = (const long long*)p[i++];
  a.rec_k = (int*)p[i++];
  a.ld0 = ip[0];
  a.ldw = ip[1];
  a.ldx = ip[2];
  a.max_tiles = (int)ip[3];
  a.Kmax = (int)ip[4];
  a.min_split_samples = (int)ip[5];
  a.max_leaf = (int)ip[6];
  if (a.max_tiles < 1 || a.Kmax < 1) throw std::invalid_argument("ex_create: bad sizes");
  a.gp.mcw = fp[0];
  a.gp.l1 = fp[1];
  a.gp.l2 = fp[2];
  a.gp.max_abs_leaf = fp[3];
  a.msl = fp[4];
  a.lr = fp[5];
  g_ex.push_back(e);
  return (int)g_ex.size() - 1;
}

// Enqueue one tree: levels 0 .. depth - 1 search and split, level `depth` only records its
// nodes (leaves). q: [N][2] int64 fixed-point (g, h) with scales (inv_g, inv_h); fidx: the
// nf searched feature slots (ascending); n: rows in the tree (sampled: ordw[0] / valw[0]
// hold each slot's kept rows in value order).
void ytk_ex_tree(int h, uintptr_t q, uintptr_t fidx, int nf, int n, int sampled, double inv_g, double inv_h,
                 int depth, float lr, uintptr_t stream) {
  ExEngine& e = g_ex.at(h);
  ExArgs a = e.a;
  a.q = (const long long*)q;
  a.fidx = (const int*)fidx;
  a.nf = nf;
  a.sampled = sampled;
  a.gp.inv_sg = inv_g;
  a.gp.inv_sh = inv_h;
  a.lr = lr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (nf < 1 || nf > 65535) throw std::invalid_argument("ex_tree: bad feature count");
  const dim3 tg(a.max_tiles, nf), t1(a.max_tiles);
  hipLaunchKernelGGL(ex_init_kernel, dim3(1), dim3(kExScanThreads), 0, s, a, n);
  for (int d = 0; d <= depth; ++d) {
    const bool last = d == depth;
    hipLaunchKernelGGL(ex_sums_kernel<0>, last ? dim3(a.max_tiles, 1) : tg, dim3(kExThreads), 0, s, a, d);
    hipLaunchKernelGGL(ex_scan_kernel<0>, dim3(last ? 1 : nf), dim3(kExScanThreads), 0, s, a, d);
    if (!last) hipLaunchKernelGGL(ex_eval_kernel, tg, dim3(kExThreads), 0, s, a, d);
    hipLaunchKernelGGL(ex_decide_kernel, dim3(1), dim3(kExScanThreads), 0, s, a, d, last ? 1 : 0);
    if (last) break;
    hipLaunchKernelGGL(ex_flag_kernel, t1, dim3(kExThreads), 0, s, a, d);
    hipLaunchKernelGGL(ex_sums_kernel<1>, tg, dim3(kExThreads), 0, s, a, d);
    hipLaunchKernelGGL(ex_scan_kernel<1>, dim3(nf), dim3(kExScanThreads), 0, s, a, d);
    hipLaunchKernelGGL(ex_part_kernel, tg, dim3(kExThreads), 0, s, a, d);
  }
  YTK_LAUNCH_CHECK();
}

int ytk_ex_tile() { return kExTile; }

}  // extern "C"
