// Exact-greedy (feature-parallel) tree maker kernels (gfx950).
//
// Reference: J/optimizer/gbdt/FeatureParallelTreeMakerByLevel.java -- initNodeStats
// :277-312, findSplit :315-343, enumerateSplit :346-398 (every distinct value of a presorted
// column is a candidate: midpoint threshold, MIN_FEA_SPLIT_GAP = 1e-16f (Constants.java:34),
// min_child_hessian_sum on both sides, strictly-greater replacement in the scan order),
// resetPosition :424-444 (value < threshold goes left) -- over J/data/gbdt/FeatureColData.java
// :38-58 (every column sorted once by value).
//
// Layout: for each searched feature slot j, position i of the level's order holds a row id
// ord[j][i], its value val[j][i] and its (g, h) qv[j][i] (float32, converted to the exact
// int64 fixed point where it is summed: 8 instead of 16 B per position moved); the rows of one
// node are contiguous (the same ranges for every feature) and sorted by value. (g, h) travel
// with the rows (gathered once per tree), so the split scan reads every array sequentially. A
// level is cut into TILES of <= kExTile positions that never straddle a node. Per level:
//   eval     per (feature, tile), in ticket order: tile (g, h) aggregate, decoupled
//            look-back over the node's earlier tiles for the exact int64 prefix, left sums
//            at every position, gap test, both children's hessians, lossChg in double as
//            the reference, tile best key -> atomicMax per (feature, node)
//   decide   one block: best feature per node (strictly greater: lowest feature on ties),
//            split iff lossChg > min_split_loss within the leaf budget (a prefix count over
//            the level's nodes in expand order), node records, split feature / threshold
//   flag     per tile of slot 0: row -> left / right / dropped, tile partials (left rows,
//            left (g, h), right (g, h))
//   layout   one block: node sums of the partials -> the children's exact (g, h) totals,
//            segments, first tiles and the next level's tile table
//   part     per (feature, tile), in ticket order: left-count look-back inside the node,
//            stable partition of (row, value, (g, h)) into the children's segments
// The last level (max_depth) runs decide only (its nodes are leaves; their totals came from
// the previous layout). Look-back status words pack (value << 2 | flag): the fixed-point
// scales leave |sums| < 2^60 (the caller passes 4 N to the scale rule).
#include "common.h"
#include "gbdt_split_node.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <vector>

namespace ytk {

constexpr int kExThreads = 256;
constexpr int kExPer = 8;
constexpr int kExTile = kExThreads * kExPer;  // positions per tile
constexpr int kExBig = 1024;                  // single-block kernels

struct ExRec {  // one expanding node of a level (48 B)
  double G, H;
  long long cnt;
  float chg, thr, value;
  int feat, split, pad;
};
static_assert(sizeof(ExRec) == 48, "ExRec layout");

// ctl words; tickets of level d's eval / part at kExTicket + 2 d (+ 1)
enum { EX_NT0 = 0, EX_NT1 = 1, EX_K0 = 2, EX_K1 = 3, EX_LEAF = 4, EX_ERR = 5, EX_TICKET = 16, EX_CTL_WORDS = 128 };

struct ExArgs {
  const int* ord0;
  const float* val0;
  long long ld0;  // presorted columns [F][ld0]
  int* ordw[2];
  float* valw[2];
  float2* qvw[2];     // [nf][ldw] (g, h)
  long long ldw;      // work ping-pong [nf][ldw]
  int sampled;        // level 0 reads ordw[0] / valw[0] (the tree's kept rows) instead of ord0
  const int* fidx;    // feature of slot j, ascending
  int nf;
  const float* XT;
  long long ldx;        // raw values [F][ldx]
  const float2* gh;     // [N] (g, h) by row
  float sg, sh;         // fixed-point scales (powers of two): q = rint(g * sg)
  int4* tiles[2];       // (node, p0, p1, 0) per level parity
  int* nbeg[2];         // [Kmax + 1] node begins
  int* ftile[2];        // [Kmax + 1] first tile of each node
  int max_tiles, Kmax;
  int* ctl;
  unsigned long long* st_gh;   // [nf][max_tiles][2] eval look-back words
  unsigned long long* st_cnt;  // [nf][max_tiles] part look-back words
  long long* tpart;   // [max_tiles][5] flag partials: left rows, left g, left h, right g, right h
  long long* nbase;   // [Kmax + 1][5] layout scratch
  unsigned long long* nkey;  // [nf][Kmax] (zero between levels: decide resets)
  long long* ntot;    // [Kmax][2] totals of the current level's nodes
  int* go_feat;
  float* go_thr;
  int* csplit;  // child index (2 * split rank) or -1
  int* cbeg;    // [Kmax][2]
  unsigned char* left_row;  // [N]
  unsigned* left_bits;      // [ceil(N / 32)]: left_row == 1 as bits (behind left_row's bytes)
  ExRec* rec;
  const long long* rec_off;  // [levels] record offset of each level
  int* rec_k;
  GainParams gp;
  int min_split_samples, max_leaf;
  float msl, lr;
};

template <int kPar>
__device__ __forceinline__ const int* ex_src_ord(const ExArgs& a, int d, int j) {
  if (d == 0 && !a.sampled) return a.ord0 + (size_t)a.fidx[j] * a.ld0;
  return a.ordw[kPar] + (size_t)j * a.ldw;
}
template <int kPar>
__device__ __forceinline__ const float* ex_src_val(const ExArgs& a, int d, int j) {
  if (d == 0 && !a.sampled) return a.val0 + (size_t)a.fidx[j] * a.ld0;
  return a.valw[kPar] + (size_t)j * a.ldw;
}
template <int kPar>
__device__ __forceinline__ const float2* ex_src_q(const ExArgs& a, int d, int j) {
  return a.qvw[kPar] + (size_t)j * a.ldw;
}

// the exact int64 fixed point of a float: (long long) rint(y), as torch.round(y).to(int64)
// in exact.py (the tensor engine's q; |y| < 2^63)
__device__ __forceinline__ long long ex_fx(float y) {
  const float r = __builtin_rintf(y);
  const float m = fabsf(r);
  const float hi = floorf(m * 0x1p-32f);
  const float lo = __builtin_fmaf(hi, -0x1p32f, m);
  const unsigned long long u = ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
  const unsigned long long neg = r < 0.f ? ~0ull : 0ull;
  return (long long)((u ^ neg) - neg);
}
__device__ __forceinline__ longlong2 ex_q(const ExArgs& a, float2 x) {
  return make_longlong2(ex_fx(x.x * a.sg), ex_fx(x.y * a.sh));
}

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// order-preserving unsigned image of a float (bits as exact.py's key: -0 below +0)
__device__ __forceinline__ unsigned f2ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// look-back status word: (value << 2) | flag, flag 1 = tile aggregate, 2 = inclusive prefix
__device__ __forceinline__ unsigned long long lb_word(long long v, int flag) {
  return ((unsigned long long)v << 2) | (unsigned long long)flag;
}
__device__ __forceinline__ long long lb_value(unsigned long long w) { return (long long)w >> 2; }

// Exclusive prefix of tile t inside its node (tiles ft..t-1) for C components, by one wave:
// the 64 lanes read a window of 64 predecessors at once (each lane spins until its tile has
// published), the window's nearest inclusive prefix ends the walk, else the window's
// aggregates are added and the next 64 are read. Tiles with lower tickets always publish
// first, and the node's first tile publishes its inclusive prefix directly. Result in every lane.
template <int C>
__device__ __forceinline__ void lb_walk(const unsigned long long* st, int t, int ft, long long* excl) {
  const int l = lane_id();
#pragma unroll
  for (int c = 0; c < C; ++c) {
    long long acc = 0;
    for (int hi = t - 1; hi >= ft; hi -= kWave) {
      const int p = hi - l;
      unsigned long long w = 0;
      if (p >= ft)
        while (((w = ld_agent(st + (size_t)p * C + c)) & 3ull) == 0ull) __builtin_amdgcn_s_sleep(1);
      const unsigned long long pm = __ballot(p >= ft && (w & 3ull) == 2ull);
      const int stop = pm ? __builtin_ctzll(pm) : kWave;  // nearest predecessor with a prefix
      const long long v = (p >= ft && l <= stop) ? lb_value(w) : 0;
      acc += readlane64(dpp_scan_add(v), kWave - 1);
      if (pm) break;
    }
    excl[c] = acc;
  }
}

// sum of (a, b, c) over the 256-thread block, to every thread
__device__ __forceinline__ void ex_block_sum3(long long& a, long long& b, long long& c) {
  __shared__ long long s[3][kExThreads / kWave];
  const long long wa = readlane64(dpp_scan_add(a), kWave - 1), wb = readlane64(dpp_scan_add(b), kWave - 1);
  const long long wc = readlane64(dpp_scan_add(c), kWave - 1);
  const int w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    s[0][w] = wa;
    s[1][w] = wb;
    s[2][w] = wc;
  }
  __syncthreads();
  a = b = c = 0;
#pragma unroll
  for (int k = 0; k < kExThreads / kWave; ++k) {
    a += s[0][k];
    b += s[1][k];
    c += s[2][k];
  }
  __syncthreads();
}

// exclusive prefix of (a, b) over the block's threads in thread order (in place) + totals
__device__ __forceinline__ void ex_block_excl2(long long& a, long long& b, long long& ta, long long& tb) {
  __shared__ long long s[2][kExThreads / kWave];
  const long long ia = dpp_scan_add(a), ib = dpp_scan_add(b);
  const int w = threadIdx.x / kWave;
  if (lane_id() == kWave - 1) {
    s[0][w] = ia;
    s[1][w] = ib;
  }
  __syncthreads();
  long long oa = 0, ob = 0;
  ta = tb = 0;
#pragma unroll
  for (int k = 0; k < kExThreads / kWave; ++k) {
    if (k < w) {
      oa += s[0][k];
      ob += s[1][k];
    }
    ta += s[0][k];
    tb += s[1][k];
  }
  a = oa + ia - a;
  b = ob + ib - b;
  __syncthreads();
}

__global__ __launch_bounds__(kExBig) void ex_init_kernel(ExArgs a, int n) {
  const int nt = n > 0 ? (n + kExTile - 1) / kExTile : 0;
  for (int t = threadIdx.x; t < nt && t < a.max_tiles; t += kExBig)
    a.tiles[0][t] = make_int4(0, t * kExTile, min(n, (t + 1) * kExTile), 0);
  for (int w = EX_TICKET + threadIdx.x; w < EX_CTL_WORDS; w += kExBig) a.ctl[w] = 0;
  if (threadIdx.x < 2) a.ntot[threadIdx.x] = 0;
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

// level 0: qv[j][i] = gh[ord[j][i]] (the only gather of (g, h) in a tree) and the root's totals
__global__ __launch_bounds__(kExThreads) void ex_gather_kernel(ExArgs a, int n) {
  const int j = blockIdx.y;
  const int* ord = ex_src_ord<0>(a, 0, j);
  float2* qo = a.qvw[0] + (size_t)j * a.ldw;
  long long sg = 0, sh = 0, dummy = 0;
  for (long long i = blockIdx.x * (long long)kExThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kExThreads) {
    const float2 x = a.gh[ord[i]];
    qo[i] = x;
    if (j == 0) {
      const longlong2 v = ex_q(a, x);
      sg += v.x;
      sh += v.y;
    }
  }
  if (j != 0) return;
  ex_block_sum3(sg, sh, dummy);
  if (threadIdx.x == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ntot), (unsigned long long)sg);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ntot + 1), (unsigned long long)sh);
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

// the block's (feature slot, tile) from the level's ticket counter (lower tickets start first)
__device__ __forceinline__ bool ex_ticket(const ExArgs& a, int word, int nt, int& j, int& t) {
  __shared__ int s_idx;
  if (threadIdx.x == 0) s_idx = atomicAdd(a.ctl + word, 1);
  __syncthreads();
  const int idx = s_idx;
  __syncthreads();
  if (idx >= nt * a.nf) return false;
  j = idx % a.nf;
  t = idx / a.nf;
  return true;
}

template <int kPar>
__global__ __launch_bounds__(kExThreads) void ex_eval_kernel(ExArgs a, int d) {
  constexpr int par = kPar;
  const int nt = a.ctl[EX_NT0 + par];
  int j, t;
  if (!ex_ticket(a, EX_TICKET + 2 * d, nt, j, t)) return;
  const int4 tl = a.tiles[par][t];
  const int k = tl.x;
  const int nb0 = a.nbeg[par][k], nb1 = a.nbeg[par][k + 1];
  const long long NG = a.ntot[2 * k], NH = a.ntot[2 * k + 1];
  const GainParams& gp = a.gp;
  const double G = (double)NG * gp.inv_sg, H = (double)NH * gp.inv_sh;
  // canSplit (UpdateStrategy.java:50-53): the same for every tile of the node, so a node
  // that cannot split publishes nothing and nobody waits on it
  if (!(H >= 2.0 * (double)gp.mcw && (nb1 - nb0) >= max(a.min_split_samples, 0))) return;
  const float root_gain = (float)calc_gain(G, H, gp);
  const float* val = ex_src_val<par>(a, d, j);
  const float2* qv = ex_src_q<par>(a, d, j);
  const ExSpan sp = ex_span(tl);
  long long g[kExPer], h[kExPer];
  float v[kExPer];
  long long tg = 0, th = 0;
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    g[e] = h[e] = 0;
    v[e] = 0.f;
    if (e < sp.n) {
      const longlong2 x = ex_q(a, qv[sp.i0 + e]);
      g[e] = x.x;
      h[e] = x.y;
      v[e] = val[sp.i0 + e];
    }
    tg += g[e];
    th += h[e];
  }
  __shared__ float s_last[kExThreads];
  __shared__ long long s_pre[2];
  s_last[threadIdx.x] = sp.n > 0 ? v[sp.n - 1] : 0.f;
  long long lg = tg, lh = th, ag, ah;
  ex_block_excl2(lg, lh, ag, ah);  // (+ barrier: s_last visible)
  unsigned long long* st = a.st_gh + (size_t)j * a.max_tiles * 2;
  const int ft = a.ftile[par][k];
  if (threadIdx.x < kWave) {  // wave 0: publish, look back, publish the inclusive prefix
    long long ex[2] = {0, 0};
    if (t == ft) {
      if (threadIdx.x == 0) {
        st_agent(st + 2 * t, lb_word(ag, 2));
        st_agent(st + 2 * t + 1, lb_word(ah, 2));
      }
    } else {
      if (threadIdx.x == 0) {
        st_agent(st + 2 * t, lb_word(ag, 1));
        st_agent(st + 2 * t + 1, lb_word(ah, 1));
      }
      lb_walk<2>(st, t, ft, ex);
      if (threadIdx.x == 0) {
        st_agent(st + 2 * t, lb_word(ex[0] + ag, 2));
        st_agent(st + 2 * t + 1, lb_word(ex[1] + ah, 2));
      }
    }
    if (threadIdx.x == 0) {
      s_pre[0] = ex[0];
      s_pre[1] = ex[1];
    }
  }
  __syncthreads();
  lg += s_pre[0];
  lh += s_pre[1];
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

template <int kPar>
__global__ __launch_bounds__(kExBig) void ex_decide_kernel(ExArgs a, int d, int final_level) {
  constexpr int par = kPar;
  const int tid = threadIdx.x;
  const int K = a.ctl[EX_K0 + par];
  const int leaf0 = a.ctl[EX_LEAF];
  const bool budget = !final_level && (a.max_leaf <= 0 || leaf0 < a.max_leaf);
  const int room = a.max_leaf > 0 ? a.max_leaf - leaf0 : 0x7fffffff;
  ExRec* rec = a.rec + a.rec_off[d];
  const GainParams& gp = a.gp;
  constexpr int kW = kExBig / kWave;
  __shared__ int s_w[kW];
  const int w = tid / kWave, l = lane_id();
  int carry = 0;
  for (int base = 0; base < K; base += kExBig) {
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
        const float* vv = ex_src_val<par>(a, d, bj);
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

// slot 0: go-left flags by row + per-tile partials of the children (exact int64)
template <int kPar>
__global__ __launch_bounds__(kExThreads) void ex_flag_kernel(ExArgs a, int d) {
  constexpr int par = kPar;
  const int t = blockIdx.x;
  if (t >= a.ctl[EX_NT0 + par]) return;
  const int4 tl = a.tiles[par][t];
  const int f = a.go_feat[tl.x];
  const float thr = a.go_thr[tl.x];
  const int* ord = ex_src_ord<par>(a, d, 0);
  const float2* qv = ex_src_q<par>(a, d, 0);
  long long nl = 0, lg = 0, lh = 0, rg = 0, rh = 0;
  for (int i = tl.y + threadIdx.x; i < tl.z; i += kExThreads) {
    const int r = ord[i];
    if (f < 0) {
      a.left_row[r] = 2;
      continue;
    }
    const longlong2 x = ex_q(a, qv[i]);
    const bool left = a.XT[(size_t)f * a.ldx + r] < thr;
    a.left_row[r] = left ? 1 : 0;
    if (left) {
      ++nl;
      lg += x.x;
      lh += x.y;
    } else {
      rg += x.x;
      rh += x.y;
    }
  }
  long long z = 0;
  ex_block_sum3(nl, lg, lh);
  ex_block_sum3(rg, rh, z);
  if (threadIdx.x == 0) {
    long long* o = a.tpart + (size_t)t * 5;
    o[0] = nl;
    o[1] = lg;
    o[2] = lh;
    o[3] = rg;
    o[4] = rh;
  }
}

// left_bits[w] = bit b set iff left_row[32 w + b] == 1 (coalesced: 32 bytes in, one word out)
__global__ __launch_bounds__(256) void ex_bits_kernel(ExArgs a, int n) {
  const int nw = (n + 31) >> 5;
  for (int w = blockIdx.x * 256 + threadIdx.x; w < nw; w += gridDim.x * 256) {
    unsigned bits = 0;
    const int base = w << 5;
    if (base + 32 <= n) {
      const uint4* p = reinterpret_cast<const uint4*>(a.left_row + base);  // 16-B aligned
      const uint4 x0 = p[0], x1 = p[1];
      const unsigned wd[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int c = 0; c < 4; ++c) bits |= (((wd[k] >> (8 * c)) & 0xffu) == 1u ? 1u : 0u) << (4 * k + c);
      }
    } else {
      for (int b = 0; base + b < n; ++b) bits |= (a.left_row[base + b] == 1 ? 1u : 0u) << b;
    }
    a.left_bits[w] = bits;
  }
}

// One block: node sums of the flag partials (global exclusive tile prefixes recorded at each
// node's first tile), the children's exact (g, h) totals (the next level's ntot), segments,
// first tiles and tile table.
template <int kPar>
__global__ __launch_bounds__(kExBig) void ex_layout_kernel(ExArgs a, int d) {
  constexpr int par = kPar, npar = par ^ 1;
  const int tid = threadIdx.x;
  const int nt = a.ctl[EX_NT0 + par], K = a.ctl[EX_K0 + par], Kn = a.ctl[EX_K0 + npar];
  const int4* tiles = a.tiles[par];
  const int* ftile = a.ftile[par];
  const int* nbg = a.nbeg[par];
  constexpr int kW = kExBig / kWave;
  __shared__ long long s1[kW];
  __shared__ int si[2][kW];
  const int w = tid / kWave, l = lane_id();
  // one component per pass over the tiles (not all five at once: five int64 scans in flight
  // spilled 79 VGPRs to scratch at 1024 threads)
#pragma unroll 1
  for (int c = 0; c < 5; ++c) {
    long long carry = 0;
    for (int base = 0; base < nt; base += kExBig) {
      const int t = base + tid;
      long long x = 0;
      int node = 0;
      if (t < nt) {
        node = tiles[t].x;
        if (a.go_feat[node] >= 0) x = a.tpart[(size_t)t * 5 + c];
      }
      const long long inc = dpp_scan_add(x);
      if (l == kWave - 1) s1[w] = inc;
      __syncthreads();
      long long o = carry, T = 0;
      for (int q = 0; q < kW; ++q) {
        if (q < w) o += s1[q];
        T += s1[q];
      }
      if (t < nt && ftile[node] == t) a.nbase[(size_t)node * 5 + c] = o + inc - x;
      carry += T;
      __syncthreads();
    }
    if (tid == 0) a.nbase[(size_t)K * 5 + c] = carry;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  auto nsum = [&](int k, int c) -> long long {
    return ld_agent(a.nbase + (size_t)(k + 1) * 5 + c) - ld_agent(a.nbase + (size_t)k * 5 + c);
  };
  // children: split node k (child index c = csplit[k]) keeps its rows, left child first
  int rcarry = 0, tcarry = 0;
  for (int base = 0; base < K; base += kExBig) {
    const int k = base + tid;
    int rows = 0, ntl = 0, left = 0, c = -1;
    if (k < K) {
      c = a.csplit[k];
      if (c >= 0) {
        rows = nbg[k + 1] - nbg[k];
        left = (int)nsum(k, 0);
        ntl = (left + kExTile - 1) / kExTile + (rows - left + kExTile - 1) / kExTile;
      }
    }
    int ir = rows, it = ntl;
    for (int off = 1; off < kWave; off <<= 1) {
      const int vr = __shfl_up(ir, off, kWave), vt = __shfl_up(it, off, kWave);
      if (l >= off) {
        ir += vr;
        it += vt;
      }
    }
    if (l == kWave - 1) {
      si[0][w] = ir;
      si[1][w] = it;
    }
    __syncthreads();
    int orr = rcarry, ot = tcarry, Tr = 0, Tt = 0;
    for (int q = 0; q < kW; ++q) {
      if (q < w) {
        orr += si[0][q];
        ot += si[1][q];
      }
      Tr += si[0][q];
      Tt += si[1][q];
    }
    if (c >= 0) {
      const int S = orr + ir - rows, ft = ot + it - ntl;
      a.cbeg[2 * k] = S;
      a.cbeg[2 * k + 1] = S + left;
      a.nbeg[npar][c] = S;
      a.nbeg[npar][c + 1] = S + left;
      a.ftile[npar][c] = ft;
      a.ftile[npar][c + 1] = ft + (left + kExTile - 1) / kExTile;
      a.ntot[2 * c] = nsum(k, 1);
      a.ntot[2 * c + 1] = nsum(k, 2);
      a.ntot[2 * c + 2] = nsum(k, 3);
      a.ntot[2 * c + 3] = nsum(k, 4);
    }
    rcarry += Tr;
    tcarry += Tt;
    __syncthreads();
  }
  if (tid == 0) {
    a.nbeg[npar][Kn] = rcarry;
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
  for (int t = tid; t < ntn; t += kExBig) {
    int lo = 0, hi = Kn - 1;  // last child with ftile <= t (children are non-empty: >= 1 tile)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (ld_agent(ftn + mid) <= t) lo = mid;
      else hi = mid - 1;
    }
    const int f0 = ld_agent(ftn + lo), b0 = ld_agent(nbn + lo), b1 = ld_agent(nbn + lo + 1);
    const int p0 = b0 + (t - f0) * kExTile;
    a.tiles[npar][t] = make_int4(lo, p0, min(b1, p0 + kExTile), 0);
  }
}

template <int kPar>
__global__ __launch_bounds__(kExThreads) void ex_part_kernel(ExArgs a, int d) {
  constexpr int par = kPar;
  const int nt = a.ctl[EX_NT0 + par];
  int j, t;
  if (!ex_ticket(a, EX_TICKET + 2 * d + 1, nt, j, t)) return;
  const int4 tl = a.tiles[par][t];
  const int k = tl.x;
  if (a.csplit[k] < 0) return;  // a leaf: its rows leave the order (block-uniform, nobody waits)
  const int* ord = ex_src_ord<par>(a, d, j);
  const float* val = ex_src_val<par>(a, d, j);
  const float2* qv = ex_src_q<par>(a, d, j);
  constexpr int no = par ^ 1;
  int* ordo = a.ordw[no] + (size_t)j * a.ldw;
  float* valo = a.valw[no] + (size_t)j * a.ldw;
  float2* qo = a.qvw[no] + (size_t)j * a.ldw;
  // lane-consecutive elements (element i = e * kExThreads + tid: every load instruction reads
  // 64 consecutive positions) ranked with wave ballots: lefts before element i = the lefts of
  // the rows e' < e of the tile, of the waves before this one in row e, and of the lanes
  // below in this wave (the thread-contiguous layout's loads were 128-B strided per lane)
  const int i0 = tl.y, n = tl.z - tl.y;
  const int tid = threadIdx.x, w = tid / kWave, l = lane_id();
  constexpr int NW = kExThreads / kWave;
  int r[kExPer];
  float v[kExPer];
  float2 q[kExPer];
  unsigned lmask = 0;
  // lanes past the tile's end load its first element again (clamped index, n >= 1: a node's
  // tiles are never empty)
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    const int i = e * kExThreads + tid;
    r[e] = ord[i0 + (i < n ? i : 0)];
  }
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    const int i = e * kExThreads + tid;
    const int ic = i < n ? i : 0;
    v[e] = val[i0 + ic];
    q[e] = qv[i0 + ic];
    // the row's direction from the bitset (1.3 MB for 10.5M rows: L2 resident, unlike the
    // 10.5 MB byte array the random gather read before)
    lmask |= (i < n && ((a.left_bits[(unsigned)r[e] >> 5] >> (r[e] & 31)) & 1u)) ? 1u << e : 0u;
  }
  __shared__ int s_wc[kExPer][NW];
  int lrank[kExPer];
  const unsigned long long lt_mask = l == 0 ? 0ull : (~0ull >> (64 - l));
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    const unsigned long long bm = __ballot((lmask >> e) & 1u);
    lrank[e] = __popcll(bm & lt_mask);
    if (l == 0) s_wc[e][w] = __popcll(bm);
  }
  __syncthreads();
  int off[kExPer];
  int tl_left = 0;
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    int o = tl_left;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      o += ww < w ? s_wc[e][ww] : 0;
      tl_left += s_wc[e][ww];
    }
    off[e] = o;
  }
  __shared__ long long s_lt;
  unsigned long long* st = a.st_cnt + (size_t)j * a.max_tiles;
  const int ft = a.ftile[par][k];
  if (threadIdx.x < kWave) {  // wave 0: publish, look back, publish the inclusive prefix
    long long ex = 0;
    if (t == ft) {
      if (threadIdx.x == 0) st_agent(st + t, lb_word(tl_left, 2));
    } else {
      if (threadIdx.x == 0) st_agent(st + t, lb_word(tl_left, 1));
      lb_walk<1>(st, t, ft, &ex);
      if (threadIdx.x == 0) st_agent(st + t, lb_word(ex + tl_left, 2));
    }
    if (threadIdx.x == 0) s_lt = ex;
  }
  __syncthreads();
  const int lt = (int)s_lt;                    // lefts of the node before this tile
  const int before = tl.y - a.nbeg[par][k];    // node positions before this tile
  // stage the tile partitioned in LDS (lefts, then rights, each in order), then store both
  // runs with consecutive lanes on consecutive positions (coalesced)
  __shared__ int s_r[kExTile];
  __shared__ float s_v[kExTile];
  __shared__ float2 s_q[kExTile];
#pragma unroll
  for (int e = 0; e < kExPer; ++e) {
    const int i = e * kExThreads + tid;
    if (i < n) {
      const int lb = off[e] + lrank[e];  // lefts before element i
      const int dst = (lmask >> e) & 1 ? lb : tl_left + (i - lb);
      s_r[dst] = r[e];
      s_v[dst] = v[e];
      s_q[dst] = q[e];
    }
  }
  __syncthreads();
  const int ntile = tl.z - tl.y;
  const int l0 = a.cbeg[2 * k] + lt, r0 = a.cbeg[2 * k + 1] + (before - lt) - tl_left;
  for (int i = threadIdx.x; i < ntile; i += kExThreads) {
    const int dst = i < tl_left ? l0 + i : r0 + i;
    ordo[dst] = s_r[i];
    valo[dst] = s_v[i];
    qo[dst] = s_q[i];
  }
}

// one level's launches; the level parity picks the ping-pong buffers at compile time
template <int kPar>
void ex_level(const ExArgs& a, int d, long long blocks, int n, int bits_grid, hipStream_t s) {
  hipLaunchKernelGGL(ex_eval_kernel<kPar>, dim3((unsigned)blocks), dim3(kExThreads), 0, s, a, d);
  hipLaunchKernelGGL(ex_decide_kernel<kPar>, dim3(1), dim3(kExBig), 0, s, a, d, 0);
  hipLaunchKernelGGL(ex_flag_kernel<kPar>, dim3(a.max_tiles), dim3(kExThreads), 0, s, a, d);
  hipLaunchKernelGGL(ex_layout_kernel<kPar>, dim3(1), dim3(kExBig), 0, s, a, d);
  hipLaunchKernelGGL(ex_bits_kernel, dim3(bits_grid), dim3(256), 0, s, a, n);
  hipLaunchKernelGGL(ex_part_kernel<kPar>, dim3((unsigned)blocks), dim3(kExThreads), 0, s, a, d);
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

// ptrs: ord0, val0, ordw0, ordw1, valw0, valw1, qvw0, qvw1, XT, tiles0, tiles1, nbeg0, nbeg1,
//       ftile0, ftile1, ctl, st_gh, st_cnt, tpart, nbase, nkey, ntot, go_feat, go_thr,
//       csplit, cbeg, left_row, rec, rec_off, rec_k
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
  a.qvw[0] = (float2*)p[i++];
  a.qvw[1] = (float2*)p[i++];
  a.XT = (const float*)p[i++];
  a.tiles[0] = (int4*)p[i++];
  a.tiles[1] = (int4*)p[i++];
  a.nbeg[0] = (int*)p[i++];
  a.nbeg[1] = (int*)p[i++];
  a.ftile[0] = (int*)p[i++];
  a.ftile[1] = (int*)p[i++];
  a.ctl = (int*)p[i++];
  a.st_gh = (unsigned long long*)p[i++];
  a.st_cnt = (unsigned long long*)p[i++];
  a.tpart = (long long*)p[i++];
  a.nbase = (long long*)p[i++];
  a.nkey = (unsigned long long*)p[i++];
  a.ntot = (long long*)p[i++];
  a.go_feat = (int*)p[i++];
  a.go_thr = (float*)p[i++];
  a.csplit = (int*)p[i++];
  a.cbeg = (int*)p[i++];
  a.left_row = (unsigned char*)p[i++];  // [align16(ldw) + 4 * ceil(ldw / 32)] bytes: bytes, then bits
  a.rec = (ExRec*)p[i++];
  a.rec_off = (const long long*)p[i++];
  a.rec_k = (int*)p[i++];
  a.ld0 = ip[0];
  a.ldw = ip[1];
  a.ldx = ip[2];
  a.left_bits = reinterpret_cast<unsigned*>(a.left_row + ((a.ldw + 15) & ~15LL));
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
// nodes (leaves). gh: [N] float (g, h) by row; the int64 fixed point is rint(g * sg),
// rint(h * sh) with power-of-two scales leaving |sums| < 2^60 (inv_g = 1 / sg, inv_h = 1 / sh);
// fidx: the nf searched feature slots (ascending); n: rows in the tree (sampled: ordw[0] /
// valw[0] hold each slot's kept rows in value order).
void ytk_ex_tree(int h, uintptr_t gh, uintptr_t fidx, int nf, int n, int sampled, double inv_g, double inv_h,
                 int depth, float lr, uintptr_t stream) {
  ExEngine& e = g_ex.at(h);
  ExArgs a = e.a;
  a.gh = (const float2*)gh;
  a.sg = (float)(1.0 / inv_g);
  a.sh = (float)(1.0 / inv_h);
  a.fidx = (const int*)fidx;
  a.nf = nf;
  a.sampled = sampled;
  a.gp.inv_sg = inv_g;
  a.gp.inv_sh = inv_h;
  a.lr = lr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (nf < 1 || nf > 65535) throw std::invalid_argument("ex_tree: bad feature count");
  if (depth < 0 || EX_TICKET + 2 * depth + 2 > EX_CTL_WORDS) throw std::invalid_argument("ex_tree: depth too large");
  const long long blocks = (long long)a.max_tiles * nf;
  if (blocks > 0x7fffffffLL) throw std::invalid_argument("ex_tree: too many (tile, feature) blocks");
  const size_t st_gh_bytes = (size_t)nf * a.max_tiles * 2 * 8, st_cnt_bytes = (size_t)nf * a.max_tiles * 8;
  hipLaunchKernelGGL(ex_init_kernel, dim3(1), dim3(kExBig), 0, s, a, n);
  // the bitset covers every row id (a sampled tree's n counts its kept rows, not the id range)
  const int nrow = (int)a.ldw;
  const int bits_grid = std::max(1, std::min(((nrow + 31) / 32 + 255) / 256, 2048));
  const int gx = std::max(1, std::min((n + kExThreads - 1) / kExThreads, 1024));
  hipLaunchKernelGGL(ex_gather_kernel, dim3(gx, nf), dim3(kExThreads), 0, s, a, n);
  for (int d = 0; d <= depth; ++d) {
    if (d == depth) {
      if (d & 1)
        hipLaunchKernelGGL(ex_decide_kernel<1>, dim3(1), dim3(kExBig), 0, s, a, d, 1);
      else
        hipLaunchKernelGGL(ex_decide_kernel<0>, dim3(1), dim3(kExBig), 0, s, a, d, 1);
      break;
    }
    YTK_HIP_CHECK(hipMemsetAsync(a.st_gh, 0, st_gh_bytes, s));
    YTK_HIP_CHECK(hipMemsetAsync(a.st_cnt, 0, st_cnt_bytes, s));
    if (d & 1)
      ex_level<1>(a, d, blocks, nrow, bits_grid, s);
    else
      ex_level<0>(a, d, blocks, nrow, bits_grid, s);
  }
  YTK_LAUNCH_CHECK();
}

int ytk_ex_tile() { return kExTile; }

}  // extern "C"
