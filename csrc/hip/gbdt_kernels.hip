// GBDT hot-path kernels for MI355X (gfx950, CDNA4, wave64).
//
// Reference semantics (what, not how):
//   histogram build      J/data/gbdt/HistogramBuilder.java:56-90
//   split enumeration    J/optimizer/gbdt/DataParallelTreeMaker.java:598-637
//   gain / leaf value    J/optimizer/gbdt/UpdateStrategy.java:50-100
//   split tie-break      J/data/gbdt/SplitInfo.java:99-104
//   row partition        J/data/gbdt/SamplePositionData.java:115-165
//   bin assignment       J/data/gbdt/FeatureApprData.java:179-205
//   tree scoring         J/data/gbdt/Tree.java:136-168
//   grad / hess          J/optimizer/GBDTOptimizer.java:513-609 + J/loss/*
//
// Design (MI355X-first, not a translation):
//  * Histograms are accumulated in LDS with a FEATURE-MINOR layout lds[bin][32]:
//    the 32 lanes of a half-wave own the 32 features of one row, so the bank of
//    every ds_add_f32 is the feature lane -> a wave-instruction updates 2 rows x 32
//    features with zero bank conflicts regardless of the (random) bin values.
//    g and h live in two 32 KiB planes (64 KiB / block -> 2 blocks per CU).
//  * Rows of a tree node are a contiguous segment of a row-index permutation;
//    one launch builds the histograms of every node of a level (work list of
//    (slot, begin, end) chunks), so launch count per level is O(1).
//  * Split finding: one workgroup per node, one wave per feature, 4 bins per lane,
//    fp64 wave prefix scans, deterministic (lossChg, feature, bin) argmax.
//    Sibling subtraction (parent - small child) is fused into the load.
//  * Partition: per-node stable two-pass (count, ballot-scatter) over chunks.
#include "common.h"

namespace ytk {

// ---------------------------------------------------------------------------
// Histogram build, uint8 bins, LDS privatized, feature-minor (conflict free).
// work[blk] = {slot, begin, end, 0}; grid = (num_work, num_feature_groups).
// hist layout: float2 [slot][B][F]  (g, h) interleaved.
// ---------------------------------------------------------------------------
template <bool kIdentity>
__global__ __launch_bounds__(256, 2) void hist_u8_lds_kernel(
    const uint8_t* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ gh, const int* __restrict__ rows,
    const int4* __restrict__ work, float2* __restrict__ hist, int B, int nb_lds) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lg = smem;
  float* lh = smem + nb_lds * 32;
  const int4 w = work[blockIdx.x];
  const int fg = blockIdx.y;
  const int tid = threadIdx.x;
  for (int i = tid; i < nb_lds * 64; i += 256) smem[i] = 0.f;
  __syncthreads();

  const int hw = tid >> 5;  // half-wave 0..7 -> row offset
  const int fl = tid & 31;  // feature lane
  const int f = fg * 32 + fl;
  const bool active = f < F;
  const uint8_t* bcol = bins + fg * 32 + fl;
  const int end = w.z;
  int pos = w.y + hw;
  // 4 rows in flight per half-wave (32 rows per block step).
  for (; pos + 24 < end; pos += 32) {
    int r0, r1, r2, r3;
    if (kIdentity) {
      r0 = pos; r1 = pos + 8; r2 = pos + 16; r3 = pos + 24;
    } else {
      r0 = rows[pos]; r1 = rows[pos + 8]; r2 = rows[pos + 16]; r3 = rows[pos + 24];
    }
    const int b0 = bcol[(long long)r0 * stride];
    const int b1 = bcol[(long long)r1 * stride];
    const int b2 = bcol[(long long)r2 * stride];
    const int b3 = bcol[(long long)r3 * stride];
    const float2 v0 = gh[r0], v1 = gh[r1], v2 = gh[r2], v3 = gh[r3];
    if (active) {
      atomicAdd(&lg[b0 * 32 + fl], v0.x); atomicAdd(&lh[b0 * 32 + fl], v0.y);
      atomicAdd(&lg[b1 * 32 + fl], v1.x); atomicAdd(&lh[b1 * 32 + fl], v1.y);
      atomicAdd(&lg[b2 * 32 + fl], v2.x); atomicAdd(&lh[b2 * 32 + fl], v2.y);
      atomicAdd(&lg[b3 * 32 + fl], v3.x); atomicAdd(&lh[b3 * 32 + fl], v3.y);
    }
  }
  for (; pos < end; pos += 8) {
    const int r = kIdentity ? pos : rows[pos];
    const int b = bcol[(long long)r * stride];
    const float2 v = gh[r];
    if (active) { atomicAdd(&lg[b * 32 + fl], v.x); atomicAdd(&lh[b * 32 + fl], v.y); }
  }
  __syncthreads();

  float2* out = hist + (size_t)w.x * B * F;
  for (int i = tid; i < nb_lds * 32; i += 256) {
    const int bin = i >> 5, l = i & 31, ff = fg * 32 + l;
    if (ff < F) {
      const float g = lg[i], h = lh[i];
      if (g != 0.f || h != 0.f) {
        float* o = reinterpret_cast<float*>(&out[(size_t)bin * F + ff]);
        atomicAdd(o, g);
        atomicAdd(o + 1, h);
      }
    }
  }
}

// Generic histogram (uint8 or uint16 bins, any bin count): direct global atomics.
// Used for > 256 bins (e.g. the 5000-bin stress config). One thread per
// (row, feature) element of the work chunk.
template <typename BinT>
__global__ __launch_bounds__(256) void hist_global_kernel(
    const BinT* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ gh, const int* __restrict__ rows,
    const int4* __restrict__ work, float2* __restrict__ hist, int B) {
  const int4 w = work[blockIdx.x];
  const long long n = (long long)(w.z - w.y) * F;
  float2* out = hist + (size_t)w.x * B * F;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const int pos = w.y + (int)(i / F);
    const int f = (int)(i % F);
    const int r = rows ? rows[pos] : pos;
    const int b = bins[(long long)r * stride + f];
    const float2 v = gh[r];
    float* o = reinterpret_cast<float*>(&out[(size_t)b * F + f]);
    atomicAdd(o, v.x);
    atomicAdd(o + 1, v.y);
  }
}

// ---------------------------------------------------------------------------
// Split finder.
// items[blk] = {slot, parent_slot, sibling_slot, derived}
// ---------------------------------------------------------------------------
struct SplitOut {
  float loss_chg;
  int feat;
  int bin_a;  // last non-empty bin going left
  int bin_b;  // first non-empty bin going right
  double gl, hl;  // left sums
  double g, h;    // node sums
};
static_assert(sizeof(SplitOut) == 48, "SplitOut layout");

struct GainParams {
  float mcw;       // min_child_hessian_sum
  float l1, l2;
  float max_abs_leaf;
};

__device__ __forceinline__ double thr_l1(double w, double lam) {
  if (w > lam) return w - lam;
  if (w < -lam) return w + lam;
  return 0.0;
}

__device__ __forceinline__ double node_value(double g, double h, const GainParams& p) {
  if (h < (double)p.mcw) return 0.0;
  double v = (p.l1 == 0.f) ? -g / (h + p.l2) : -thr_l1(g, p.l1) / (h + p.l2);
  if (p.max_abs_leaf > 0.f) {
    if (v > p.max_abs_leaf) v = p.max_abs_leaf;
    else if (v < -p.max_abs_leaf) v = -p.max_abs_leaf;
  }
  return v;
}

__device__ __forceinline__ double calc_gain(double g, double h, const GainParams& p) {
  if (h < (double)p.mcw) return 0.0;
  if (p.max_abs_leaf <= 0.f) {
    if (p.l1 == 0.f) return g * g / (h + p.l2);
    const double t = thr_l1(g, p.l1);
    return t * t / (h + p.l2);
  }
  const double v = node_value(g, h, p);
  return -2.0 * (g * v + 0.5 * (h + p.l2) * v * v + p.l1 * fabs(v));
}

// (chg, feat, bin) lexicographic "better": larger chg, then lower feat, then lower bin.
__device__ __forceinline__ bool better(float c1, int f1, int b1, float c2, int f2, int b2) {
  if (c1 != c2) return c1 > c2;
  if (f1 != f2) return f1 < f2;
  return b1 < b2;
}

__global__ __launch_bounds__(256) void split_find_kernel(
    float2* __restrict__ hist, int B, int F, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp) {
  __shared__ float s_chg[4];
  __shared__ int s_feat[4], s_a[4], s_b[4];
  __shared__ double s_gl[4], s_hl[4];

  const int4 it = items[blockIdx.x];
  const int wid = threadIdx.x >> 6;
  const int l = lane_id();
  float2* hn = hist + (size_t)it.x * B * F;
  const float2* hp = hist + (size_t)it.y * B * F;
  const float2* hs = hist + (size_t)it.z * B * F;
  const bool derived = it.w != 0;

  auto load = [&](int f, int bin) -> float2 {
    const size_t idx = (size_t)bin * F + f;
    if (derived) {
      const float2 p = hp[idx], s = hs[idx];
      return make_float2(p.x - s.x, p.y - s.y);
    }
    return hn[idx];
  };

  // Node totals from the first sampled feature (reference semantics:
  // DataParallelTreeMaker.updateTreeMakerNodeStats). Every wave computes it
  // identically -> no cross-wave hand-off needed.
  double G = 0.0, H = 0.0;
  {
    const int nb0 = nbins_f[f0];
    double sg = 0.0, sh = 0.0;
    for (int bin = l; bin < nb0; bin += kWave) {
      const float2 v = load(f0, bin);
      sg += v.x; sh += v.y;
    }
    G = wave_sum(sg);
    H = wave_sum(sh);
  }
  const float root_gain = (float)calc_gain(G, H, gp);

  float best_chg = -INFINITY;
  int best_f = 0x7fffffff, best_a = -1, best_b = 0x7fffffff;
  double best_gl = 0.0, best_hl = 0.0;

  for (int f = wid; f < F; f += 4) {
    if (!fmask[f]) continue;
    const int nb = nbins_f[f];
    double carry_g = 0.0, carry_h = 0.0;
    int carry_last = -1;
    for (int c = 0; c < B; c += 4 * kWave) {
      float2 v[4];
      double sg = 0.0, sh = 0.0;
      int lastne = -1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bin = c + 4 * l + k;
        v[k] = make_float2(0.f, 0.f);
        if (bin < nb) v[k] = load(f, bin);
        if (derived && bin < B) hn[(size_t)bin * F + f] = v[k];
        sg += v[k].x;
        sh += v[k].y;
        if (v[k].x != 0.f || v[k].y != 0.f) lastne = bin;
      }
      const double ig = wave_incl_scan(sg);
      const double ih = wave_incl_scan(sh);
      const int im = wave_incl_max(lastne);
      int em = __shfl_up(im, 1, kWave);
      if (l == 0) em = -1;
      double pg = ig - sg + carry_g;
      double ph = ih - sh + carry_h;
      int prev = max(em, carry_last);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bin = c + 4 * l + k;
        const bool ne = (v[k].x != 0.f || v[k].y != 0.f);
        if (ne) {
          if (prev >= 0 && ph != 0.0 && ph >= (double)gp.mcw) {
            const double rg = G - pg, rh = H - ph;
            if (rh >= (double)gp.mcw) {
              const float chg = (float)(calc_gain(pg, ph, gp) + calc_gain(rg, rh, gp) - (double)root_gain);
              if (better(chg, f, bin, best_chg, best_f, best_b)) {
                best_chg = chg; best_f = f; best_a = prev; best_b = bin;
                best_gl = pg; best_hl = ph;
              }
            }
          }
          pg += v[k].x;
          ph += v[k].y;
          prev = bin;
        }
      }
      carry_g += __shfl(ig, kWave - 1, kWave);
      carry_h += __shfl(ih, kWave - 1, kWave);
      carry_last = max(carry_last, __shfl(im, kWave - 1, kWave));
    }
  }
  // wave argmax
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const float oc = __shfl_xor(best_chg, off, kWave);
    const int of = __shfl_xor(best_f, off, kWave);
    const int oa = __shfl_xor(best_a, off, kWave);
    const int ob = __shfl_xor(best_b, off, kWave);
    const double ogl = __shfl_xor(best_gl, off, kWave);
    const double ohl = __shfl_xor(best_hl, off, kWave);
    if (better(oc, of, ob, best_chg, best_f, best_b)) {
      best_chg = oc; best_f = of; best_a = oa; best_b = ob; best_gl = ogl; best_hl = ohl;
    }
  }
  if (l == 0) {
    s_chg[wid] = best_chg; s_feat[wid] = best_f; s_a[wid] = best_a; s_b[wid] = best_b;
    s_gl[wid] = best_gl; s_hl[wid] = best_hl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bw = 0;
    for (int w2 = 1; w2 < 4; ++w2)
      if (better(s_chg[w2], s_feat[w2], s_b[w2], s_chg[bw], s_feat[bw], s_b[bw])) bw = w2;
    SplitOut o;
    o.loss_chg = s_chg[bw];
    o.feat = (s_feat[bw] == 0x7fffffff) ? -1 : s_feat[bw];
    o.bin_a = s_a[bw];
    o.bin_b = (s_b[bw] == 0x7fffffff) ? -1 : s_b[bw];
    o.gl = s_gl[bw]; o.hl = s_hl[bw];
    o.g = G; o.h = H;
    out[blockIdx.x] = o;
  }
}

// ---------------------------------------------------------------------------
// Stable partition of node segments. items[blk] = {split_idx, begin, end, blk_in_node}
// per split i: feat[i], thr[i] (go left iff bin <= thr), node_begin[i], first_blk[i], nblk[i]
// ---------------------------------------------------------------------------
template <typename BinT>
__global__ __launch_bounds__(256) void partition_count_kernel(
    const BinT* __restrict__ bins, long long stride, const int* __restrict__ rows,
    const int4* __restrict__ items, const int* __restrict__ feat, const int* __restrict__ thr,
    int* __restrict__ counts) {
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int4 it = items[blockIdx.x];
  const int f = feat[it.x], t = thr[it.x];
  int c = 0;
  for (int pos = it.y + threadIdx.x; pos < it.z; pos += 256) {
    const int r = rows[pos];
    c += (int)bins[(long long)r * stride + f] <= t;
  }
  c = wave_sumi(c);
  if (lane_id() == 0) atomicAdd(&s_cnt, c);
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = s_cnt;
}

template <typename BinT>
__global__ __launch_bounds__(256) void partition_scatter_kernel(
    const BinT* __restrict__ bins, long long stride, const int* __restrict__ rows,
    int* __restrict__ rows_out, const int4* __restrict__ items,
    const int* __restrict__ feat, const int* __restrict__ thr,
    const int* __restrict__ node_begin, const int* __restrict__ first_blk,
    const int* __restrict__ nblk, const int* __restrict__ counts,
    int* __restrict__ left_total_out) {
  __shared__ int s_red[8];
  __shared__ int s_wl[4], s_wv[4];
  const int4 it = items[blockIdx.x];
  const int si = it.x;
  const int f = feat[si], t = thr[si];
  const int nbeg = node_begin[si], fb = first_blk[si], nb = nblk[si];
  const int tid = threadIdx.x, wid = tid >> 6, l = lane_id();

  // left rows before this block, and total left rows of the node
  int before = 0, total = 0;
  for (int j = tid; j < nb; j += 256) {
    const int c = counts[fb + j];
    total += c;
    if (fb + j < (int)blockIdx.x) before += c;
  }
  before = wave_sumi(before);
  total = wave_sumi(total);
  if (l == 0) { s_red[wid] = before; s_red[4 + wid] = total; }
  __syncthreads();
  before = s_red[0] + s_red[1] + s_red[2] + s_red[3];
  total = s_red[4] + s_red[5] + s_red[6] + s_red[7];
  if (it.w == 0 && tid == 0) left_total_out[si] = total;

  int lbase = nbeg + before;
  int rbase = nbeg + total + (it.y - nbeg - before);
  const unsigned long long lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  for (int tile = it.y; tile < it.z; tile += 256) {
    const int pos = tile + tid;
    const bool valid = pos < it.z;
    int r = 0;
    bool left = false;
    if (valid) {
      r = rows[pos];
      left = (int)bins[(long long)r * stride + f] <= t;
    }
    const unsigned long long lm = __ballot(left);
    const unsigned long long vm = __ballot(valid);
    const int lrank = __popcll(lm & lt_mask);
    const int vrank = __popcll(vm & lt_mask);
    __syncthreads();  // previous tile's s_wl reads done
    if (l == 0) { s_wl[wid] = __popcll(lm); s_wv[wid] = __popcll(vm); }
    __syncthreads();
    int wl_pre = 0, wv_pre = 0, tl = 0, tv = 0;
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) {
      if (w2 < wid) { wl_pre += s_wl[w2]; wv_pre += s_wv[w2]; }
      tl += s_wl[w2]; tv += s_wv[w2];
    }
    if (valid) {
      if (left) rows_out[lbase + wl_pre + lrank] = r;
      else rows_out[rbase + (wv_pre - wl_pre) + (vrank - lrank)] = r;
    }
    lbase += tl;
    rbase += tv - tl;
  }
}

// ---------------------------------------------------------------------------
// Training-score update: traverse one tree on binned rows, score += value.
// node arrays: feat (<0 => leaf), thr (go left iff bin <= thr), left, right, value
// ---------------------------------------------------------------------------
template <typename BinT>
__global__ __launch_bounds__(256) void tree_add_bins_kernel(
    const BinT* __restrict__ bins, long long stride, long long N,
    const int* __restrict__ tfeat, const int* __restrict__ tthr,
    const int* __restrict__ tleft, const int* __restrict__ tright,
    const float* __restrict__ tval, int nnodes,
    float* __restrict__ score, int sstride, int soff) {
  extern __shared__ __attribute__((aligned(16))) int tsm[];
  int* sf = tsm;
  int* st = tsm + nnodes;
  int* sl = tsm + 2 * nnodes;
  int* sr = tsm + 3 * nnodes;
  float* sv = reinterpret_cast<float*>(tsm + 4 * nnodes);
  for (int i = threadIdx.x; i < nnodes; i += blockDim.x) {
    sf[i] = tfeat[i]; st[i] = tthr[i]; sl[i] = tleft[i]; sr[i] = tright[i]; sv[i] = tval[i];
  }
  __syncthreads();
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < N;
       r += (long long)gridDim.x * blockDim.x) {
    int n = 0;
    const BinT* row = bins + r * stride;
    while (sf[n] >= 0) n = ((int)row[sf[n]] <= st[n]) ? sl[n] : sr[n];
    score[r * sstride + soff] += sv[n];
  }
}

// Forest inference on raw float features (NaN => default direction).
// Trees are flattened: node arrays indexed globally, tree_root[t], tree_out[t]
// (output column). x_le_thr => left (Tree.java:161-166).
__global__ __launch_bounds__(256) void forest_predict_kernel(
    const float* __restrict__ X, long long xstride, long long N,
    const int* __restrict__ nfeat, const float* __restrict__ nthr,
    const int* __restrict__ nleft, const int* __restrict__ nright,
    const uint8_t* __restrict__ ndefl, const float* __restrict__ nval,
    const int* __restrict__ troot, const int* __restrict__ tout, int T,
    float* __restrict__ out, int ostride, float scale, int* __restrict__ leaf_out) {
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < N;
       r += (long long)gridDim.x * blockDim.x) {
    const float* x = X + r * xstride;
    for (int t = 0; t < T; ++t) {
      int n = troot[t];
      while (nfeat[n] >= 0) {
        const float v = x[nfeat[n]];
        const bool left = (v != v) ? (ndefl[n] != 0) : (v <= nthr[n]);
        n = left ? nleft[n] : nright[n];
      }
      if (leaf_out) leaf_out[r * T + t] = n - troot[t];
      else out[r * ostride + tout[t]] += scale * nval[n];
    }
  }
}

// ---------------------------------------------------------------------------
// Bin assignment: nearest candidate (FeatureApprData.convertFeaVal2ApprFeaIndex)
// ---------------------------------------------------------------------------
template <typename BinT>
__global__ __launch_bounds__(256) void bin_assign_kernel(
    const float* __restrict__ X, long long xstride, long long N, int F,
    const float* __restrict__ cand, const int* __restrict__ coff,
    BinT* __restrict__ out, long long ostride) {
  const long long total = N * F;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / F;
    const int f = (int)(i - r * F);
    const float* c = cand + coff[f];
    const int n = coff[f + 1] - coff[f];
    int idx = 0;
    if (n > 1) {
      const float x = X[r * xstride + f];
      if (x > c[n - 1]) {
        idx = n - 1;
      } else {
        int lo = 0, hi = n - 1;
        while (lo <= hi) {
          const int mid = (lo + hi) >> 1;
          if (x >= c[mid]) lo = mid + 1; else hi = mid - 1;
        }
        const int u = max(0, hi);
        idx = (c[u] == x) ? u : min(n - 1, lo);
        if (idx >= 1 && x < (c[idx] + c[idx - 1]) * 0.5f) idx -= 1;
      }
    }
    out[r * ostride + f] = (BinT)idx;
  }
}

// ---------------------------------------------------------------------------
// Gradients / hessians + weighted loss sum.
// loss ids: 0 sigmoid, 1 l2, 2 l1, 3 poisson, 4 huber(delta), 5 softmax (K>1)
// score/init/label are [N][K]; gh is [K][N] float2; pred [N][K]
// ---------------------------------------------------------------------------
__device__ __forceinline__ double sigmoid_d(double s) {
  if (s >= 0.0) return 1.0 / (1.0 + exp(-s));
  const double e = exp(s);
  return e / (1.0 + e);
}

__global__ __launch_bounds__(256) void grad_hess_kernel(
    const float* __restrict__ score, const float* __restrict__ init, const float* __restrict__ label,
    const float* __restrict__ weight, long long N, int K, int loss_id, float p0, float score_div,
    float* __restrict__ pred, float2* __restrict__ gh, double* __restrict__ loss_acc, int want_grad) {
  __shared__ double s_loss[4], s_w[4];
  double lsum = 0.0, wsum = 0.0;
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < N;
       r += (long long)gridDim.x * blockDim.x) {
    const double w = weight ? (double)weight[r] : 1.0;
    wsum += w;
    if (loss_id == 5) {
      double zmax = -INFINITY;
      for (int k = 0; k < K; ++k) {
        const double z = (double)score[r * K + k] / score_div + (double)init[r * K + k];
        zmax = fmax(zmax, z);
      }
      double den = 0.0;
      for (int k = 0; k < K; ++k) {
        const double z = (double)score[r * K + k] / score_div + (double)init[r * K + k];
        den += exp(z - zmax);
      }
      const double logden = log(den) + zmax;
      double l = 0.0;
      for (int k = 0; k < K; ++k) {
        const double z = (double)score[r * K + k] / score_div + (double)init[r * K + k];
        const double p = exp(z - logden);
        const double y = label[r * K + k];
        l -= y * (z - logden);
        pred[r * K + k] = (float)p;
        if (want_grad) gh[k * N + r] = make_float2((float)((p - y) * w), (float)(2.0 * p * (1.0 - p) * w));
      }
      lsum += w * l;
    } else {
      const double z = (double)score[r] / score_div + (double)init[r];
      const double y = label[r];
      double l, p, g, h;
      switch (loss_id) {
        case 0: {  // sigmoid
          l = (z >= 0.0) ? log1p(exp(-z)) + z * (1.0 - y) : log1p(exp(z)) - z * y;
          p = sigmoid_d(z);
          p = (double)(float)p;  // reference stores predict as float then derives
          g = p - y; h = p * (1.0 - p);
          if (p0 != 0.f) {
            const double zz = (h != 0.0) ? -(g / h) : 0.0;
            if (zz > p0) h = -(g / p0);
            else if (zz < -p0) h = -(g / -p0);
          }
          break;
        }
        case 1: l = 0.5 * (y - z) * (y - z); p = z; p = (double)(float)p; g = p - y; h = 1.0; break;
        case 2: l = fabs(y - z); p = z; p = (double)(float)p; g = (p - y > 0) - (p - y < 0); h = 1.0; break;
        case 3: {  // poisson: -yz + e^min(z,30) + log(y!)
          const double zc = fmin(z, 30.0);
          l = -y * z + exp(zc) + lgamma(y + 1.0);
          p = exp(zc);
          p = (double)(float)p;
          g = p - y; h = p;
          break;
        }
        default: {  // huber, delta = p0
          const double a = z - y, d = p0;
          l = (fabs(a) <= d) ? 0.5 * a * a : d * (fabs(a) - 0.5 * d);
          p = z; p = (double)(float)p;
          const double aa = p - y;
          g = (fabs(aa) <= d) ? aa : ((aa > 0) - (aa < 0)) * d;
          h = 0.0;
          break;
        }
      }
      lsum += w * l;
      pred[r] = (float)p;
      if (want_grad) gh[r] = make_float2((float)(g * w), (float)(h * w));
    }
  }
  lsum = wave_sum(lsum);
  wsum = wave_sum(wsum);
  const int wid = threadIdx.x >> 6;
  if (lane_id() == 0) { s_loss[wid] = lsum; s_w[wid] = wsum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&loss_acc[0], s_loss[0] + s_loss[1] + s_loss[2] + s_loss[3]);
    atomicAdd(&loss_acc[1], s_w[0] + s_w[1] + s_w[2] + s_w[3]);
  }
}

}  // namespace ytk

// ===========================================================================
// Host launchers (C ABI; pointers as uintptr_t, stream as hipStream_t)
// ===========================================================================
using namespace ytk;

extern "C" {

void ytk_hist_u8(uintptr_t bins, long long stride, int F, uintptr_t gh, uintptr_t rows,
                 uintptr_t work, int nwork, uintptr_t hist, int B, uintptr_t stream) {
  if (nwork <= 0) return;
  const int groups = (F + 31) / 32;
  const int nb_lds = B;  // B <= 256 guaranteed by caller
  const size_t lds = (size_t)nb_lds * 64 * sizeof(float);
  dim3 grid(nwork, groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    hipLaunchKernelGGL(hist_u8_lds_kernel<true>, grid, dim3(256), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)gh, (const int*)nullptr,
                       (const int4*)work, (float2*)hist, B, nb_lds);
  } else {
    hipLaunchKernelGGL(hist_u8_lds_kernel<false>, grid, dim3(256), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)gh, (const int*)rows,
                       (const int4*)work, (float2*)hist, B, nb_lds);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_hist_global(uintptr_t bins, int bin_bytes, long long stride, int F, uintptr_t gh,
                     uintptr_t rows, uintptr_t work, int nwork, uintptr_t hist, int B,
                     uintptr_t stream) {
  if (nwork <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(hist_global_kernel<uint8_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint8_t*)bins, stride, F, (const float2*)gh, (const int*)rows,
                       (const int4*)work, (float2*)hist, B);
  } else {
    hipLaunchKernelGGL(hist_global_kernel<uint16_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint16_t*)bins, stride, F, (const float2*)gh, (const int*)rows,
                       (const int4*)work, (float2*)hist, B);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_split_find(uintptr_t hist, int B, int F, uintptr_t nbins_f, uintptr_t fmask, int f0,
                    uintptr_t items, int nitems, uintptr_t out, float mcw, float l1, float l2,
                    float max_abs_leaf, uintptr_t stream) {
  if (nitems <= 0) return;
  GainParams gp{mcw, l1, l2, max_abs_leaf};
  hipLaunchKernelGGL(split_find_kernel, dim3(nitems), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (float2*)hist, B, F,
                     (const int*)nbins_f, (const uint8_t*)fmask, f0, (const int4*)items,
                     (SplitOut*)out, gp);
  YTK_LAUNCH_CHECK();
}

void ytk_partition(uintptr_t bins, int bin_bytes, long long stride, uintptr_t rows,
                   uintptr_t rows_out, uintptr_t items, int nitems, uintptr_t feat,
                   uintptr_t thr, uintptr_t node_begin, uintptr_t first_blk, uintptr_t nblk,
                   uintptr_t counts, uintptr_t left_total, uintptr_t stream) {
  if (nitems <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(partition_count_kernel<uint8_t>, dim3(nitems), dim3(256), 0, s,
                       (const uint8_t*)bins, stride, (const int*)rows, (const int4*)items,
                       (const int*)feat, (const int*)thr, (int*)counts);
    YTK_LAUNCH_CHECK();
    hipLaunchKernelGGL(partition_scatter_kernel<uint8_t>, dim3(nitems), dim3(256), 0, s,
                       (const uint8_t*)bins, stride, (const int*)rows, (int*)rows_out,
                       (const int4*)items, (const int*)feat, (const int*)thr,
                       (const int*)node_begin, (const int*)first_blk, (const int*)nblk,
                       (const int*)counts, (int*)left_total);
  } else {
    hipLaunchKernelGGL(partition_count_kernel<uint16_t>, dim3(nitems), dim3(256), 0, s,
                       (const uint16_t*)bins, stride, (const int*)rows, (const int4*)items,
                       (const int*)feat, (const int*)thr, (int*)counts);
    YTK_LAUNCH_CHECK();
    hipLaunchKernelGGL(partition_scatter_kernel<uint16_t>, dim3(nitems), dim3(256), 0, s,
                       (const uint16_t*)bins, stride, (const int*)rows, (int*)rows_out,
                       (const int4*)items, (const int*)feat, (const int*)thr,
                       (const int*)node_begin, (const int*)first_blk, (const int*)nblk,
                       (const int*)counts, (int*)left_total);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_tree_add_bins(uintptr_t bins, int bin_bytes, long long stride, long long N,
                       uintptr_t tfeat, uintptr_t tthr, uintptr_t tleft, uintptr_t tright,
                       uintptr_t tval, int nnodes, uintptr_t score, int sstride, int soff,
                       uintptr_t stream) {
  if (N <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int grid = (int)std::min<long long>((N + 255) / 256, 256LL * 8);
  const size_t lds = (size_t)nnodes * 5 * sizeof(int);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(tree_add_bins_kernel<uint8_t>, dim3(grid), dim3(256), lds, s,
                       (const uint8_t*)bins, stride, N, (const int*)tfeat, (const int*)tthr,
                       (const int*)tleft, (const int*)tright, (const float*)tval, nnodes,
                       (float*)score, sstride, soff);
  } else {
    hipLaunchKernelGGL(tree_add_bins_kernel<uint16_t>, dim3(grid), dim3(256), lds, s,
                       (const uint16_t*)bins, stride, N, (const int*)tfeat, (const int*)tthr,
                       (const int*)tleft, (const int*)tright, (const float*)tval, nnodes,
                       (float*)score, sstride, soff);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_forest_predict(uintptr_t X, long long xstride, long long N, uintptr_t nfeat,
                        uintptr_t nthr, uintptr_t nleft, uintptr_t nright, uintptr_t ndefl,
                        uintptr_t nval, uintptr_t troot, uintptr_t tout, int T, uintptr_t out,
                        int ostride, float scale, uintptr_t leaf_out, uintptr_t stream) {
  if (N <= 0 || T <= 0) return;
  const int grid = (int)std::min<long long>((N + 255) / 256, 256LL * 8);
  hipLaunchKernelGGL(forest_predict_kernel, dim3(grid), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const float*)X, xstride, N,
                     (const int*)nfeat, (const float*)nthr, (const int*)nleft,
                     (const int*)nright, (const uint8_t*)ndefl, (const float*)nval,
                     (const int*)troot, (const int*)tout, T, (float*)out, ostride, scale,
                     (int*)leaf_out);
  YTK_LAUNCH_CHECK();
}

void ytk_bin_assign(uintptr_t X, long long xstride, long long N, int F, uintptr_t cand,
                    uintptr_t coff, uintptr_t out, int bin_bytes, long long ostride,
                    uintptr_t stream) {
  if (N <= 0) return;
  const long long total = N * F;
  const int grid = (int)std::min<long long>((total + 255) / 256, 256LL * 16);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(bin_assign_kernel<uint8_t>, dim3(grid), dim3(256), 0, s,
                       (const float*)X, xstride, N, F, (const float*)cand, (const int*)coff,
                       (uint8_t*)out, ostride);
  } else {
    hipLaunchKernelGGL(bin_assign_kernel<uint16_t>, dim3(grid), dim3(256), 0, s,
                       (const float*)X, xstride, N, F, (const float*)cand, (const int*)coff,
                       (uint16_t*)out, ostride);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_grad_hess(uintptr_t score, uintptr_t init, uintptr_t label, uintptr_t weight,
                   long long N, int K, int loss_id, float p0, float score_div, uintptr_t pred,
                   uintptr_t gh, uintptr_t loss_acc, int want_grad, uintptr_t stream) {
  if (N <= 0) return;
  const int grid = (int)std::min<long long>((N + 255) / 256, 256LL * 4);
  hipLaunchKernelGGL(grad_hess_kernel, dim3(grid), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const float*)score,
                     (const float*)init, (const float*)label, (const float*)weight, N, K,
                     loss_id, p0, score_div, (float*)pred, (float2*)gh, (double*)loss_acc,
                     want_grad);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
