// GBDT scoring, binning and gradient kernels (gfx950 / CDNA4, wave64).
//
// Reference semantics:
//   tree scoring (train, bin space)  J/data/gbdt/Tree.java:142-154, GBDTOptimizer.java:641-658
//   forest inference (raw floats)    J/data/gbdt/Tree.java:114-168 (x <= cond -> left,
//                                    missing -> default child), GBDTOnlinePredictor.java:170-270
//   bin assignment                   J/data/gbdt/FeatureApprData.java:179-205
//   grad / hess / loss               J/optimizer/GBDTOptimizer.java:513-609 + J/loss/*
//
// Design: the training-score update is FUSED with the loss/gradient pass
// (tree_grad_kernel): one read of score/label/weight per row per round, the new
// tree's leaf found by walking the ROW-MAJOR bin matrix (all levels of the walk hit
// the same 32-B row segment: ~32 B/row vs ~118 B/row for a column-major walk whose
// lanes diverge over features), the node arrays staged in LDS, float math per row,
// an fp64 block sum of the weighted loss, and the max |g| / |h| the next tree's
// fixed-point histogram scales need (block max -> one uint atomicMax per block).
#include "common.h"

#include <stdexcept>

namespace ytk {

// ------------------------------------------------------------------ scoring
template <typename BinT>
__global__ __launch_bounds__(256) void tree_add_bins_kernel(
    const BinT* __restrict__ binsT, long long N, const int* __restrict__ tfeat,
    const int* __restrict__ tthr, const int* __restrict__ tleft, const int* __restrict__ tright,
    const float* __restrict__ tval, int nnodes, float* __restrict__ score, int sstride,
    int soff) {
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
    while (sf[n] >= 0) n = ((int)binsT[(size_t)sf[n] * N + r] <= st[n]) ? sl[n] : sr[n];
    score[r * sstride + soff] += sv[n];
  }
}

// Forest inference on raw float features. Trees flattened: node arrays indexed
// globally, troot[t], tout[t] (output column).
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

// Register walk for narrow dense rows (F = 4 * kF4 <= 32 floats, 16-B aligned): the whole
// row is fetched with kF4 independent 16-B loads and the nodes are staged in LDS, so a
// tree level costs a select chain instead of three dependent global round trips (node
// feature -> x[feature] -> threshold / children). Same comparisons as
// forest_predict_kernel (missing -> default child, v <= thr -> left).
template <int kF4>
__global__ __launch_bounds__(256) void forest_predict_regs_kernel(
    const float* __restrict__ X, long long N, const int* __restrict__ nfeat, const float* __restrict__ nthr,
    const int* __restrict__ nleft, const int* __restrict__ nright, const uint8_t* __restrict__ ndefl,
    const float* __restrict__ nval, const int* __restrict__ troot, const int* __restrict__ tout, int T,
    int nnodes, float* __restrict__ out, int ostride, float scale, int* __restrict__ leaf_out) {
  extern __shared__ __attribute__((aligned(16))) int fsm[];
  int* sf = fsm;  // feature, or -1 (leaf); the default direction rides in bit 30
  float* sth = reinterpret_cast<float*>(fsm + nnodes);
  int* sl = fsm + 2 * nnodes;
  int* sr = fsm + 3 * nnodes;
  float* sv = reinterpret_cast<float*>(fsm + 4 * nnodes);
  for (int i = threadIdx.x; i < nnodes; i += blockDim.x) {
    const int f = nfeat[i];
    sf[i] = f < 0 ? -1 : (f | (ndefl[i] ? (1 << 30) : 0));
    sth[i] = nthr[i]; sl[i] = nleft[i]; sr[i] = nright[i]; sv[i] = nval[i];
  }
  __syncthreads();
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < N;
       r += (long long)gridDim.x * blockDim.x) {
    float x[4 * kF4];
    const float4* r4 = reinterpret_cast<const float4*>(X + r * (4 * kF4));
#pragma unroll
    for (int i = 0; i < kF4; ++i) {
      const float4 v = r4[i];
      x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
    }
    for (int t = 0; t < T; ++t) {
      const int root = troot[t];
      int n = root;
      int fe = sf[n];
      while (fe >= 0) {
        const int f = fe & 0xffff;
        float v = x[0];
#pragma unroll
        for (int i = 1; i < 4 * kF4; ++i) v = (f == i) ? x[i] : v;
        const bool left = (v != v) ? ((fe >> 30) & 1) : (v <= sth[n]);
        n = left ? sl[n] : sr[n];
        fe = sf[n];
      }
      if (leaf_out) leaf_out[r * T + t] = n - root;
      else out[r * ostride + tout[t]] += scale * sv[n];
    }
  }
}

// ------------------------------------------------------------------ binning
template <typename BinT>
__global__ __launch_bounds__(256) void bin_assign_kernel(
    const float* __restrict__ X, long long xstride, long long N, int F,
    const float* __restrict__ cand, const int* __restrict__ coff,
    BinT* __restrict__ out, long long ostride, BinT* __restrict__ outT) {
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
    if (outT) outT[(size_t)f * N + r] = (BinT)idx;
  }
}

// LDS-tiled bin assignment (<= 256 bins, every feature's candidates in LDS): a block loads
// kBinRows rows of X coalesced into LDS, then thread (f, r) -- r fastest, so the column-major
// store of a feature is one contiguous run -- binary-searches its value in the LDS table
// (the same rule as bin_assign_kernel). Replaces per-element searches through L2 and the
// stride-N byte stores (prep: 5.8 ms at 7 % of HBM bandwidth for Higgs).
constexpr int kBinRows = 256;
constexpr int kBinLdsFloats = 8192;  // candidates + X tile
template <typename BinT>
__global__ __launch_bounds__(256) void bin_assign_lds_kernel(
    const float* __restrict__ X, long long xstride, long long N, int F, const float* __restrict__ cand,
    const int* __restrict__ coff, BinT* __restrict__ out, long long ostride, BinT* __restrict__ outT) {
  extern __shared__ float s_mem[];
  const int C = coff[F];
  float* s_cand = s_mem;            // [C]
  float* s_x = s_mem + C;           // [kBinRows][F]
  int* s_off = reinterpret_cast<int*>(s_x + (size_t)kBinRows * F);  // [F + 1]
  for (int i = threadIdx.x; i < C; i += 256) s_cand[i] = cand[i];
  for (int i = threadIdx.x; i <= F; i += 256) s_off[i] = coff[i];
  for (long long r0 = (long long)blockIdx.x * kBinRows; r0 < N; r0 += (long long)gridDim.x * kBinRows) {
    const int R = (int)min((long long)kBinRows, N - r0);
    __syncthreads();
    for (int i = threadIdx.x; i < R * F; i += 256) {
      const int rr = i / F, f = i - rr * F;
      s_x[i] = X[(r0 + rr) * xstride + f];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R * F; i += 256) {
      const int f = i / R, rr = i - f * R;
      const float* c = s_cand + s_off[f];
      const int n = s_off[f + 1] - s_off[f];
      int idx = 0;
      if (n > 1) {
        const float x = s_x[rr * F + f];
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
      out[(r0 + rr) * ostride + f] = (BinT)idx;
      if (outT) outT[(size_t)f * N + r0 + rr] = (BinT)idx;
    }
  }
}

// ------------------------------------------------------------------ loss / grad
// loss ids: 0 sigmoid, 1 l2, 2 l1, 3 poisson, 4 huber(delta=p0), 5 softmax (K>1)
// fp64 like the CPU path and the reference (z = score / div + init in double, the
// prediction rounded to float, g / h from that float prediction in double, then g * w and
// h * w rounded to float): the GPU path reproduces the reference's per-round losses to
// 1e-12 (test_gbdt_demo_readme_losses_on_device).
struct LossOut {
  float p;
  double g, h;
  double l;
};

// kLoss is a compile-time parameter of the kernels: only the selected loss's fp64 code is
// compiled into a kernel (a runtime switch over all five kept ~200 VGPRs live: 2 waves/SIMD)
// lgy1: the Poisson loss's label term lgamma(y + 1), computed once per data set on the host side
// (ops/gbdt.py): the device lgamma inlined into the fused gradient + histogram kernel cost 238
// VGPR spills and 512 B of scratch per thread (as gbst.hip's GbstArgs::lgy)
template <int kLoss>
__device__ __forceinline__ LossOut point_loss(double z, double y, double p0, double lgy1 = 0.0) {
  LossOut o;
  switch (kLoss) {
    case 0: {  // sigmoid (SigmoidFunction: stable log-loss, zmax hessian clamp)
      const double az = fabs(z);
      const double e = exp(-az);
      o.l = log1p(e) + (z >= 0.0 ? z * (1.0 - y) : -z * y);
      o.p = (float)((z >= 0.0) ? 1.0 / (1.0 + e) : e / (1.0 + e));
      const double p = (double)o.p;
      o.g = p - y;
      o.h = p * (1.0 - p);
      if (p0 != 0.0) {
        const double zz = (o.h != 0.0) ? -(o.g / o.h) : 0.0;
        if (zz > p0) o.h = -(o.g / p0);
        else if (zz < -p0) o.h = -(o.g / -p0);
      }
      break;
    }
    case 1:
      o.l = 0.5 * (y - z) * (y - z);
      o.p = (float)z; o.g = (double)o.p - y; o.h = 1.0;
      break;
    case 2: {
      o.l = fabs(y - z);
      o.p = (float)z;
      const double d = (double)o.p - y;
      o.g = (double)((d > 0.0) - (d < 0.0)); o.h = 1.0;
      break;
    }
    case 3: {
      const double zc = fmin(z, 30.0);
      const double ez = exp(zc);
      o.l = -y * z + ez + lgy1;
      o.p = (float)ez;
      o.g = (double)o.p - y; o.h = (double)o.p;
      break;
    }
    default: {
      const double a = z - y, d = p0;
      o.l = (fabs(a) <= d) ? 0.5 * a * a : d * (fabs(a) - 0.5 * d);
      o.p = (float)z;
      const double aa = (double)o.p - y;
      o.g = (fabs(aa) <= d) ? aa : ((aa > 0.0) - (aa < 0.0)) * d;
      o.h = 0.0;
      break;
    }
  }
  return o;
}

__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Block reduction of (loss, weight) sums and (max|g|, max|h|); one atomic each per block.
// Deterministic grid reduction of the (loss, weight) sums: every block stores its partial
// into loss_acc[kAccPart + 2 * block]; acc_finish_kernel (one block, launched right after)
// adds them in block order -- the fp64 sums are bitwise reproducible run to run (float
// atomics would add in arrival order; a last-block-done counter serialised ~2k returning
// atomics on one address: measured +40 us per launch). (max|g|, max|h|) use integer
// atomicMax (order independent). loss_acc must hold kAccLen doubles.
constexpr int kAccPart = 4;
constexpr int kAccMaxBlocks = 256 * 8;
constexpr int kAccLen = kAccPart + 2 * kAccMaxBlocks;

__device__ __forceinline__ void block_acc(double lsum, double wsum, double* loss_acc, float mg,
                                          float mh, float* ghmax) {
  __shared__ double s_loss[4], s_w[4];
  __shared__ float s_mg[4], s_mh[4];
  lsum = wave_sum(lsum);
  wsum = wave_sum(wsum);
  mg = wave_maxf(mg);
  mh = wave_maxf(mh);
  const int wid = threadIdx.x >> 6;
  if (lane_id() == 0) { s_loss[wid] = lsum; s_w[wid] = wsum; s_mg[wid] = mg; s_mh[wid] = mh; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* part = loss_acc + kAccPart;
    part[2 * blockIdx.x] = s_loss[0] + s_loss[1] + s_loss[2] + s_loss[3];
    part[2 * blockIdx.x + 1] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    if (ghmax) {  // non-negative floats order like their bit patterns
      atomicMax(reinterpret_cast<unsigned*>(&ghmax[0]),
                __float_as_uint(fmaxf(fmaxf(s_mg[0], s_mg[1]), fmaxf(s_mg[2], s_mg[3]))));
      atomicMax(reinterpret_cast<unsigned*>(&ghmax[1]),
                __float_as_uint(fmaxf(fmaxf(s_mh[0], s_mh[1]), fmaxf(s_mh[2], s_mh[3]))));
    }
  }
}

// loss_acc[0:2] = sum over the nblocks partials, in block order (fixed per-thread strides,
// then thread order).
// out (optional): where the two sums go (default loss_acc[0:2]) -- the round tail writes the
// train and test sums next to each other so one copy reads them back.
__device__ __forceinline__ void acc_finish_body(double* __restrict__ loss_acc, int nblocks,
                                                double* __restrict__ out = nullptr) {
  __shared__ double s_red[2][256];
  const double* part = loss_acc + kAccPart;
  double a = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < nblocks; i += 256) {
    a += part[2 * i];
    c += part[2 * i + 1];
  }
  s_red[0][threadIdx.x] = a;
  s_red[1][threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = 0.0, tc = 0.0;
    for (int t = 0; t < 256; ++t) { ta += s_red[0][t]; tc += s_red[1][t]; }
    double* o = out ? out : loss_acc;
    o[0] = ta;
    o[1] = tc;
  }
}

// block 0: loss_acc -> out (or in place); block 1 (acc2 != nullptr): acc2 -> out2 -- a second
// pass's partials (the test-set tail) finished by the same launch
__global__ __launch_bounds__(256) void acc_finish_kernel(double* __restrict__ loss_acc, int nblocks,
                                                         double* __restrict__ out, double* __restrict__ acc2,
                                                         int nblocks2, double* __restrict__ out2) {
  if (blockIdx.x == 0) acc_finish_body(loss_acc, nblocks, out);
  else acc_finish_body(acc2, nblocks2, out2);
}

// Test-set round tail in one pass (K == 1, one new tree): walk the raw row held in
// registers (as forest_predict_regs_kernel), score += leaf value, then the point loss and
// prediction (as tree_grad_kernel without gradients). Same grid and row -> thread mapping
// as the grad_hess launch it replaces, so the fp64 loss sums are bitwise the same.
template <int kF4, int kLoss>
__global__ __launch_bounds__(256) void forest_loss_regs_kernel(
    const float* __restrict__ X, long long N, const int* __restrict__ nfeat, const float* __restrict__ nthr,
    const int* __restrict__ nleft, const int* __restrict__ nright, const uint8_t* __restrict__ ndefl,
    const float* __restrict__ nval, int root, int nnodes, float* __restrict__ score,
    const float* __restrict__ init, const float* __restrict__ label, const double* __restrict__ lgy,
    const float* __restrict__ weight, float p0, float score_div, float* __restrict__ pred,
    double* __restrict__ loss_acc) {
  extern __shared__ __attribute__((aligned(16))) int fsm[];
  int* sf = fsm;
  float* sth = reinterpret_cast<float*>(fsm + nnodes);
  int* sl = fsm + 2 * nnodes;
  int* sr = fsm + 3 * nnodes;
  float* sv = reinterpret_cast<float*>(fsm + 4 * nnodes);
  for (int i = threadIdx.x; i < nnodes; i += blockDim.x) {
    const int f = nfeat[i];
    sf[i] = f < 0 ? -1 : (f | (ndefl[i] ? (1 << 30) : 0));
    sth[i] = nthr[i]; sl[i] = nleft[i]; sr[i] = nright[i]; sv[i] = nval[i];
  }
  __syncthreads();
  double lsum = 0.0, wsum = 0.0;
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < N;
       r += (long long)gridDim.x * blockDim.x) {
    float x[4 * kF4];
    const float4* r4 = reinterpret_cast<const float4*>(X + r * (4 * kF4));
#pragma unroll
    for (int i = 0; i < kF4; ++i) {
      const float4 v = r4[i];
      x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
    }
    const float s0 = score[r], ini = init[r], lab = label[r];
    const float w = weight ? weight[r] : 1.f;
    // the row goes to a thread-private LDS slot (4 kF4 + 1 floats: odd stride) and each level
    // reads its feature with one LDS load instead of a (4 kF4)-way register select chain
    float* slot = reinterpret_cast<float*>(fsm + 5 * nnodes) + (size_t)threadIdx.x * (4 * kF4 + 1);
#pragma unroll
    for (int i = 0; i < 4 * kF4; ++i) slot[i] = x[i];
    int n = root;
    int fe = sf[n];
    while (fe >= 0) {
      const float v = slot[fe & 0xffff];
      const bool left = (v != v) ? ((fe >> 30) & 1) : (v <= sth[n]);
      n = left ? sl[n] : sr[n];
      fe = sf[n];
    }
    const float s = s0 + 1.0f * sv[n];  // forest_predict: out += scale * value, scale 1
    score[r] = s;
    const LossOut o = point_loss<kLoss>((double)s / (double)score_div + (double)ini, (double)lab, (double)p0,
                                        kLoss == 3 ? lgy[r] : 0.0);
    lsum += (double)w * o.l;
    wsum += (double)w;
    if (pred) pred[r] = o.p;
  }
  block_acc(lsum, wsum, loss_acc, 0.f, 0.f, nullptr);
}

// Leaf of a bin-threshold tree for one row held in registers (kDw dwords, packed bins):
// the whole row is fetched with 16-B loads (a wave reads 64 contiguous rows), then
// every level extracts its feature with a select chain -- no dependent memory loads.
template <int kDw>
__device__ __forceinline__ void load_row_regs(const void* row, uint32_t (&d)[kDw]) {
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
#pragma unroll
  for (int i = 0; i < kDw / 4; ++i) {
    const uint4 v = r4[i];
    d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
  }
}

template <typename BinT, int kDw>
__device__ __forceinline__ int walk_regs(const uint32_t (&d)[kDw], const int* sf, const int* st,
                                         const int* sl, const int* sr) {
  constexpr int kPer = 4 / sizeof(BinT);
  constexpr unsigned kMask = sizeof(BinT) == 1 ? 0xffu : 0xffffu;
  int n = 0;
  while (sf[n] >= 0) {
    const int f = sf[n];
    const int w = f / kPer;
    uint32_t v = d[0];
#pragma unroll
    for (int i = 1; i < kDw; ++i) v = (w == i) ? d[i] : v;
    const int b = (int)((v >> ((f % kPer) * 8 * sizeof(BinT))) & kMask);
    n = (b <= st[n]) ? sl[n] : sr[n];
  }
  return n;
}

template <typename BinT, int kDw>
__device__ __forceinline__ int walk_row_regs(const BinT* row, const int* sf, const int* st,
                                             const int* sl, const int* sr) {
  uint32_t d[kDw];
  load_row_regs<kDw>(row, d);
  return walk_regs<BinT, kDw>(d, sf, st, sl, sr);
}

// rows per thread whose loads are in flight together in tree_grad_kernel's register walk
// (1 -> 2: 148 -> 136 us per Higgs round; 4: 121 VGPRs, 141 us)
constexpr int kTreeGradRows = 2;

// K == 1 losses, optionally fused with the new tree's score update (row-major bins walk).
// kDw > 0: rows of exactly kDw dwords walked in registers; kDw == 0: generic byte loads.
// kNodesGlobal: the node arrays do not fit in LDS (trees of > ~8k nodes, e.g. a host-built
// leaf-wise tree with a large max_leaf_cnt): the walk reads them from global memory (byte
// walk only, no leaf counts)
template <typename BinT, int kDw, int kLoss, bool kLdsWalk = false, bool kNodesGlobal = false>
__global__ __launch_bounds__(256) void tree_grad_kernel(
    const BinT* __restrict__ bins, long long stride, const int* __restrict__ tfeat,
    const int* __restrict__ tthr, const int* __restrict__ tleft, const int* __restrict__ tright,
    const float* __restrict__ tval, int nnodes, float* __restrict__ score,
    const float* __restrict__ init, const float* __restrict__ label, const double* __restrict__ lgy,
    const float* __restrict__ weight, long long N, int loss_id, float p0, float score_div,
    float* __restrict__ pred, float2* __restrict__ gh, double* __restrict__ loss_acc,
    int want_grad, float* __restrict__ ghmax, int* __restrict__ leaf_part) {
  extern __shared__ __attribute__((aligned(16))) int tsm[];
  static_assert(!kNodesGlobal || (kDw == 0 && !kLdsWalk), "global-node walk: byte walk only");
  const int* sf = kNodesGlobal ? tfeat : tsm;
  const int* st = kNodesGlobal ? tthr : tsm + nnodes;
  const int* sl = kNodesGlobal ? tleft : tsm + 2 * nnodes;
  const int* sr = kNodesGlobal ? tright : tsm + 3 * nnodes;
  const float* sv = kNodesGlobal ? tval : reinterpret_cast<const float*>(tsm + 4 * nnodes);
  int* sc = tsm + 5 * nnodes;  // leaf_part: rows per node of this block
  if constexpr (!kNodesGlobal) {
    float* svw = reinterpret_cast<float*>(tsm + 4 * nnodes);
    for (int i = threadIdx.x; i < nnodes; i += blockDim.x) {
      tsm[i] = tfeat[i]; tsm[nnodes + i] = tthr[i]; tsm[2 * nnodes + i] = tleft[i];
      tsm[3 * nnodes + i] = tright[i]; svw[i] = tval[i];
      if (leaf_part) sc[i] = 0;
    }
    __syncthreads();
  }
  double lsum = 0.0, wsum = 0.0;
  float mg = 0.f, mh = 0.f;
  long long r0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long G = (long long)gridDim.x * blockDim.x;
  // the leaf / loss / gradient of one row whose inputs are already in registers
  auto finish_row = [&](long long r, float s, int n, float ini, float lab, float w) {
    s += sv[n];
    score[r] = s;
    if (leaf_part) atomicAdd(&sc[n], 1);
    const LossOut o = point_loss<kLoss>((double)s / (double)score_div + (double)ini, (double)lab, (double)p0,
                                        kLoss == 3 ? lgy[r] : 0.0);
    lsum += (double)w * o.l;
    wsum += (double)w;
    if (pred) pred[r] = o.p;
    if (want_grad) {
      const float gg = (float)(o.g * (double)w), hh = (float)(o.h * (double)w);
      gh[r] = make_float2(gg, hh);
      mg = fmaxf(mg, fabsf(gg));
      mh = fmaxf(mh, fabsf(hh));
    }
  };
  if constexpr (kDw > 0) {
    if (nnodes > 0) {
      // kTreeGradRows rows (r, r + G, ...) per iteration with every load issued before any
      // walk: the row loop was latency bound at one row in flight per thread. The rows of
      // a thread are still accumulated in the order r, r + G, r + 2G, ... (fp64 sums
      // unchanged)
      constexpr int U = kTreeGradRows;
      for (; r0 + (U - 1) * G < N; r0 += U * G) {
        uint32_t d[U][kDw];
        float sc0[U], in0[U], lb0[U], wt0[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long r = r0 + u * G;
          load_row_regs<kDw>(bins + r * stride, d[u]);
          sc0[u] = score[r];
          in0[u] = init[r];
          lb0[u] = label[r];
          wt0[u] = weight ? weight[r] : 1.f;
        }
        if constexpr (kLdsWalk) {
          // the rows go to thread-private LDS slots (kDw + 1 dwords: odd stride, the byte
          // reads of a wave spread over the banks) and each level reads its feature's bin
          // with one LDS byte load instead of a kDw-way register select chain (the walk's
          // VALU work; the kernel is VALU-bound with the fp64 loss)
          uint32_t* s_rows = reinterpret_cast<uint32_t*>(tsm + (leaf_part ? 6 : 5) * nnodes);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            uint32_t* slot = s_rows + ((size_t)u * blockDim.x + threadIdx.x) * (kDw + 1);
#pragma unroll
            for (int k = 0; k < kDw; ++k) slot[k] = d[u][k];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const BinT* rb = reinterpret_cast<const BinT*>(s_rows + ((size_t)u * blockDim.x + threadIdx.x) * (kDw + 1));
            int n = 0;
            for (int f = sf[0]; f >= 0; f = sf[n]) n = ((int)rb[f] <= st[n]) ? sl[n] : sr[n];
            finish_row(r0 + u * G, sc0[u], n, in0[u], lb0[u], wt0[u]);
          }
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            finish_row(r0 + u * G, sc0[u], walk_regs<BinT, kDw>(d[u], sf, st, sl, sr), in0[u], lb0[u], wt0[u]);
        }
      }
    }
  }
  for (long long r = r0; r < N; r += G) {
    float s = score[r];
    if (nnodes > 0) {
      const BinT* row = bins + r * stride;
      int n = 0;
      if constexpr (kDw > 0) {
        n = walk_row_regs<BinT, kDw>(row, sf, st, sl, sr);
      } else {
        while (sf[n] >= 0) n = ((int)row[sf[n]] <= st[n]) ? sl[n] : sr[n];
      }
      s += sv[n];
      score[r] = s;
      if (!kNodesGlobal && leaf_part) atomicAdd(&sc[n], 1);
    }
    const float w = weight ? weight[r] : 1.f;
    const LossOut o = point_loss<kLoss>((double)s / (double)score_div + (double)init[r], (double)label[r],
                                        (double)p0, kLoss == 3 ? lgy[r] : 0.0);
    lsum += (double)w * o.l;
    wsum += (double)w;
    if (pred) pred[r] = o.p;
    if (want_grad) {
      const float gg = (float)(o.g * (double)w), hh = (float)(o.h * (double)w);
      gh[r] = make_float2(gg, hh);
      mg = fmaxf(mg, fabsf(gg));
      mh = fmaxf(mh, fabsf(hh));
    }
  }
  block_acc(lsum, wsum, loss_acc, mg, mh, ghmax);
  if (!kNodesGlobal && leaf_part) {
    __syncthreads();
    for (int i = threadIdx.x; i < nnodes; i += blockDim.x) leaf_part[(size_t)blockIdx.x * nnodes + i] = sc[i];
  }
}

// ------------------------------------------------------------------ fused root histogram
// tree_grad + the NEXT tree's root histogram in one pass (K == 1, uint8 rows of 32 bytes,
// no row sampling, fixed-point scales fixed before the pass -- the sigmoid gradient bound).
// The gradient pass already holds every row's 32-byte bin row and produces its (g, h), so
// the root histogram (HistogramBuilder.java:56-90 over all rows) costs LDS atomics here
// instead of a second read of the bins and (g, h) (~420 MB per Higgs round).
//
// Layout: 1024-thread blocks, one per CU (the exact int64 histogram is 256 bins x [32 g | 32 h]
// words = 128 KiB of LDS). Each block is FOUR virtual 256-thread blocks of tree_grad_kernel:
// virtual block vb = 4 blockIdx.x + tid / 256 walks exactly the rows tree_grad_kernel's
// block vb walks and writes its fp64 loss partial to the same slot, so the loss sums, (g, h),
// scores and leaf counts are bitwise those of the unfused kernel.
// Histogram adds: a thread owns a whole row; lane l rotates its row by l % 32 bytes so that
// at step k the 16 lanes of an ds_add_u64 group update 16 distinct features ((k + l) % 32):
// word bin * 64 + f (g) / + 32 (h) -> bank pair f % 16, conflict free. Bytes past F are the
// row padding (bin 0): they land in columns the flush never reads.
constexpr int kTGHThreads = 1024;
constexpr int kTGHVirtual = kTGHThreads / 256;
constexpr size_t kTGHHistBytes = (size_t)256 * 64 * sizeof(unsigned long long);

__device__ __forceinline__ unsigned long long tgh_fx_round(float y) {  // == fx_round (gbdt_hist.hip)
  const float r = __builtin_rintf(y);
  const float a = fabsf(r);
  const float hi = floorf(a * 0x1p-32f);
  const float lo = __builtin_fmaf(hi, -0x1p32f, a);
  const unsigned long long u = ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
  const unsigned long long m = r < 0.f ? ~0ull : 0ull;
  return (u ^ m) - m;
}

__device__ __forceinline__ void tgh_add_row(const uint32_t (&d)[8], int rot, unsigned long long gi,
                                            unsigned long long hi, unsigned long long* hsm) {
  // e = the row rotated by rot / 4 dwords, then r = e shifted by rot % 4 bytes: byte k of r is
  // byte (k + rot) % 32 of the row
  const int q = rot >> 2, b = rot & 3;
  uint32_t e[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t x = d[i & 7];
#pragma unroll
    for (int j = 1; j < 8; ++j) x = (q == j) ? d[(i + j) & 7] : x;
    e[i] = x;
  }
  e[8] = e[0];
  uint32_t r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = __builtin_amdgcn_alignbyte(e[i + 1], e[i], b);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const unsigned bin = __builtin_amdgcn_ubfe(r[k >> 2], 8 * (k & 3), 8);
    const int f = (k + rot) & 31;
    unsigned long long* p = hsm + (bin * 64 + f);
    atomicAdd(p, gi);
    atomicAdd(p + 32, hi);
  }
}

template <int kLoss, int kRows>
__global__ __launch_bounds__(kTGHThreads) void tree_grad_hist_kernel(
    const uint8_t* __restrict__ bins, long long stride, const int* __restrict__ tfeat,
    const int* __restrict__ tthr, const int* __restrict__ tleft, const int* __restrict__ tright,
    const float* __restrict__ tval, int nnodes, float* __restrict__ score,
    const float* __restrict__ init, const float* __restrict__ label, const double* __restrict__ lgy,
    const float* __restrict__ weight, long long N, float p0, float score_div,
    float* __restrict__ pred, float2* __restrict__ gh, double* __restrict__ loss_acc,
    float* __restrict__ ghmax, int* __restrict__ leaf_part, int nvb, const float* __restrict__ scales,
    long long* __restrict__ staging, int B, unsigned long long* __restrict__ zero, long long zero_n) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long hsm[];
  int* tsm = reinterpret_cast<int*>(hsm + 256 * 64);
  if (zero) {
    // the histogram slab of the next tree (16-byte aligned, zero_n uint64): zeroed here instead
    // of by a fill launch at the end of the previous tree; the root reduce behind this kernel
    // accumulates into it
    ulonglong2* z2 = reinterpret_cast<ulonglong2*>(zero);
    for (long long i = (long long)blockIdx.x * kTGHThreads + threadIdx.x; i < (zero_n >> 1);
         i += (long long)gridDim.x * kTGHThreads)
      z2[i] = make_ulonglong2(0ull, 0ull);
    if ((zero_n & 1) && blockIdx.x == 0 && threadIdx.x == 0) zero[zero_n - 1] = 0ull;
  }
  int* sf = tsm;
  int* st = tsm + nnodes;
  int* sl = tsm + 2 * nnodes;
  int* sr = tsm + 3 * nnodes;
  float* sv = reinterpret_cast<float*>(tsm + 4 * nnodes);
  int* sc = tsm + 5 * nnodes;  // leaf_part: rows per node of this block's virtual blocks
  const int tid = threadIdx.x;
  for (int i = tid; i < 256 * 64; i += kTGHThreads) hsm[i] = 0ull;
  for (int i = tid; i < nnodes; i += kTGHThreads) {
    sf[i] = tfeat[i]; st[i] = tthr[i]; sl[i] = tleft[i]; sr[i] = tright[i]; sv[i] = tval[i];
  }
  if (leaf_part)
    for (int i = tid; i < kTGHVirtual * nnodes; i += kTGHThreads) sc[i] = 0;
  __syncthreads();
  const float sg = scales[0], sh = scales[1];
  const int vsub = tid >> 8;
  const int vb = blockIdx.x * kTGHVirtual + vsub;
  const int rot = tid & 31;
  int* scv = sc + vsub * nnodes;
  double lsum = 0.0, wsum = 0.0;
  float mg = 0.f, mh = 0.f;
  if (vb < nvb) {
    const long long G = (long long)nvb * 256;
    long long r0 = (long long)vb * 256 + (tid & 255);
    auto finish_row = [&](long long r, const uint32_t (&d)[8], float s, int n, float ini, float lab, float w) {
      s += sv[n];
      score[r] = s;
      if (leaf_part) atomicAdd(&scv[n], 1);
      const LossOut o = point_loss<kLoss>((double)s / (double)score_div + (double)ini, (double)lab, (double)p0,
                                          kLoss == 3 ? lgy[r] : 0.0);
      lsum += (double)w * o.l;
      wsum += (double)w;
      if (pred) pred[r] = o.p;
      const float gg = (float)(o.g * (double)w), hh = (float)(o.h * (double)w);
      gh[r] = make_float2(gg, hh);
      mg = fmaxf(mg, fabsf(gg));
      mh = fmaxf(mh, fabsf(hh));
      tgh_add_row(d, rot, tgh_fx_round(gg * sg), tgh_fx_round(hh * sh), hsm);
    };
    constexpr int U = kRows;  // rows in flight per thread (YTK_TGH_ROWS)
    for (; r0 + (U - 1) * G < N; r0 += U * G) {
      uint32_t d[U][8];
      float sc0[U], in0[U], lb0[U], wt0[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long r = r0 + u * G;
        load_row_regs<8>(bins + r * stride, d[u]);
        sc0[u] = score[r];
        in0[u] = init[r];
        lb0[u] = label[r];
        wt0[u] = weight ? weight[r] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        finish_row(r0 + u * G, d[u], sc0[u], walk_regs<uint8_t, 8>(d[u], sf, st, sl, sr), in0[u], lb0[u], wt0[u]);
    }
    for (long long r = r0; r < N; r += G) {
      uint32_t d[8];
      load_row_regs<8>(bins + r * stride, d);
      const float w = weight ? weight[r] : 1.f;
      finish_row(r, d, score[r], walk_regs<uint8_t, 8>(d, sf, st, sl, sr), init[r], label[r], w);
    }
  }
  // per virtual block: the fp64 partials in tree_grad_kernel's order (wave sums, then the
  // virtual block's 4 waves left to right), in its partial slot
  {
    __shared__ double s_loss[kTGHThreads / 64], s_w[kTGHThreads / 64];
    __shared__ float s_mg[kTGHThreads / 64], s_mh[kTGHThreads / 64];
    lsum = wave_sum(lsum);
    wsum = wave_sum(wsum);
    mg = wave_maxf(mg);
    mh = wave_maxf(mh);
    const int wid = tid >> 6;
    if (lane_id() == 0) { s_loss[wid] = lsum; s_w[wid] = wsum; s_mg[wid] = mg; s_mh[wid] = mh; }
    __syncthreads();
    if (tid < kTGHVirtual) {
      const int v = blockIdx.x * kTGHVirtual + tid;
      if (v < nvb) {
        double* part = loss_acc + kAccPart;
        const double* a = s_loss + 4 * tid;
        const double* c = s_w + 4 * tid;
        part[2 * v] = a[0] + a[1] + a[2] + a[3];
        part[2 * v + 1] = c[0] + c[1] + c[2] + c[3];
      }
    }
    if (tid == 0 && ghmax) {
      float x = 0.f, y = 0.f;
      for (int i = 0; i < kTGHThreads / 64; ++i) { x = fmaxf(x, s_mg[i]); y = fmaxf(y, s_mh[i]); }
      atomicMax(reinterpret_cast<unsigned*>(&ghmax[0]), __float_as_uint(x));
      atomicMax(reinterpret_cast<unsigned*>(&ghmax[1]), __float_as_uint(y));
    }
  }
  __syncthreads();
  if (leaf_part) {
    for (int i = tid; i < kTGHVirtual * nnodes; i += kTGHThreads) {
      const int v = blockIdx.x * kTGHVirtual + i / nnodes;
      if (v < nvb) leaf_part[(size_t)v * nnodes + (i % nnodes)] = sc[i];
    }
  }
  // the block's histogram partial -> staging item blockIdx.x (hist_reduce_kernel layout:
  // entry bin * 32 + f, one (g, h) pair each; split-K reduced into the root slot)
  longlong2* stg = reinterpret_cast<longlong2*>(staging) + (size_t)blockIdx.x * B * 32;
  for (int i = tid; i < B * 32; i += kTGHThreads) {
    const int bin = i >> 5, f = i & 31;
    stg[i] = make_longlong2((long long)hsm[bin * 64 + f], (long long)hsm[bin * 64 + 32 + f]);
  }
}

// out[node] = rows of the tree's node over all tree_grad blocks (one block per node, block
// order sums: deterministic), as doubles next to the round's loss sums
__global__ __launch_bounds__(256) void leaf_count_reduce_kernel(const int* __restrict__ part, int nblocks, int nnodes,
                                                                double* __restrict__ out, double* __restrict__ loss_acc,
                                                                double* __restrict__ acc_out, double* __restrict__ acc2,
                                                                int nblocks2, double* __restrict__ acc2_out) {
  __shared__ long long s_red[256];
  if (blockIdx.x == (unsigned)nnodes) {  // the extra block: the loss sums (acc_finish_kernel's work)
    acc_finish_body(loss_acc, nblocks, acc_out);
    return;
  }
  if (blockIdx.x == (unsigned)nnodes + 1) {  // a second pass's loss sums (the test-set tail)
    acc_finish_body(acc2, nblocks2, acc2_out);
    return;
  }
  const int node = blockIdx.x;
  long long a = 0;
  for (int b = threadIdx.x; b < nblocks; b += 256) a += part[(size_t)b * nnodes + node];
  s_red[threadIdx.x] = a;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) s_red[threadIdx.x] += s_red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[node] = (double)s_red[0];
}

// softmax over K classes; ghmax is [K][2] (one (max|g|, max|h|) pair per class tree)
__global__ __launch_bounds__(256) void softmax_grad_kernel(
    const float* __restrict__ score, const float* __restrict__ init,
    const float* __restrict__ label, const float* __restrict__ weight, long long N, int K,
    float score_div, float* __restrict__ pred, float2* __restrict__ gh,
    double* __restrict__ loss_acc, int want_grad, float* __restrict__ ghmax) {
  double lsum = 0.0, wsum = 0.0;
  for (long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x; r < N;
       r += (long long)gridDim.x * blockDim.x) {
    const float w = weight ? weight[r] : 1.f;
    wsum += (double)w;
    // the CPU path's order: z = score / div + init in fp64, lse = max + log(sum exp(z - max)),
    // p = exp(z - lse), loss = -sum y (z - lse)
    auto zk = [&](int k) { return (double)score[r * K + k] / (double)score_div + (double)init[r * K + k]; };
    double zmax = -INFINITY;
    for (int k = 0; k < K; ++k) zmax = fmax(zmax, zk(k));
    double den = 0.0;
    for (int k = 0; k < K; ++k) den += exp(zk(k) - zmax);
    const double lse = zmax + log(den);
    double lt = 0.0;
    for (int k = 0; k < K; ++k) lt += (double)label[r * K + k] * (zk(k) - lse);
    lsum += (double)w * -lt;
    for (int k = 0; k < K; ++k) {
      const double p = exp(zk(k) - lse);
      const double y = label[r * K + k];
      if (pred) pred[r * K + k] = (float)p;
      if (want_grad) {
        const float gg = (float)((p - y) * (double)w), hh = (float)(2.0 * p * (1.0 - p) * (double)w);
        gh[k * N + r] = make_float2(gg, hh);
        if (ghmax) {
          atomicMax(reinterpret_cast<unsigned*>(&ghmax[2 * k]), __float_as_uint(fabsf(gg)));
          atomicMax(reinterpret_cast<unsigned*>(&ghmax[2 * k + 1]), __float_as_uint(fabsf(hh)));
        }
      }
    }
  }
  block_acc(lsum, wsum, loss_acc, 0.f, 0.f, nullptr);
}

}  // namespace ytk

using namespace ytk;

static inline int grid_for(long long n, int cap) {
  return (int)std::min<long long>((n + 255) / 256, (long long)cap);
}

// Virtual blocks (256 rows each per step) of the fused gradient + root histogram pass: at
// most YTK_TGH_VBLOCKS (default 1024 = 256 physical 1024-thread blocks, one per CU: each
// holds the 128-KiB root histogram in LDS). Every physical block flushes a 128-KiB partial
// that the root reduce reads back, so fewer, longer blocks trade row parallelism for flush +
// reduce bytes. Measured (profiles/r5/chk4_*_vb*): 2048 -> 1024 virtual blocks 1.333 ->
// 1.315 ms per full tree, 0.433 -> 0.418 ms at the 1/8 shard; 512: 1.508 / 0.437.
// rows each thread of the fused pass keeps in flight (YTK_TGH_ROWS = 1 | 2)
static int tgh_rows() {
  static const int v = [] {
    const char* e = getenv("YTK_TGH_ROWS");
    return (e && e[0] == '1') ? 1 : 2;
  }();
  return v;
}

static int tgh_vblocks(long long N) {
  static const int cap = [] {
    const char* e = getenv("YTK_TGH_VBLOCKS");
    const int v = e ? atoi(e) : 1024;
    return std::max(4, std::min(v, 8192)) & ~3;
  }();
  return grid_for(N, cap);
}

extern "C" {

void ytk_tree_add_bins(uintptr_t binsT, int bin_bytes, long long N, uintptr_t tfeat,
                       uintptr_t tthr, uintptr_t tleft, uintptr_t tright, uintptr_t tval,
                       int nnodes, uintptr_t score, int sstride, int soff, uintptr_t stream) {
  if (N <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = (size_t)nnodes * 5 * sizeof(int);
  const int grid = grid_for(N, 256 * 16);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(tree_add_bins_kernel<uint8_t>, dim3(grid), dim3(256), lds, s,
                       (const uint8_t*)binsT, N, (const int*)tfeat, (const int*)tthr,
                       (const int*)tleft, (const int*)tright, (const float*)tval, nnodes,
                       (float*)score, sstride, soff);
  } else {
    hipLaunchKernelGGL(tree_add_bins_kernel<uint16_t>, dim3(grid), dim3(256), lds, s,
                       (const uint16_t*)binsT, N, (const int*)tfeat, (const int*)tthr,
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
  hipLaunchKernelGGL(forest_predict_kernel, dim3(grid_for(N, 256 * 16)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const float*)X, xstride, N,
                     (const int*)nfeat, (const float*)nthr, (const int*)nleft,
                     (const int*)nright, (const uint8_t*)ndefl, (const float*)nval,
                     (const int*)troot, (const int*)tout, T, (float*)out, ostride, scale,
                     (int*)leaf_out);
  YTK_LAUNCH_CHECK();
}

// Fused test-set tail (forest_loss_regs_kernel + the ordered acc finish); returns 0
// (nothing launched) when the row layout / tree size does not qualify.
int ytk_forest_loss_regs(uintptr_t X, long long xstride, long long N, uintptr_t nfeat, uintptr_t nthr,
                         uintptr_t nleft, uintptr_t nright, uintptr_t ndefl, uintptr_t nval, int root, int nnodes,
                         uintptr_t score, uintptr_t init, uintptr_t label, uintptr_t lgy, uintptr_t weight,
                         int loss_id, float p0, float score_div, uintptr_t pred, uintptr_t loss_acc, int finish,
                         uintptr_t stream) {
  if (N <= 0) return 0;
  if (loss_id == 3 && !lgy) throw std::invalid_argument("forest_loss_regs: poisson needs lgamma(y + 1)");
  const int kf4 = (int)(xstride / 4);
  if (xstride % 4 != 0 || kf4 < 1 || kf4 > 8 || (X % 16) != 0 || nnodes <= 0 || nnodes > 2048 || loss_id < 0 ||
      loss_id > 4)
    return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // node arrays + one (4 kf4 + 1)-float row slot per thread (LDS-staged walk)
  const size_t lds = (size_t)nnodes * 5 * sizeof(int) + (size_t)256 * (4 * kf4 + 1) * sizeof(float);
  const int grid = grid_for(N, 256 * 8);
#define YTK_FLR(K, L)                                                                                       \
  hipLaunchKernelGGL((forest_loss_regs_kernel<K, L>), dim3(grid), dim3(256), lds, s, (const float*)X, N,      \
                     (const int*)nfeat, (const float*)nthr, (const int*)nleft, (const int*)nright,              \
                     (const uint8_t*)ndefl, (const float*)nval, root, nnodes, (float*)score, (const float*)init, \
                     (const float*)label, (const double*)lgy, (const float*)weight, p0, score_div, (float*)pred, \
                     (double*)loss_acc)
#define YTK_FLR_L(K)                          \
  switch (loss_id) {                          \
    case 0: YTK_FLR(K, 0); break;             \
    case 1: YTK_FLR(K, 1); break;             \
    case 2: YTK_FLR(K, 2); break;             \
    case 3: YTK_FLR(K, 3); break;             \
    default: YTK_FLR(K, 4); break;            \
  }
  switch (kf4) {
    case 1: YTK_FLR_L(1); break;
    case 2: YTK_FLR_L(2); break;
    case 3: YTK_FLR_L(3); break;
    case 4: YTK_FLR_L(4); break;
    case 5: YTK_FLR_L(5); break;
    case 6: YTK_FLR_L(6); break;
    case 7: YTK_FLR_L(7); break;
    default: YTK_FLR_L(8); break;
  }
#undef YTK_FLR_L
#undef YTK_FLR
  YTK_LAUNCH_CHECK();
  if (finish) {  // else the caller finishes the partials later (ytk_tree_grad_hist's acc2 / ytk_acc_finish)
    hipLaunchKernelGGL(acc_finish_kernel, dim3(1), dim3(256), 0, s, (double*)loss_acc, grid, (double*)nullptr,
                       (double*)nullptr, 0, (double*)nullptr);
    YTK_LAUNCH_CHECK();
  }
  return grid;  // the number of partials
}

// Ordered finish of one or two partial vectors (see acc_finish_kernel); out == 0: in place.
void ytk_acc_finish(uintptr_t loss_acc, int nblocks, uintptr_t out, uintptr_t acc2, int nblocks2, uintptr_t out2,
                    uintptr_t stream) {
  hipLaunchKernelGGL(acc_finish_kernel, dim3(acc2 ? 2 : 1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (double*)loss_acc, nblocks, (double*)out, (double*)acc2, nblocks2, (double*)out2);
  YTK_LAUNCH_CHECK();
}

// forest_predict with the row-register walk; returns 0 (nothing launched) when the layout
// does not qualify (caller then runs ytk_forest_predict).
int ytk_forest_predict_regs(uintptr_t X, long long xstride, long long N, uintptr_t nfeat, uintptr_t nthr,
                            uintptr_t nleft, uintptr_t nright, uintptr_t ndefl, uintptr_t nval, uintptr_t troot,
                            uintptr_t tout, int T, int nnodes, uintptr_t out, int ostride, float scale,
                            uintptr_t leaf_out, uintptr_t stream) {
  if (N <= 0 || T <= 0) return 1;
  const int kf4 = (int)(xstride / 4);
  if (xstride % 4 != 0 || kf4 < 1 || kf4 > 8 || (X % 16) != 0 || nnodes <= 0 || nnodes > 2048 ||
      nnodes >= (1 << 30))
    return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = (size_t)nnodes * 5 * sizeof(int);
  const dim3 grid(grid_for(N, 256 * 16));
#define YTK_FPR(K)                                                                                      \
  hipLaunchKernelGGL(forest_predict_regs_kernel<K>, grid, dim3(256), lds, s, (const float*)X, N,        \
                     (const int*)nfeat, (const float*)nthr, (const int*)nleft, (const int*)nright,          \
                     (const uint8_t*)ndefl, (const float*)nval, (const int*)troot, (const int*)tout, T,     \
                     nnodes, (float*)out, ostride, scale, (int*)leaf_out)
  switch (kf4) {
    case 1: YTK_FPR(1); break;
    case 2: YTK_FPR(2); break;
    case 3: YTK_FPR(3); break;
    case 4: YTK_FPR(4); break;
    case 5: YTK_FPR(5); break;
    case 6: YTK_FPR(6); break;
    case 7: YTK_FPR(7); break;
    default: YTK_FPR(8); break;
  }
#undef YTK_FPR
  YTK_LAUNCH_CHECK();
  return 1;
}

void ytk_bin_assign(uintptr_t X, long long xstride, long long N, int F, uintptr_t cand,
                    uintptr_t coff, uintptr_t out, int bin_bytes, long long ostride,
                    uintptr_t outT, uintptr_t stream) {
  if (N <= 0) return;
  const int grid = grid_for(N * F, 256 * 16);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int ncand = 0;
  YTK_HIP_CHECK(hipMemcpyAsync(&ncand, reinterpret_cast<const int*>(coff) + F, sizeof(int), hipMemcpyDeviceToHost, s));
  YTK_HIP_CHECK(hipStreamSynchronize(s));
  const size_t lds = ((size_t)ncand + (size_t)kBinRows * F) * sizeof(float) + (size_t)(F + 1) * sizeof(int);
  const char* lds_env = getenv("YTK_BIN_ASSIGN_LDS");  // "0": the per-element kernel
  if (bin_bytes == 1 && lds <= 64 * 1024 && !(lds_env && lds_env[0] == '0')) {
    const int g2 = (int)std::min<long long>((N + kBinRows - 1) / kBinRows, 256 * 8);
    hipLaunchKernelGGL(bin_assign_lds_kernel<uint8_t>, dim3(g2), dim3(256), lds, s, (const float*)X, xstride, N, F,
                       (const float*)cand, (const int*)coff, (uint8_t*)out, ostride, (uint8_t*)outT);
    YTK_LAUNCH_CHECK();
    return;
  }
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(bin_assign_kernel<uint8_t>, dim3(grid), dim3(256), 0, s,
                       (const float*)X, xstride, N, F, (const float*)cand, (const int*)coff,
                       (uint8_t*)out, ostride, (uint8_t*)outT);
  } else {
    hipLaunchKernelGGL(bin_assign_kernel<uint16_t>, dim3(grid), dim3(256), 0, s,
                       (const float*)X, xstride, N, F, (const float*)cand, (const int*)coff,
                       (uint16_t*)out, ostride, (uint16_t*)outT);
  }
  YTK_LAUNCH_CHECK();
}

// score [N][K], init [N][K], label [N][K], gh [K][N]; pred / ghmax optional (0)
void ytk_grad_hess(uintptr_t score, uintptr_t init, uintptr_t label, uintptr_t lgy, uintptr_t weight,
                   long long N, int K, int loss_id, float p0, float score_div, uintptr_t pred,
                   uintptr_t gh, uintptr_t loss_acc, int want_grad, uintptr_t ghmax,
                   uintptr_t stream) {
  if (N <= 0) return;
  if (loss_id == 3 && !lgy) throw std::invalid_argument("grad_hess: poisson needs lgamma(y + 1)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_for(N, 256 * 8);
  if (loss_id == 5) {
    hipLaunchKernelGGL(softmax_grad_kernel, dim3(grid), dim3(256), 0, s, (const float*)score,
                       (const float*)init, (const float*)label, (const float*)weight, N, K,
                       score_div, (float*)pred, (float2*)gh, (double*)loss_acc, want_grad,
                       (float*)ghmax);
  } else {
#define YTK_GH(LID)                                                                                \
  hipLaunchKernelGGL((tree_grad_kernel<uint8_t, 0, LID>), dim3(grid), dim3(256), 0, s,             \
                     (const uint8_t*)nullptr, 0LL, (const int*)nullptr, (const int*)nullptr,        \
                     (const int*)nullptr, (const int*)nullptr, (const float*)nullptr, 0,            \
                     (float*)score, (const float*)init, (const float*)label, (const double*)lgy,    \
                     (const float*)weight, N, loss_id, p0, score_div, (float*)pred,                 \
                     (float2*)gh, (double*)loss_acc, want_grad, (float*)ghmax, (int*)nullptr)
    switch (loss_id) {
      case 0: YTK_GH(0); break;
      case 1: YTK_GH(1); break;
      case 2: YTK_GH(2); break;
      case 3: YTK_GH(3); break;
      default: YTK_GH(4); break;
    }
#undef YTK_GH
  }
  YTK_LAUNCH_CHECK();
  hipLaunchKernelGGL(acc_finish_kernel, dim3(1), dim3(256), 0, s, (double*)loss_acc, grid, (double*)nullptr,
                     (double*)nullptr, 0, (double*)nullptr);
  YTK_LAUNCH_CHECK();
}

// Fused: score += tree(row) (row-major bins walk) then loss / grad (K == 1).
// Returns 1, or 0 (nothing launched) when the per-node leaf counts (leaf_part) do not fit in
// LDS with the node arrays -- the caller must then count leaves another way.
int ytk_tree_grad(uintptr_t bins, int bin_bytes, long long stride, uintptr_t tfeat,
                   uintptr_t tthr, uintptr_t tleft, uintptr_t tright, uintptr_t tval, int nnodes,
                   uintptr_t score, uintptr_t init, uintptr_t label, uintptr_t lgy, uintptr_t weight,
                   long long N, int loss_id, float p0, float score_div, uintptr_t pred,
                   uintptr_t gh, uintptr_t loss_acc, int want_grad, uintptr_t ghmax,
                   uintptr_t leaf_part, uintptr_t leaf_out, uintptr_t stream) {
  if (N <= 0) return 1;
  if (loss_id == 3 && !lgy) throw std::invalid_argument("tree_grad: poisson needs lgamma(y + 1)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // leaf_part (optional, >= grid * nnodes ints) + leaf_out (nnodes doubles): rows per tree
  // node -- the level engine's last-level leaf counts, taken from this walk instead of a
  // separate counting partition pass
  if (leaf_part && nnodes <= 0) leaf_part = 0;
  const size_t lds = (size_t)nnodes * (leaf_part ? 6 : 5) * sizeof(int);
  if (leaf_part && lds > kLdsBudget) return 0;
  // the node arrays alone exceed the LDS budget: walk them in global memory
  const bool nodes_global = lds > kLdsBudget;
  const int grid = grid_for(N, 256 * 8);
  const long long row_bytes = stride * bin_bytes;
  const bool aligned = (bins % 16) == 0;
  // register walk for 16/32/64-byte rows (F <= 64 uint8 features), byte loads otherwise
  const int dw = (aligned && (row_bytes == 16 || row_bytes == 32 || row_bytes == 64))
                     ? (int)(row_bytes / 4) : 0;
  // rows staged in LDS for the walk (kDw > 0): 135 -> 124 us per Higgs round (level-wise
  // 1.364 / 1.353 -> 1.350 / 1.345 ms/tree, leaf-wise 3.339 -> 3.311); YTK_TG_LDS_WALK=0: the
  // register select-chain walk
  const char* lw = getenv("YTK_TG_LDS_WALK");
  const size_t lds_rows_need = (size_t)kTreeGradRows * 256 * (dw + 1) * sizeof(uint32_t);
  // the row slots only where they fit beside the node arrays (else the select-chain walk)
  const bool lds_walk = !(lw && lw[0] == '0') && dw > 0 && !nodes_global && lds + lds_rows_need <= kLdsBudget;
  const size_t lds_rows = lds_walk ? lds_rows_need : 0;
#define YTK_TG_ONE(BT, DW, LID)                                                                   \
  do { if (lds_walk) YTK_TG_ONE2(BT, DW, LID, true); else YTK_TG_ONE2(BT, DW, LID, false); } while (0)
#define YTK_TG_ONE2(BT, DW, LID, LW)                                                              \
  hipLaunchKernelGGL((tree_grad_kernel<BT, DW, LID, LW>), dim3(grid), dim3(256), lds + ((LW) ? lds_rows : 0), s, (const BT*)bins, \
                     stride, (const int*)tfeat, (const int*)tthr, (const int*)tleft,                \
                     (const int*)tright, (const float*)tval, nnodes, (float*)score,                 \
                     (const float*)init, (const float*)label, (const double*)lgy, (const float*)weight, N, loss_id, \
                     p0, score_div, (float*)pred, (float2*)gh, (double*)loss_acc, want_grad,        \
                     (float*)ghmax, (int*)leaf_part)
#define YTK_TG_LAUNCH(BT, DW)                   \
  do {                                          \
    switch (loss_id) {                          \
      case 0: YTK_TG_ONE(BT, DW, 0); break;     \
      case 1: YTK_TG_ONE(BT, DW, 1); break;     \
      case 2: YTK_TG_ONE(BT, DW, 2); break;     \
      case 3: YTK_TG_ONE(BT, DW, 3); break;     \
      default: YTK_TG_ONE(BT, DW, 4); break;    \
    }                                           \
  } while (0)
  if (nodes_global) {
#define YTK_TG_G(BT, LID)                                                                          \
  hipLaunchKernelGGL((tree_grad_kernel<BT, 0, LID, false, true>), dim3(grid), dim3(256), 0, s, (const BT*)bins, \
                     stride, (const int*)tfeat, (const int*)tthr, (const int*)tleft,                \
                     (const int*)tright, (const float*)tval, nnodes, (float*)score,                 \
                     (const float*)init, (const float*)label, (const double*)lgy, (const float*)weight, N, loss_id, \
                     p0, score_div, (float*)pred, (float2*)gh, (double*)loss_acc, want_grad,        \
                     (float*)ghmax, (int*)nullptr)
#define YTK_TG_GL(BT)                         \
    switch (loss_id) {                        \
      case 0: YTK_TG_G(BT, 0); break;         \
      case 1: YTK_TG_G(BT, 1); break;         \
      case 2: YTK_TG_G(BT, 2); break;         \
      case 3: YTK_TG_G(BT, 3); break;         \
      default: YTK_TG_G(BT, 4); break;        \
    }
    if (bin_bytes == 1) { YTK_TG_GL(uint8_t); } else { YTK_TG_GL(uint16_t); }
#undef YTK_TG_GL
#undef YTK_TG_G
  } else if (bin_bytes == 1) {
    if (dw == 4) YTK_TG_LAUNCH(uint8_t, 4);
    else if (dw == 8) YTK_TG_LAUNCH(uint8_t, 8);
    else if (dw == 16) YTK_TG_LAUNCH(uint8_t, 16);
    else YTK_TG_LAUNCH(uint8_t, 0);
  } else {
    if (dw == 4) YTK_TG_LAUNCH(uint16_t, 4);
    else if (dw == 8) YTK_TG_LAUNCH(uint16_t, 8);
    else if (dw == 16) YTK_TG_LAUNCH(uint16_t, 16);
    else YTK_TG_LAUNCH(uint16_t, 0);
  }
#undef YTK_TG_LAUNCH
#undef YTK_TG_ONE
#undef YTK_TG_ONE2
  if (leaf_part) {  // leaf counts + the loss sums in one launch (block nnodes = acc_finish)
    hipLaunchKernelGGL(leaf_count_reduce_kernel, dim3(nnodes + 1), dim3(256), 0, s, (const int*)leaf_part, grid,
                       nnodes, (double*)leaf_out, (double*)loss_acc, (double*)nullptr, (double*)nullptr, 0,
                       (double*)nullptr);
  } else {
    hipLaunchKernelGGL(acc_finish_kernel, dim3(1), dim3(256), 0, s, (double*)loss_acc, grid, (double*)nullptr,
                     (double*)nullptr, 0, (double*)nullptr);
  }
  YTK_LAUNCH_CHECK();
  return 1;
}

void ytk_hist_reduce(uintptr_t staging, uintptr_t work, int nwork, uintptr_t hist, int B, int F, int slot_base,
                     int nslots, uintptr_t stream);

// Fused score/gradient pass + next root histogram (tree_grad_hist_kernel). Returns 0 (nothing
// launched) when the layout does not qualify; the caller then runs ytk_tree_grad and the
// root histogram separately. root_slot: the histogram slot to accumulate into (must be
// zero); staging: >= ceil(grid) * B * 32 * 16 bytes; work: >= grid int4 zeros.
int ytk_tree_grad_hist(uintptr_t bins, long long stride, uintptr_t tfeat, uintptr_t tthr, uintptr_t tleft,
                       uintptr_t tright, uintptr_t tval, int nnodes, uintptr_t score, uintptr_t init, uintptr_t label,
                       uintptr_t lgy, uintptr_t weight, long long N, int loss_id, float p0, float score_div,
                       uintptr_t pred,
                       uintptr_t gh, uintptr_t loss_acc, uintptr_t ghmax, uintptr_t leaf_part, uintptr_t leaf_out,
                       uintptr_t scales, uintptr_t staging, uintptr_t work, uintptr_t root_slot, int B, int F,
                       uintptr_t acc_out, uintptr_t acc2, int nblocks2, uintptr_t acc2_out, uintptr_t zero,
                       long long zero_n, uintptr_t stream) {
  // zero / zero_n (optional): a 16-byte aligned int64 range (the histogram slab) the kernel
  // zeroes before the root reduce adds into it
  // acc_out (optional): where the loss sums go (default loss_acc[0:2]); acc2 / nblocks2 /
  // acc2_out (optional): another pass's partials (the test-set tail) finished by the same
  // launch -- the round's sums then sit next to each other for one readback copy
  if (N <= 0 || nnodes <= 0) return 0;
  if (loss_id == 3 && !lgy) throw std::invalid_argument("tree_grad_hist: poisson needs lgamma(y + 1)");
  if (stride != 32 || (bins % 16) != 0 || B > 256 || F > 32 || loss_id < 0 || loss_id > 4) return 0;
  const size_t lds = kTGHHistBytes + (size_t)nnodes * 5 * sizeof(int) +
                     (leaf_part ? (size_t)kTGHVirtual * nnodes * sizeof(int) : 0);
  if (lds > kLdsBudget) return 0;
  if (zero && (zero % 16) != 0) return 0;
  if (zero_n <= 0) zero = 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nvb = tgh_vblocks(N);  // virtual blocks (tree_grad_kernel's grid by default)
  const int grid = (nvb + kTGHVirtual - 1) / kTGHVirtual;
#define YTK_TGH(LID) \
  do { if (tgh_rows() == 1) YTK_TGH2(LID, 1); else YTK_TGH2(LID, 2); } while (0)
#define YTK_TGH2(LID, U)                                                                                      \
  hipLaunchKernelGGL((tree_grad_hist_kernel<LID, U>), dim3(grid), dim3(kTGHThreads), lds, s, (const uint8_t*)bins, \
                     stride, (const int*)tfeat, (const int*)tthr, (const int*)tleft, (const int*)tright,         \
                     (const float*)tval, nnodes, (float*)score, (const float*)init, (const float*)label,         \
                     (const double*)lgy, (const float*)weight, N, p0, score_div, (float*)pred, (float2*)gh, (double*)loss_acc,       \
                     (float*)ghmax, (int*)leaf_part, nvb, (const float*)scales, (long long*)staging, B,    \
                     (unsigned long long*)zero, zero_n)
  switch (loss_id) {
    case 0: YTK_TGH(0); break;
    case 1: YTK_TGH(1); break;
    case 2: YTK_TGH(2); break;
    case 3: YTK_TGH(3); break;
    default: YTK_TGH(4); break;
  }
#undef YTK_TGH
#undef YTK_TGH2
  YTK_LAUNCH_CHECK();
  if (leaf_part) {
    hipLaunchKernelGGL(leaf_count_reduce_kernel, dim3(nnodes + (acc2 ? 2 : 1)), dim3(256), 0, s,
                       (const int*)leaf_part, nvb, nnodes, (double*)leaf_out, (double*)loss_acc, (double*)acc_out,
                       (double*)acc2, nblocks2, (double*)acc2_out);
  } else {
    hipLaunchKernelGGL(acc_finish_kernel, dim3(acc2 ? 2 : 1), dim3(256), 0, s, (double*)loss_acc, nvb,
                       (double*)acc_out, (double*)acc2, nblocks2, (double*)acc2_out);
  }
  YTK_LAUNCH_CHECK();
  ytk_hist_reduce(staging, work, grid, root_slot, B, F, 0, 1, stream);
  return 1;
}

// Device -> pinned host bytes as a kernel (16-B stores through the host mapping): the round's
// snapshot readback inside a captured round graph -- one graph node instead of a blit copy
// launched by the host after every replay (profiled: ~4 us copy + ~15 us of gaps per round).
__global__ __launch_bounds__(256) void copy_to_mapped_kernel(const int4* __restrict__ src, int4* __restrict__ dst,
                                                             long long n16) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n16; i += (long long)gridDim.x * 256) dst[i] = src[i];
}

void ytk_copy_to_mapped(uintptr_t dst_dev, uintptr_t src, long long nbytes, uintptr_t stream) {
  if (nbytes <= 0) return;
  if ((dst_dev | src | (uintptr_t)nbytes) & 15) throw std::invalid_argument("copy_to_mapped: 16-B aligned sizes");
  const long long n16 = nbytes / 16;
  hipLaunchKernelGGL(copy_to_mapped_kernel, dim3((unsigned)std::min<long long>((n16 + 255) / 256, 64)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const int4*)src, (int4*)dst_dev, n16);
  YTK_LAUNCH_CHECK();
}

// blocks of tree_grad_hist (staging items of its root histogram)
int ytk_tree_grad_hist_grid(long long N) { return (tgh_vblocks(N) + kTGHVirtual - 1) / kTGHVirtual; }

// tree_grad launches min(ceil(N / 256), 2048) blocks: the leaf_part scratch size
int ytk_tree_grad_grid(long long N) { return grid_for(N, 256 * 8); }

}  // extern "C"
