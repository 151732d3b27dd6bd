// Gradient-boosted soft trees (gbmlr / gbsdt / gbhmlr / gbhsdt): fused gate + expert mix +
// loss + gradient epilogue over A = X W (gfx950, wave64).
//
// Reference hot loops (one per variant, per row): J/optimizer/GBMLRHoagOptimizer.java:159-222
// (softmax gate, linear experts), GBSDTHoagOptimizer.java:135-230 (softmax gate, scalar
// leaves), GBHMLRHoagOptimizer.java:174-223 (heap-indexed sigmoid gate over any K: leaf probability =
// product of sigma(+/-) along the path, bottom-up mu sums, gate gradient
// mu_{2p} - sigma_p mu_p), GBHSDTHoagOptimizer.java:142-250.
//
// Design: the two sparse products (A = X W before, G = X^T D after) are the segmented
// SpMM kernels of sparse.hip; everything per row in between is THIS kernel. A row is worked
// by a group of G lanes (G = pow2 >= K, <= 64), lane k owning expert k (and, for the tree
// gate, internal heap node k + 1): the row's A entries are read coalesced (lane k: gate
// logit k, expert value k), the softmax max / sum and the mixture are group butterflies, a
// tree-gate leaf walks its <= 6 ancestors' sigmas by lane shuffles, and the heap sums mu[p]
// of the tree-gate gradient are formed bottom-up, one heap depth per step, in a small
// per-group LDS row (the same mu[2p] + mu[2p+1] order as the reference loop). Every lane
// holds a handful of doubles -- no per-row [K] / [2K] register arrays, so no scratch at any
// K <= 64 and a high occupancy (the round-4 thread-per-row kernel spilled 100 / 1050 VGPRs
// at K = 32 / 64 and ran one wave per SIMD at K = 16). fp64 math (the reference
// accumulates in double); every scalar loss of losses/functions.py by a loss id. One pass:
// read A row (+ z, y, weight, row mask), write the D row (the coefficients X^T multiplies)
// and pred, and reduce the loss, the random-forest loss, the expert sample masses and the
// scalar-leaf gradients per block (group butterflies -> LDS -> one fp64 atomic per value
// per block).
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace ytk {

constexpr int kGbstThreads = 256;

struct GbstArgs {
  const float* A;  // [n, lda]: gate logits [0, K-1), linear experts [K-1, 2K-1)
  int lda;
  const float* z;     // running boosting score [n]
  const float* y;     // label [n]
  const float* w;     // weight [n] (nullable -> 1)
  const uint8_t* mask;  // row sample mask [n] (nullable -> all rows)
  double inv_rate;    // 1 / instance_sample_rate (train only)
  const float* leaves;  // scalar experts [K] (gbsdt / gbhsdt)
  int n, K;
  int linear;   // 1: linear experts (A columns), 0: scalar leaves
  int loss_id;  // kLoss* below
  double lparam;  // huber delta
  int rf;       // random-forest averaging
  int T;        // trees incl. this one (rf)
  int want_grad;
  float* D;     // [n, ldd] gradient coefficients (want_grad)
  int ldd;
  float* pred;  // [n] (nullable)
  double* acc;  // [2 + 2K]: loss, rf loss, samples[K], leaf grads[K]
  const double* lgy;  // poisson: lgamma(y + 1) per row (the label term, set up once on the host:
                      // the device lgamma alone doubled this kernel's VGPRs)
};

// loss ids (ytk_learn_amd/models/gbst/model.py GBST_LOSS_IDS): the scalar losses of
// losses/functions.py (reference J/loss/*), fp64
enum { kLossSigmoid = 0, kLossL2, kLossL1, kLossHuber, kLossPoisson, kLossHinge, kLossSmoothHinge, kLossL2Hinge,
       kLossExponential, kLossMape, kLossSmape, kLossInvMape };
constexpr double kPoissonMaxZ = 30.0;
constexpr double kExpMax = 8.0;

__device__ __forceinline__ double sig_d(double x) { return 1.0 / (1.0 + exp(-x)); }
__device__ __forceinline__ double sgn_d(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); }

// poisson: without the lgamma(y + 1) label term (added from GbstArgs::lgy)
__device__ __forceinline__ double loss_val(int id, double z, double y, double lp) {
  switch (id) {
    case kLossSigmoid: return z >= 0.0 ? log1p(exp(-z)) + z * (1.0 - y) : log1p(exp(z)) - z * y;
    case kLossL2: { const double d = y - z; return 0.5 * d * d; }
    case kLossL1: return fabs(y - z);
    case kLossHuber: { const double a = fabs(z - y); return a <= lp ? 0.5 * a * a : lp * (a - 0.5 * lp); }
    case kLossPoisson: return -y * z + exp(fmin(z, kPoissonMaxZ));  // + lgamma(y + 1): GbstArgs::lgy
    case kLossHinge: return fmax(1.0 - (2.0 * y - 1.0) * z, 0.0);
    case kLossSmoothHinge: {
      const double m = (2.0 * y - 1.0) * z;
      return m <= 0.0 ? 0.5 - m : (m < 1.0 ? 0.5 * (1.0 - m) * (1.0 - m) : 0.0);
    }
    case kLossL2Hinge: { const double m = fmax(1.0 - (2.0 * y - 1.0) * z, 0.0); return 0.5 * m * m; }
    case kLossExponential: return exp(fmin(-z * (2.0 * y - 1.0), kExpMax));
    case kLossMape: return fabs((y - z) / y);
    case kLossSmape: return fabs(z - y) / ((y + fabs(z)) / 2.0);
    default: return fabs((y - z) / z);  // inv_mape
  }
}
__device__ __forceinline__ double loss_grad(int id, double z, double y, double lp) {
  switch (id) {
    case kLossSigmoid: return sig_d(z) - y;
    case kLossL2: return z - y;
    case kLossL1: return sgn_d(z - y);
    case kLossHuber: { const double a = z - y; return fabs(a) <= lp ? a : sgn_d(a) * lp; }
    case kLossPoisson: return exp(fmin(z, kPoissonMaxZ)) - y;
    case kLossHinge: { const double xl = 2.0 * y - 1.0; return xl * z < 1.0 ? -xl : 0.0; }
    case kLossSmoothHinge: {
      const double m = (2.0 * y - 1.0) * z;
      return m <= 0.0 ? 1.0 - 2.0 * y : (m < 1.0 ? (1.0 - 2.0 * y) * (1.0 - m) : 0.0);
    }
    case kLossL2Hinge: { const double xl = 2.0 * y - 1.0, m = xl * z; return m <= 1.0 ? (m - 1.0) * xl : 0.0; }
    case kLossExponential: { const double l = 2.0 * y - 1.0; return -l * exp(fmin(-z * l, kExpMax)); }
    case kLossMape: return sgn_d(z - y) / y;
    case kLossSmape: {
      const double d = (y + fabs(z)) / 2.0;
      return (sgn_d(z - y) * d - 0.5 * sgn_d(z) * fabs(z - y)) / (d * d);
    }
    default: return sgn_d((z - y) / z) * y / (z * z);  // inv_mape
  }
}
__device__ __forceinline__ double loss_pred(int id, double z) {
  if (id == kLossSigmoid) return sig_d(z);
  if (id == kLossPoisson) return exp(fmin(z, kPoissonMaxZ));
  return z;
}

template <int G>
__device__ __forceinline__ double grp_sum(double v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, G);
  return v;
}
template <int G>
__device__ __forceinline__ double grp_max(double v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, G));
  return v;
}
__device__ __forceinline__ void gbst_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int G, bool kTree>
__global__ __launch_bounds__(kGbstThreads) void gbst_epilogue_kernel(GbstArgs a) {
  constexpr int RPB = kGbstThreads / G;  // rows per block step
  constexpr int NW = kGbstThreads / kWave;
  __shared__ double s_mu[kTree ? RPB : 1][kTree ? 2 * G : 1];  // tree gate: heap sums of the group's row
  __shared__ double s_red[NW][2 + 2 * G];
  const int K = a.K;
  const int k = threadIdx.x & (G - 1);  // expert of this lane
  const int grp = threadIdx.x / G;
  const bool ek = k < K;
  // per-lane block accumulators: lane k -> samples[k], leaf grads[k]; k == 0 also the losses
  double acc_loss = 0.0, acc_rf = 0.0, acc_smp = 0.0, acc_leaf = 0.0;
  const double leaf_k = (!a.linear && ek) ? (double)a.leaves[k] : 0.0;
  // heap depth of internal node k + 1 (tree gate): floor(log2(k + 1))
  const int my_depth = 31 - __clz(k + 1);
  const long long nsteps = ((long long)a.n + RPB - 1) / RPB;
  for (long long st = blockIdx.x; st < nsteps; st += gridDim.x) {
    const long long i = st * RPB + grp;
    const bool row_ok = i < a.n;  // group-uniform
    const float* Ar = a.A + (row_ok ? i : 0) * a.lda;
    const double H = ek ? (a.linear ? (double)Ar[K - 1 + k] : leaf_k) : 0.0;
    double g = 0.0, sg = 0.0, mix = 0.0;
    if (!kTree) {  // softmax over K-1 logits + an implicit 0 logit (expert K-1)
      const double lg = k < K - 1 ? (double)Ar[k] : 0.0;
      const double mx = grp_max<G>(ek ? lg : 0.0);
      const double e = ek ? exp(lg - mx) : 0.0;
      g = e / grp_sum<G>(e);
      mix = grp_sum<G>(g * H);
    } else {  // heap-indexed sigmoid tree: prob[2p] = prob[p] sigma_p, prob[2p+1] = prob[p](1 - sigma_p)
      sg = k < K - 1 ? sig_d((double)Ar[k]) : 0.0;  // sigma of internal node k + 1
      // leaf k is heap node K + k (GBHMLRDataFlow.java:52: any K >= 2); walk to the root
      double prob = 1.0;
      int h = K + k;
#pragma unroll
      for (int d = 0; d < 7; ++d) {  // depth of heap node 2K - 1 <= 7 for K <= 64
        const int p = h >> 1;
        const double sp = __shfl(sg, (p >= 1 ? p : 1) - 1, G);
        if (h > 1) prob *= (h & 1) ? (1.0 - sp) : sp;
        h = p > 0 ? p : 1;
      }
      g = ek ? prob : 0.0;
      // heap sums: leaves, then the internal nodes one depth at a time (deepest first)
      double* mu = s_mu[grp];
      if (ek) mu[K + k] = g * H;
      gbst_wave_sync();
      const int top = 31 - __clz(K - 1 > 0 ? K - 1 : 1);  // deepest internal-node depth
      for (int dd = top; dd >= 0; --dd) {
        if (k < K - 1 && my_depth == dd) mu[k + 1] = mu[2 * (k + 1)] + mu[2 * (k + 1) + 1];
        gbst_wave_sync();
      }
      mix = mu[1];
    }
    if (row_ok) {
      const double zz = (double)a.z[i];
      const double yy = (double)a.y[i];
      const double fx = a.rf ? mix : zz + mix;
      double wt = a.w ? (double)a.w[i] : 1.0;
      const double m = a.mask ? (double)a.mask[i] : 1.0;
      if (a.mask) wt = wt * m * a.inv_rate;
      if (k == 0) {
        const double ly = a.lgy ? a.lgy[i] : 0.0;
        acc_loss += wt * (loss_val(a.loss_id, fx, yy, a.lparam) + ly);
        if (a.rf) {
          const double avg = (zz + mix) / (double)a.T;
          acc_rf += wt * (loss_val(a.loss_id, avg, yy, a.lparam) + ly);
          if (a.pred) a.pred[i] = (float)loss_pred(a.loss_id, avg);
        } else if (a.pred) {
          a.pred[i] = (float)loss_pred(a.loss_id, fx);
        }
      }
      if (a.mask) acc_smp += g * m;
      if (a.want_grad) {
        const double c = wt * loss_grad(a.loss_id, fx, yy, a.lparam);
        const double purefx = fx - zz;  // reference quirk kept: in RF mode fx excludes z
        float* Dr = a.D + i * a.ldd;
        if (k < K - 1) {
          if (!kTree) {
            Dr[k] = (float)(c * g * (H - purefx));
          } else {
            const double* mu = s_mu[grp];
            Dr[k] = (float)(c * (mu[2 * (k + 1)] - sg * mu[k + 1]));
          }
        }
        if (a.linear) {
          if (ek) Dr[K - 1 + k] = (float)(c * g);
        } else {
          acc_leaf += c * g;
        }
      }
    }
    if (kTree) gbst_wave_sync();  // the group's mu row is rewritten by its next row
  }
  // block reduction: lanes of one expert across the wave's groups, then across waves
#pragma unroll
  for (int off = G; off < kWave; off <<= 1) {
    acc_loss += __shfl_xor(acc_loss, off, kWave);
    acc_rf += __shfl_xor(acc_rf, off, kWave);
    acc_smp += __shfl_xor(acc_smp, off, kWave);
    acc_leaf += __shfl_xor(acc_leaf, off, kWave);
  }
  const int wid = threadIdx.x >> 6, l = lane_id();
  if (l < G) {
    if (l == 0) { s_red[wid][0] = acc_loss; s_red[wid][1] = acc_rf; }
    s_red[wid][2 + l] = acc_smp;
    s_red[wid][2 + G + l] = acc_leaf;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < 2 + 2 * G; v += kGbstThreads) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += s_red[q][v];
    int dst = -1;
    if (v < 2) dst = v;
    else if (v < 2 + G) { if (v - 2 < K) dst = v; }                    // samples[k]
    else if (v - 2 - G < K) dst = 2 + K + (v - 2 - G);                 // leaf grads after the K samples
    if (dst >= 0 && s != 0.0) atomicAdd(&a.acc[dst], s);
  }
}

// K > 64 (up to kGbstWideMax): ONE wave per row, lane l owning experts l + 64 j (j < KPL) in
// registers; softmax max / sums and the mixture are wave butterflies over the lanes' partials.
// The tree gate keeps the row's internal-node sigmas [K - 1] and heap sums mu [2K] in a per-wave
// LDS row (a leaf walks its <= log2(2K) ancestors' sigmas from LDS; the heap sums are formed one
// depth at a time, deepest first, the lanes striding over a depth's nodes). Same formulas and
// the same leaf-to-root product order as gbst_epilogue_kernel (sums differ from it only in
// association). Block accumulators: LDS fp64 atomics, then one global atomic per value.
constexpr int kGbstWideMax = 512;

__device__ __forceinline__ double wave_maxd(double v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
  return v;
}

template <int KPL, bool kTree>
__global__ __launch_bounds__(kGbstThreads) void gbst_epilogue_wide_kernel(GbstArgs a) {
  constexpr int NW = kGbstThreads / kWave;  // rows per block step: one per wave
  extern __shared__ __attribute__((aligned(16))) double gw_sm[];
  const int K = a.K;
  const int wid = threadIdx.x >> 6, l = lane_id();
  double* s_acc = gw_sm;                                    // [2 + 2K]: losses, samples, leaf grads
  double* s_sg = gw_sm + (2 + 2 * K) + (size_t)wid * 3 * K;  // tree gate: sigma of node p at [p - 1]
  double* s_mu = s_sg + K;                                  // tree gate: heap sums mu [2K]
  for (int v = threadIdx.x; v < 2 + 2 * K; v += kGbstThreads) s_acc[v] = 0.0;
  __syncthreads();
  double acc_loss = 0.0, acc_rf = 0.0, acc_smp[KPL], acc_leaf[KPL];
#pragma unroll
  for (int j = 0; j < KPL; ++j) acc_smp[j] = acc_leaf[j] = 0.0;
  const int top = 31 - __clz(K - 1);  // deepest internal-node depth (K - 1 >= 1)
  const long long nsteps = ((long long)a.n + NW - 1) / NW;
  for (long long st = blockIdx.x; st < nsteps; st += gridDim.x) {
    const long long i = st * NW + wid;
    if (i >= a.n) continue;  // wave-uniform
    const float* Ar = a.A + i * a.lda;
    double H[KPL], g[KPL], sg[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const int k = l + kWave * j;
      H[j] = k < K ? (a.linear ? (double)Ar[K - 1 + k] : (double)a.leaves[k]) : 0.0;
    }
    double mix;
    if (!kTree) {  // softmax over K-1 logits + an implicit 0 logit (expert K-1)
      double mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const int k = l + kWave * j;
        g[j] = k < K - 1 ? (double)Ar[k] : 0.0;  // the logit, then the gate probability
        if (k < K) mx = fmax(mx, g[j]);
      }
      mx = wave_maxd(mx);
      double es = 0.0;
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const int k = l + kWave * j;
        g[j] = k < K ? exp(g[j] - mx) : 0.0;
        es += g[j];
      }
      es = wave_sum(es);
      double m = 0.0;
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        g[j] = g[j] / es;
        m += g[j] * H[j];
      }
      mix = wave_sum(m);
    } else {  // heap-indexed sigmoid tree: leaf k is heap node K + k
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const int k = l + kWave * j;
        sg[j] = k < K - 1 ? sig_d((double)Ar[k]) : 0.0;  // sigma of internal node k + 1
        if (k < K - 1) s_sg[k] = sg[j];
      }
      gbst_wave_sync();
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const int k = l + kWave * j;
        double prob = 0.0;
        if (k < K) {
          prob = 1.0;
          for (int h = K + k; h > 1; h >>= 1) {
            const double sp = s_sg[(h >> 1) - 1];
            prob *= (h & 1) ? (1.0 - sp) : sp;
          }
          s_mu[K + k] = prob * H[j];
        }
        g[j] = prob;
      }
      gbst_wave_sync();
      for (int dd = top; dd >= 0; --dd) {  // internal nodes [2^dd, min(2^(dd+1), K)), deepest first
        const int n1 = min(2 << dd, K);
        for (int q = (1 << dd) + l; q < n1; q += kWave) s_mu[q] = s_mu[2 * q] + s_mu[2 * q + 1];
        gbst_wave_sync();
      }
      mix = s_mu[1];
    }
    const double zz = (double)a.z[i];
    const double yy = (double)a.y[i];
    const double fx = a.rf ? mix : zz + mix;
    double wt = a.w ? (double)a.w[i] : 1.0;
    const double m = a.mask ? (double)a.mask[i] : 1.0;
    if (a.mask) wt = wt * m * a.inv_rate;
    if (l == 0) {
      const double ly = a.lgy ? a.lgy[i] : 0.0;
      acc_loss += wt * (loss_val(a.loss_id, fx, yy, a.lparam) + ly);
      if (a.rf) {
        const double avg = (zz + mix) / (double)a.T;
        acc_rf += wt * (loss_val(a.loss_id, avg, yy, a.lparam) + ly);
        if (a.pred) a.pred[i] = (float)loss_pred(a.loss_id, avg);
      } else if (a.pred) {
        a.pred[i] = (float)loss_pred(a.loss_id, fx);
      }
    }
    if (a.mask) {
#pragma unroll
      for (int j = 0; j < KPL; ++j) acc_smp[j] += g[j] * m;
    }
    if (a.want_grad) {
      const double c = wt * loss_grad(a.loss_id, fx, yy, a.lparam);
      const double purefx = fx - zz;  // reference quirk kept: in RF mode fx excludes z
      float* Dr = a.D + i * a.ldd;
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const int k = l + kWave * j;
        if (k < K - 1)
          Dr[k] = kTree ? (float)(c * (s_mu[2 * (k + 1)] - sg[j] * s_mu[k + 1])) : (float)(c * g[j] * (H[j] - purefx));
        if (a.linear) {
          if (k < K) Dr[K - 1 + k] = (float)(c * g[j]);
        } else {
          acc_leaf[j] += c * g[j];
        }
      }
    }
    if (kTree) gbst_wave_sync();  // the wave's sigma / mu rows are rewritten by its next row
  }
  if (l == 0) {
    atomicAdd(&s_acc[0], acc_loss);
    atomicAdd(&s_acc[1], acc_rf);
  }
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int k = l + kWave * j;
    if (k < K) {
      if (acc_smp[j] != 0.0) atomicAdd(&s_acc[2 + k], acc_smp[j]);
      if (acc_leaf[j] != 0.0) atomicAdd(&s_acc[2 + K + k], acc_leaf[j]);
    }
  }
  __syncthreads();
  for (int v = threadIdx.x; v < 2 + 2 * K; v += kGbstThreads)
    if (s_acc[v] != 0.0) atomicAdd(&a.acc[v], s_acc[v]);
}

}  // namespace ytk

using namespace ytk;

extern "C" int ytk_gbst_wide_max() { return kGbstWideMax; }

extern "C" void ytk_gbst_epilogue(uintptr_t A, int lda, uintptr_t z, uintptr_t y, uintptr_t w, uintptr_t mask,
                                  double inv_rate, uintptr_t leaves, int n, int K, int tree_gate, int linear,
                                  int loss_id, double lparam, int rf, int T, int want_grad, uintptr_t D, int ldd,
                                  uintptr_t pred, uintptr_t acc, uintptr_t lgy, uintptr_t stream) {
  if (n <= 0) return;
  if (K < 2 || K > kGbstWideMax) throw std::invalid_argument("gbst_epilogue: 2 <= K <= 512");
  if (loss_id < kLossSigmoid || loss_id > kLossInvMape) throw std::invalid_argument("gbst_epilogue: loss id");
  if (loss_id == kLossPoisson && !lgy) throw std::invalid_argument("gbst_epilogue: poisson needs lgamma(y + 1)");
  GbstArgs a{(const float*)A, lda, (const float*)z, (const float*)y, (const float*)w, (const uint8_t*)mask,
             inv_rate, (const float*)leaves, n, K, linear, loss_id, lparam, rf, T, want_grad, (float*)D, ldd,
             (float*)pred, (double*)acc, (const double*)lgy};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_GBST(GG)                                                                                       \
  do {                                                                                                     \
    const int grid = std::min(ceil_div(n, kGbstThreads / GG), 256 * 8);                                    \
    if (tree_gate)                                                                                         \
      hipLaunchKernelGGL((gbst_epilogue_kernel<GG, true>), dim3(grid), dim3(kGbstThreads), 0, s, a);       \
    else                                                                                                   \
      hipLaunchKernelGGL((gbst_epilogue_kernel<GG, false>), dim3(grid), dim3(kGbstThreads), 0, s, a);      \
  } while (0)
#define YTK_GBSTW(KPL)                                                                                     \
  do {                                                                                                     \
    const int grid = std::min(ceil_div(n, kGbstThreads / kWave), 256 * 8);                                 \
    const size_t lds = (size_t)(2 + 2 * K) * 8 + (tree_gate ? (size_t)(kGbstThreads / kWave) * 3 * K * 8 : 0); \
    if (tree_gate)                                                                                         \
      hipLaunchKernelGGL((gbst_epilogue_wide_kernel<KPL, true>), dim3(grid), dim3(kGbstThreads), lds, s, a); \
    else                                                                                                   \
      hipLaunchKernelGGL((gbst_epilogue_wide_kernel<KPL, false>), dim3(grid), dim3(kGbstThreads), lds, s, a); \
  } while (0)
  if (K <= 2) YTK_GBST(2);
  else if (K <= 4) YTK_GBST(4);
  else if (K <= 8) YTK_GBST(8);
  else if (K <= 16) YTK_GBST(16);
  else if (K <= 32) YTK_GBST(32);
  else if (K <= 64) YTK_GBST(64);
  else if (K <= 128) YTK_GBSTW(2);
  else if (K <= 256) YTK_GBSTW(4);
  else YTK_GBSTW(8);
#undef YTK_GBST
#undef YTK_GBSTW
  YTK_LAUNCH_CHECK();
}
