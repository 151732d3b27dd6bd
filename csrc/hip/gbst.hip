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
// SpMM kernels of sparse.hip; everything per row in between is THIS kernel -- one thread
// per row, the K-expert mixture held in registers (kKMax = compile-time bound on K, so
// every heap / expert index is static), fp64 math (the reference accumulates in double),
// one pass: read A row (+ z, y, weight, row mask), write the D row (the gradient
// coefficients X^T multiplies) and pred, and reduce the loss, the random-forest loss,
// the expert sample masses and the scalar-leaf gradients per block (wave shuffles ->
// LDS -> one fp64 atomic per value per block). Replaces ~a dozen fp64 torch launches
// and their [n, 2K] temporaries per loss/gradient evaluation.
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
  int loss_id;  // 0 sigmoid, 1 l2
  int rf;       // random-forest averaging
  int T;        // trees incl. this one (rf)
  int want_grad;
  float* D;     // [n, ldd] gradient coefficients (want_grad)
  int ldd;
  float* pred;  // [n] (nullable)
  double* acc;  // [2 + 2K]: loss, rf loss, samples[K], leaf grads[K]
};

__device__ __forceinline__ double sig_d(double x) { return 1.0 / (1.0 + exp(-x)); }

__device__ __forceinline__ double loss_val(int id, double z, double y) {
  if (id == 0) return z >= 0.0 ? log1p(exp(-z)) + z * (1.0 - y) : log1p(exp(z)) - z * y;
  const double d = y - z;
  return 0.5 * d * d;
}
__device__ __forceinline__ double loss_grad(int id, double z, double y) {
  return id == 0 ? sig_d(z) - y : z - y;
}
__device__ __forceinline__ double loss_pred(int id, double z) { return id == 0 ? sig_d(z) : z; }

template <int kKMax, bool kTree>
__global__ __launch_bounds__(kGbstThreads) void gbst_epilogue_kernel(GbstArgs a) {
  constexpr int kVals = 2 + 2 * kKMax;
  constexpr int NW = kGbstThreads / kWave;
  __shared__ double s_red[NW][kVals];
  extern __shared__ double s_leaf[];  // tree gate, K < kKMax: [threads][kKMax] leaf probabilities
  const int K = a.K;
  double racc[kVals];
#pragma unroll
  for (int v = 0; v < kVals; ++v) racc[v] = 0.0;
  for (long long i = (long long)blockIdx.x * kGbstThreads + threadIdx.x; i < a.n;
       i += (long long)gridDim.x * kGbstThreads) {
    const float* Ar = a.A + i * a.lda;
    double g[kKMax], H[kKMax];
    double sig[kKMax];            // tree gate: sigma of internal node p at sig[p - 1]
    double mu[2 * kKMax];         // tree gate: heap node sums (mu[1] = mixture)
    double mix = 0.0;
    if (!kTree) {  // softmax over K-1 logits + an implicit 0 logit
      double mx = 0.0;
#pragma unroll
      for (int k = 0; k < kKMax - 1; ++k)
        if (k < K - 1) mx = fmax(mx, (double)Ar[k]);
      double e[kKMax], se = 0.0;
#pragma unroll
      for (int k = 0; k < kKMax; ++k) {
        e[k] = 0.0;
        if (k < K) {
          e[k] = exp((k < K - 1 ? (double)Ar[k] : 0.0) - mx);
          se += e[k];
        }
      }
#pragma unroll
      for (int k = 0; k < kKMax; ++k) g[k] = k < K ? e[k] / se : 0.0;
    } else {  // heap-indexed sigmoid tree: prob[2p] = prob[p] sigma_p, prob[2p+1] = prob[p](1 - sigma_p)
      // Heap nodes 1..2K-1 for ANY K (GBHMLRDataFlow.java:52 accepts every K >= 2): internal
      // nodes 1..K-1, expert k = node K + k. Every register index below is a compile-time
      // heap index (the unrolled loops run to kKMax, the next power of two, and test K at run
      // time); the leaves' probabilities go to expert order through this thread's LDS row
      // when K is not kKMax (node K + k is then not a static index).
      double prob[2 * kKMax];
      prob[1] = 1.0;
#pragma unroll
      for (int p = 1; p < kKMax; ++p) {
        if (p < K) {
          sig[p - 1] = sig_d((double)Ar[p - 1]);
          prob[2 * p] = prob[p] * sig[p - 1];
          prob[2 * p + 1] = prob[p] * (1.0 - sig[p - 1]);
        }
      }
      if (K == kKMax) {
#pragma unroll
        for (int k = 0; k < kKMax; ++k) g[k] = prob[kKMax + k];
      } else {
        double* gl = s_leaf + (size_t)threadIdx.x * kKMax;
#pragma unroll
        for (int h = 2; h < 2 * kKMax; ++h)
          if (h >= K && h < 2 * K) gl[h - K] = prob[h];
#pragma unroll
        for (int k = 0; k < kKMax; ++k) g[k] = k < K ? gl[k] : 0.0;
      }
#pragma unroll
      for (int h = 1; h < 2 * kKMax; ++h) {  // leaf sums mu[K + k] = g_k H_k, in heap order
        mu[h] = 0.0;
        if (h >= K && h < 2 * K)
          mu[h] = prob[h] * (a.linear ? (double)Ar[K - 1 + (h - K)] : (double)a.leaves[h - K]);
      }
#pragma unroll
      for (int p = kKMax - 1; p >= 1; --p)
        if (p < K) mu[p] = mu[2 * p] + mu[2 * p + 1];
      mix = mu[1];
    }
#pragma unroll
    for (int k = 0; k < kKMax; ++k)
      H[k] = k < K ? (a.linear ? (double)Ar[K - 1 + k] : (double)a.leaves[k]) : 0.0;
    if (!kTree) {
#pragma unroll
      for (int k = 0; k < kKMax; ++k) mix += g[k] * H[k];
    }
    const double zz = (double)a.z[i];
    const double yy = (double)a.y[i];
    const double fx = a.rf ? mix : zz + mix;
    double wt = a.w ? (double)a.w[i] : 1.0;
    const double m = a.mask ? (double)a.mask[i] : 1.0;
    if (a.mask) wt = wt * m * a.inv_rate;
    racc[0] += wt * loss_val(a.loss_id, fx, yy);
    if (a.rf) {
      const double avg = (zz + mix) / (double)a.T;
      racc[1] += wt * loss_val(a.loss_id, avg, yy);
      if (a.pred) a.pred[i] = (float)loss_pred(a.loss_id, avg);
    } else if (a.pred) {
      a.pred[i] = (float)loss_pred(a.loss_id, fx);
    }
    if (a.mask) {
#pragma unroll
      for (int k = 0; k < kKMax; ++k) racc[2 + k] += g[k] * m;
    }
    if (a.want_grad) {
      const double c = wt * loss_grad(a.loss_id, fx, yy);
      const double purefx = fx - zz;  // reference quirk kept: in RF mode fx excludes z
      float* Dr = a.D + i * a.ldd;
      if (!kTree) {
#pragma unroll
        for (int k = 0; k < kKMax - 1; ++k)
          if (k < K - 1) Dr[k] = (float)(c * g[k] * (H[k] - purefx));
      } else {
#pragma unroll
        for (int p = 1; p < kKMax; ++p)
          if (p < K) Dr[p - 1] = (float)(c * (mu[2 * p] - sig[p - 1] * mu[p]));
      }
      if (a.linear) {
#pragma unroll
        for (int k = 0; k < kKMax; ++k)
          if (k < K) Dr[K - 1 + k] = (float)(c * g[k]);
      } else {
#pragma unroll
        for (int k = 0; k < kKMax; ++k) racc[2 + kKMax + k] += c * g[k];
      }
    }
  }
  // block reduction: wave shuffles, LDS across waves, one fp64 atomic per value
  const int wid = threadIdx.x >> 6, l = lane_id();
#pragma unroll
  for (int v = 0; v < kVals; ++v) {
    const double s = wave_sum(racc[v]);
    if (l == 0) s_red[wid][v] = s;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < kVals; v += kGbstThreads) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += s_red[q][v];
    const int k = v - 2;
    int dst = v;
    if (v >= 2 + kKMax) dst = 2 + K + (v - 2 - kKMax);  // leaf grads after the K samples
    if (v < 2 || (k < kKMax && k < K) || (v >= 2 + kKMax && v - 2 - kKMax < K))
      if (s != 0.0) atomicAdd(&a.acc[dst], s);
  }
}

}  // namespace ytk

using namespace ytk;

extern "C" void ytk_gbst_epilogue(uintptr_t A, int lda, uintptr_t z, uintptr_t y, uintptr_t w, uintptr_t mask,
                                  double inv_rate, uintptr_t leaves, int n, int K, int tree_gate, int linear,
                                  int loss_id, int rf, int T, int want_grad, uintptr_t D, int ldd, uintptr_t pred,
                                  uintptr_t acc, uintptr_t stream) {
  if (n <= 0) return;
  if (K < 2 || K > 64) throw std::invalid_argument("gbst_epilogue: 2 <= K <= 64");
  GbstArgs a{(const float*)A, lda, (const float*)z, (const float*)y, (const float*)w, (const uint8_t*)mask,
             inv_rate, (const float*)leaves, n, K, linear, loss_id, rf, T, want_grad, (float*)D, ldd,
             (float*)pred, (double*)acc};
  const int grid = std::min(ceil_div(n, kGbstThreads), 256 * 8);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_GBST(KM)                                                                                   \
  do {                                                                                                 \
    const size_t lds = (tree_gate && K != KM) ? (size_t)kGbstThreads * KM * sizeof(double) : 0;       \
    if (tree_gate)                                                                                     \
      hipLaunchKernelGGL((gbst_epilogue_kernel<KM, true>), dim3(grid), dim3(kGbstThreads), lds, s, a); \
    else                                                                                               \
      hipLaunchKernelGGL((gbst_epilogue_kernel<KM, false>), dim3(grid), dim3(kGbstThreads), 0, s, a);   \
  } while (0)
  if (K <= 2) YTK_GBST(2);
  else if (K <= 4) YTK_GBST(4);
  else if (K <= 8) YTK_GBST(8);
  else if (K <= 16) YTK_GBST(16);
  else if (K <= 32) YTK_GBST(32);
  else YTK_GBST(64);
#undef YTK_GBST
  YTK_LAUNCH_CHECK();
}
