// Vector reductions for the L-BFGS/OWL-QN driver (gfx950 / CDNA4, wave64).
//
// The two-loop recursion (optim/lbfgs.py, reference J/optimizer/HoagOptimizer.java:904-929)
// and the line search need fp64 dot products of fp32 vectors of the full model dimension
// (161M for FFM on Criteo). Converting both operands to fp64 tensors costs ~8 bytes of
// traffic per byte of input; here each thread streams 16-B fp32 loads, accumulates in
// fp64, and a fixed-shape two-stage reduction (per-block partials in block order, then one
// block) makes the result bitwise reproducible.
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace ytk {

constexpr int kDotBlocks = 1024;

// mode 0: sum a*b; 1: sum a*a; 2: sum |a|
template <int kMode>
__global__ __launch_bounds__(256) void dot_partial_kernel(const float* __restrict__ a,
                                                          const float* __restrict__ b, long long n,
                                                          int vec, double* __restrict__ part) {
  double acc = 0.0;
  const long long tid = blockIdx.x * 256LL + threadIdx.x, nth = (long long)gridDim.x * 256;
  long long tail = 0;
  if (vec) {
    const long long n4 = n >> 2;
    const float4* a4 = reinterpret_cast<const float4*>(a);
    const float4* b4 = reinterpret_cast<const float4*>(b);
    for (long long i = tid; i < n4; i += nth) {
      const float4 x = a4[i];
      if (kMode == 0) {
        const float4 y = b4[i];
        acc += (double)x.x * y.x + (double)x.y * y.y + (double)x.z * y.z + (double)x.w * y.w;
      } else if (kMode == 1) {
        acc += (double)x.x * x.x + (double)x.y * x.y + (double)x.z * x.z + (double)x.w * x.w;
      } else {
        acc += (double)fabsf(x.x) + (double)fabsf(x.y) + (double)fabsf(x.z) + (double)fabsf(x.w);
      }
    }
    tail = n4 << 2;
  }
  for (long long i = tail + tid; i < n; i += nth) {
    const float x = a[i];
    acc += kMode == 0 ? (double)x * b[i] : kMode == 1 ? (double)x * x : (double)fabsf(x);
  }
  __shared__ double s[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (s[0] + s[1]) + (s[2] + s[3]);
}

__global__ __launch_bounds__(256) void dot_final_kernel(const double* __restrict__ part, int nb,
                                                        double* __restrict__ out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) acc += part[i];
  __shared__ double s[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out = (s[0] + s[1]) + (s[2] + s[3]);
}

// p <- (p + alpha * x) * scale, and the partial sums of d . p_new (the two-loop recursion's
// next dot product) in the same pass: 4 instead of 5 vector streams per step. fp32 update
// in torch's order (add, then scale); fp64 dot accumulation as dot_partial_kernel.
__global__ __launch_bounds__(256) void axpy_dot_partial_kernel(float* __restrict__ p, const float* __restrict__ x,
                                                               float alpha, float scale, const float* __restrict__ d,
                                                               long long n, int vec, double* __restrict__ part) {
  double acc = 0.0;
  const long long tid = blockIdx.x * 256LL + threadIdx.x, nth = (long long)gridDim.x * 256;
  long long tail = 0;
  auto upd = [&](float pv, float xv) { return (pv + alpha * xv) * scale; };
  if (vec) {
    const long long n4 = n >> 2;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* d4 = reinterpret_cast<const float4*>(d);
    // (a 2x unrolled variant, both groups loaded before either store: 12.7 -> 13.9 ms for
    // the 12-pair two-loop at 161M, profiles/r3s4_fused_two_loop_ab/)
    long long i = tid;
    for (; i < n4; i += nth) {
      const float4 a = p4[i], b = x4[i], c = d4[i];
      float4 r;
      r.x = upd(a.x, b.x); r.y = upd(a.y, b.y); r.z = upd(a.z, b.z); r.w = upd(a.w, b.w);
      p4[i] = r;
      acc += (double)c.x * r.x + (double)c.y * r.y + (double)c.z * r.z + (double)c.w * r.w;
    }
    tail = n4 << 2;
  }
  for (long long i = tail + tid; i < n; i += nth) {
    const float r = upd(p[i], x[i]);
    p[i] = r;
    acc += (double)d[i] * r;
  }
  __shared__ double s[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (s[0] + s[1]) + (s[2] + s[3]);
}

// Per-row loss of the single-output L-BFGS models (linear / FM / FFM: LinearHoagOptimizer.java
// :127-147): z = z0 (+ z1) in fp64, pred = f(z), c = weight * l'(z) (the transposed product's
// input) and the fp64 partial sums of weight * loss(z) -- one pass instead of ~12 fp64 torch
// elementwise launches (~340 us per 4M-row evaluation). The math is torch's fp64 formulas:
// sigmoid 1 / (1 + exp(-z)), loss log1p(exp(-|z|)) + max(z, 0) - z y written as its two branches.
// kLoss 0: sigmoid, 1: l2. The loss sum reduces in a fixed shape (bitwise reproducible).
template <int kLoss, typename TZ>
__global__ __launch_bounds__(256) void row_loss_partial_kernel(const TZ* __restrict__ z0, const float* __restrict__ z1,
                                                               const float* __restrict__ y, long long ldy,
                                                               const float* __restrict__ wt, long long n,
                                                               float* __restrict__ pred, float* __restrict__ c,
                                                               double* __restrict__ part) {
  double acc = 0.0;
  const long long tid = blockIdx.x * 256LL + threadIdx.x, nth = (long long)gridDim.x * 256;
  for (long long i = tid; i < n; i += nth) {
    const double z = (double)z0[i] + (z1 ? (double)z1[i] : 0.0);
    const double yv = (double)y[i * ldy], w = (double)wt[i];
    double lv, p, d1;
    if (kLoss == 0) {
      lv = z >= 0.0 ? log1p(exp(-z)) + z * (1.0 - yv) : log1p(exp(z)) - z * yv;
      p = 1.0 / (1.0 + exp(-z));
      d1 = p - yv;
    } else {
      const double r = yv - z;
      lv = 0.5 * (r * r);
      p = z;
      d1 = z - yv;
    }
    acc += w * lv;
    pred[i] = (float)p;
    if (c) c[i] = (float)(w * d1);
  }
  __shared__ double s[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (s[0] + s[1]) + (s[2] + s[3]);
}

// Per-row loss epilogue of the multiclass linear model (MulticlassLinearHoagOptimizer.java
// :82-149; the loss classes SoftmaxFunction.java:116-151, Multiclass{,L2,Smooth}HingeFunction,
// HSoftmaxFunction): the SpMM's fp32 scores S [n, J = K-1] with the implicit zero K-th logit,
// labels y [n, K], weights -> pred [n, K] fp32, D = weight * d1[:, :J] fp32 (the transposed
// SpMM's input) and the fixed-shape partial sums of weight * loss -- one pass instead of the
// ~15 fp64 ATen launches over n x K that the torch formulas take.
//
// One wave per block, 64 rows per tile, grid-stride over tiles. A tile's S rows and y rows are
// contiguous runs of 64*J and 64*K floats: they are staged through LDS with coalesced loads
// (odd row pitch: lane t's row walk is bank-conflict free), each lane runs its row's math from
// LDS in fp64 (torch's formulas and operation order), writes pred over its y row and D over
// its S row, and the tile leaves with coalesced stores. hsoftmax also keeps the heap's label
// sums mu [2K-1] per row in LDS (node-major, lane-minor doubles).
// kLoss 0 softmax, 1 multiclass_hinge, 2 multiclass_l2_hinge, 3 multiclass_smooth_hinge, 4 hsoftmax.
constexpr int kMcRows = 64;

template <int kLoss>
__global__ __launch_bounds__(64) void mc_row_loss_kernel(const float* __restrict__ S, int K,
                                                         const float* __restrict__ y, const float* __restrict__ wt,
                                                         long long n, float* __restrict__ pred,
                                                         float* __restrict__ D, double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double mc_sm[];
  const int J = K - 1, Jp = J | 1, Kp = K | 1, t = threadIdx.x;
  double* mu = mc_sm;                                                         // hsoftmax: [2K-1][64]
  float* sz = reinterpret_cast<float*>(mc_sm + (kLoss == 4 ? (2 * K - 1) * kMcRows : 0));  // [64][Jp]
  float* sy = sz + kMcRows * Jp;                                              // [64][Kp]
  double acc = 0.0;
  const long long tiles = (n + kMcRows - 1) / kMcRows;
  for (long long tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const long long r0 = tile * kMcRows;
    const int rows = (int)min<long long>(kMcRows, n - r0);
    __syncthreads();  // the previous tile's stores have read the LDS rows
    for (int i = t; i < rows * J; i += kMcRows) sz[(i / J) * Jp + i % J] = S[r0 * J + i];
    for (int i = t; i < rows * K; i += kMcRows) sy[(i / K) * Kp + i % K] = y[r0 * K + i];
    __syncthreads();
    if (t < rows) {
      float* z = sz + t * Jp;
      float* yr = sy + t * Kp;  // y in, pred out
      const double w = (double)wt[r0 + t];
      double lv;
      if (kLoss == 0) {
        double m = 0.0;  // the implicit K-th logit
        for (int j = 0; j < J; ++j) m = fmax(m, (double)z[j]);
        double es = 0.0, zy = 0.0;  // column order, the implicit logit last
        for (int j = 0; j < J; ++j) {
          const double zz = (double)z[j] - m;
          es += exp(zz);
          zy += zz * (double)yr[j];
        }
        es += exp(-m);
        zy += -m * (double)yr[J];
        lv = log(es) - zy;
        for (int j = 0; j < K; ++j) {
          const double zz = (j < J ? (double)z[j] : 0.0) - m;
          const float pf = (float)(exp(zz) / es);
          const double d1 = (double)pf - (double)yr[j];
          yr[j] = pf;
          if (j < J) z[j] = (float)(d1 * w);
        }
      } else if (kLoss <= 3) {
        int tg = -1;  // the last class whose label is exactly 1.0
        for (int j = 0; j < K; ++j)
          if (yr[j] == 1.0f) tg = j;
        if (tg < 0) {
          lv = __builtin_nan("");  // no target class: the reference throws; the loss sum says so
          tg = K - 1;
        } else {
          lv = 0.0;
        }
        const double zt = tg < J ? (double)z[tg] : 0.0;
        double dsum = 0.0, lsum = 0.0;
        for (int j = 0; j < K; ++j) {
          const double zj = j < J ? (double)z[j] : 0.0;
          const double dd = zj - zt;
          double d, l;
          if (kLoss == 1) {
            const double mg = dd + 1.0;
            l = fmax(mg, 0.0);
            d = mg > 0.0 ? 1.0 : 0.0;
          } else if (kLoss == 2) {
            const double mg = fmax(dd + 1.0, 0.0);
            l = mg * mg;
            d = mg;
          } else {
            l = dd >= 0.0 ? dd + 0.5 : (dd < -1.0 ? 0.0 : 0.5 * ((1.0 + dd) * (1.0 + dd)));
            d = dd >= 0.0 ? 1.0 : (dd < -1.0 ? 0.0 : 1.0 + dd);
          }
          lsum += l;
          dsum += d;
          yr[j] = (float)zj;
          if (j < J && j != tg) z[j] = (float)(d * w);
        }
        if (tg < J) z[tg] = (float)((-dsum + 1.0) * w);
        lv += kLoss == 1 ? lsum - 1.0 : kLoss == 2 ? 0.5 * (lsum - 1.0) : lsum - 0.5;
      } else {
        // heap of 2K-1 nodes: internal j < K-1 has logit z[j], leaf g is node K-1+g
        for (int g = 0; g < K; ++g) mu[(J + g) * kMcRows + t] = (double)yr[g];
        for (int j = J - 1; j >= 0; --j)
          mu[j * kMcRows + t] = mu[(2 * j + 1) * kMcRows + t] + mu[(2 * j + 2) * kMcRows + t];
        for (int g = 0; g < K; ++g) {  // leaf probability, bottom-up (torch's product order)
          double p = 1.0;
          int prev = g + K;
          while (true) {
            const int cur = prev >> 1;
            const double gx = 1.0 / (1.0 + exp(-(double)z[cur - 1]));
            p = p * ((prev & 1) == 0 ? gx : 1.0 - gx);
            prev = cur;
            if (cur == 1) break;
          }
          yr[g] = (float)p;
        }
        lv = 0.0;
        for (int j = 0; j < J; ++j) {
          const double s = (double)z[j];
          const double mp = mu[j * kMcRows + t], ml = mu[(2 * j + 1) * kMcRows + t],
                       mr = mu[(2 * j + 2) * kMcRows + t];
          lv += s >= 0.0 ? mr * s + mp * log1p(exp(-s)) : mp * log1p(exp(s)) - ml * s;
          const double gx = 1.0 / (1.0 + exp(-s));
          z[j] = (float)((gx * mp - ml) * w);
        }
      }
      acc += w * lv;
    }
    __syncthreads();
    for (int i = t; i < rows * K; i += kMcRows) pred[r0 * K + i] = sy[(i / K) * Kp + i % K];
    if (D)
      for (int i = t; i < rows * J; i += kMcRows) D[r0 * J + i] = sz[(i / J) * Jp + i % J];
  }
  acc = wave_sum(acc);
  if (t == 0) part[blockIdx.x] = acc;
}

}  // namespace ytk

using namespace ytk;

extern "C" {

// *out (fp64, device) = reduction of a (and b) per mode; part: >= 1024 doubles of scratch.
void ytk_dot(uintptr_t a, uintptr_t b, long long n, int mode, uintptr_t part, uintptr_t out,
             uintptr_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vec = ((a | (mode == 0 ? b : 0)) & 15) == 0;
  long long want = (n / 4 + 255) / 256;
  const int nb = (int)std::max<long long>(1, std::min<long long>(kDotBlocks, want));
  switch (mode) {
    case 0: hipLaunchKernelGGL(dot_partial_kernel<0>, dim3(nb), dim3(256), 0, s, (const float*)a,
                               (const float*)b, n, vec, (double*)part); break;
    case 1: hipLaunchKernelGGL(dot_partial_kernel<1>, dim3(nb), dim3(256), 0, s, (const float*)a,
                               (const float*)b, n, vec, (double*)part); break;
    default: hipLaunchKernelGGL(dot_partial_kernel<2>, dim3(nb), dim3(256), 0, s, (const float*)a,
                                (const float*)b, n, vec, (double*)part); break;
  }
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(256), 0, s, (const double*)part, nb,
                     (double*)out);
  YTK_LAUNCH_CHECK();
}

// p <- (p + alpha * x) * scale; *out (fp64, device) = d . p_new. part: >= 1024 doubles.
void ytk_axpy_dot(uintptr_t p, uintptr_t x, float alpha, float scale, uintptr_t d, long long n, uintptr_t part,
                  uintptr_t out, uintptr_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vec = ((p | x | d) & 15) == 0;
  long long want = (n / 4 + 255) / 256;
  const int nb = (int)std::max<long long>(1, std::min<long long>(kDotBlocks, want));
  hipLaunchKernelGGL(axpy_dot_partial_kernel, dim3(nb), dim3(256), 0, s, (float*)p, (const float*)x, alpha, scale,
                     (const float*)d, n, vec, (double*)part);
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(256), 0, s, (const double*)part, nb, (double*)out);
  YTK_LAUNCH_CHECK();
}

// Fused per-row loss (row_loss_partial_kernel): z0 fp32 (z64 = 0) or fp64 (z64 = 1), z1
// optional fp32 addend, y strided by ldy, wt fp32; pred / c fp32 [n] (c optional); *out (fp64,
// device) = sum weight * loss. part: >= 1024 doubles. loss: 0 sigmoid, 1 l2.
void ytk_row_loss(int loss, uintptr_t z0, int z64, uintptr_t z1, uintptr_t y, long long ldy, uintptr_t wt, long long n,
                  uintptr_t pred, uintptr_t c, uintptr_t part, uintptr_t out, uintptr_t stream) {
  if (loss < 0 || loss > 1) throw std::invalid_argument("row_loss: unsupported loss id");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = (int)std::max<long long>(1, std::min<long long>(kDotBlocks, (n + 1023) / 1024));
#define YTK_RL(L, T)                                                                                            \
  hipLaunchKernelGGL((row_loss_partial_kernel<L, T>), dim3(nb), dim3(256), 0, s, (const T*)z0, (const float*)z1, \
                     (const float*)y, ldy, (const float*)wt, n, (float*)pred, (float*)c, (double*)part)
  if (loss == 0) {
    if (z64) YTK_RL(0, double); else YTK_RL(0, float);
  } else {
    if (z64) YTK_RL(1, double); else YTK_RL(1, float);
  }
#undef YTK_RL
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(256), 0, s, (const double*)part, nb, (double*)out);
  YTK_LAUNCH_CHECK();
}

// Multiclass loss epilogue (mc_row_loss_kernel): S fp32 [n, K-1], y fp32 [n, K], wt fp32 [n] ->
// pred fp32 [n, K], D fp32 [n, K-1] (optional); *out (fp64, device) = sum weight * loss.
// part: >= max_blocks doubles. loss: 0 softmax, 1 multiclass_hinge, 2 multiclass_l2_hinge,
// 3 multiclass_smooth_hinge, 4 hsoftmax. 2 <= K <= 64.
void ytk_mc_row_loss(int loss, uintptr_t S, int K, uintptr_t y, uintptr_t wt, long long n, uintptr_t pred, uintptr_t D,
                     uintptr_t part, int max_blocks, uintptr_t out, uintptr_t stream) {
  if (loss < 0 || loss > 4) throw std::invalid_argument("mc_row_loss: unsupported loss id");
  if (K < 2 || K > 64) throw std::invalid_argument("mc_row_loss: K must be in [2, 64]");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const long long tiles = (n + kMcRows - 1) / kMcRows;
  const int nb = (int)std::max<long long>(1, std::min<long long>(max_blocks, tiles));
  const size_t lds = (size_t)(loss == 4 ? (2 * K - 1) * kMcRows * 8 : 0) +
                     (size_t)kMcRows * (((K - 1) | 1) + (K | 1)) * 4;
#define YTK_MC(L)                                                                                          \
  hipLaunchKernelGGL(mc_row_loss_kernel<L>, dim3(nb), dim3(kMcRows), lds, s, (const float*)S, K,         \
                     (const float*)y, (const float*)wt, n, (float*)pred, (float*)D, (double*)part)
  switch (loss) {
    case 0: YTK_MC(0); break;
    case 1: YTK_MC(1); break;
    case 2: YTK_MC(2); break;
    case 3: YTK_MC(3); break;
    default: YTK_MC(4); break;
  }
#undef YTK_MC
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(256), 0, s, (const double*)part, nb, (double*)out);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
