// Factorization machine loss/gradient kernels (gfx950 / CDNA4, wave64).
//
// Reference: J/optimizer/FMHoagOptimizer.java:60-160
//   fx(r)   = sum_i w_i x_i + 1/2 sum_f [ S_rf^2 - sum_i V_if^2 x_i^2 ],  S_rf = sum_i V_if x_i
//   g_w(i)  = sum_r c_r x_ri
//   g_V(if) = sum_r c_r x_ri (S_rf - V_if x_ri) = sum_r c_r x_ri S_rf - V_if sum_r c_r x_ri^2
// The unfused form costs five segmented products (X w, X V, (X∘X)(V∘V), X^T c, X^T(c∘S),
// (X∘X)^T c) -- six passes over the nonzeros. Here the forward is one pass over the rows
// (each V row gathered once, giving S, the square term and the linear term together) and
// the backward one pass over the CSC chunks (each S row gathered once per nonzero, giving
// the three column sums together); an ordered chunk_reduce + elementwise finish the
// gradient. Lanes map to latent index f in groups of G = pow2 >= k (<= 64), so a wave
// works on 64/G rows (or chunks) at once and the V / S row gathers are G-wide and
// contiguous. Deterministic: fixed reduction orders, no atomics.
#include "common.h"

#include <hip/hip_bf16.h>

#include <algorithm>

namespace ytk {

// Latent factors may be stored in bf16 (SGD with optimization.sgd.dtype = bf16): the
// row passes gather half the bytes; math stays fp32 and the fp32 master copy takes the
// updates (see fm_sgd_update_kernel).
__device__ __forceinline__ float ld_v(const float* p) { return *p; }
__device__ __forceinline__ float ld_v(const __hip_bfloat16* p) { return __bfloat162float(*p); }

// gathers in flight per lane group in the row / chunk walks (4 measured 3.54 ms forward,
// 4.46 ms backward per 164M-entry Criteo-shape pass)
#ifndef YTK_FM_U
#define YTK_FM_U 8
#endif
constexpr int kFmU = YTK_FM_U;

template <int G, typename VT>
__global__ __launch_bounds__(256) void fm_forward_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    long long nrows, const float* __restrict__ w, const VT* __restrict__ V, int k,
    double* __restrict__ fx, float* __restrict__ S) {
  const long long gid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / G;
  const int f = threadIdx.x & (G - 1);
  if (gid >= nrows) return;
  const long long b = indptr[gid], e = indptr[gid + 1];
  float s = 0.f, q = 0.f, lin = 0.f;
  for (long long t = b; t < e; t += G) {
    // lane f loads entry t+f, then the group walks the G entries by shuffle
    int my_i = 0;
    float my_x = 0.f;
    if (t + f < e) { my_i = idx[t + f]; my_x = val[t + f]; lin += w[my_i] * my_x; }
    const int n = (int)min<long long>(G, e - t);
    int j = 0;
    for (; j + kFmU <= n; j += kFmU) {  // kFmU independent gathers in flight
      float v[kFmU], xs[kFmU];
#pragma unroll
      for (int u = 0; u < kFmU; ++u) {
        const int i = __shfl(my_i, j + u, G);
        xs[u] = __shfl(my_x, j + u, G);
        v[u] = f < k ? ld_v(V + (long long)i * k + f) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kFmU; ++u) {
        const float vx = v[u] * xs[u];
        s += vx;
        q += vx * vx;
      }
    }
    for (; j < n; ++j) {
      const int i = __shfl(my_i, j, G);
      const float x = __shfl(my_x, j, G);
      if (f < k) {
        const float vx = ld_v(V + (long long)i * k + f) * x;
        s += vx;
        q += vx * vx;
      }
    }
  }
  double part = 0.5 * ((double)s * s - (double)q) + (double)lin;
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) part += __shfl_xor(part, off, G);
  if (f < k) S[gid * k + f] = s;
  if (f == 0) fx[gid] = part;  // (k == 0: no latent lanes, S may be null)
}

// part[chunk, 0:k] = sum c_r x S_r;  part[chunk, k] = sum c_r x;  part[chunk, k+1] = sum c_r x^2
template <int G>
__global__ __launch_bounds__(256) void fm_backward_kernel(
    const long long* __restrict__ chunk_beg, const long long* __restrict__ chunk_end, long long nch,
    const int* __restrict__ csc_rows, const float* __restrict__ csc_vals, const float* __restrict__ coef,
    const float* __restrict__ S, int k, float* __restrict__ part) {
  const long long ch = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / G;
  const int f = threadIdx.x & (G - 1);
  if (ch >= nch) return;
  const long long b = chunk_beg[ch], e = chunk_end[ch];
  float gs = 0.f, lin = 0.f, sq = 0.f;
  for (long long t = b; t < e; t += G) {
    int my_r = 0;
    float my_cx = 0.f;
    if (t + f < e) {
      my_r = csc_rows[t + f];
      const float x = csc_vals[t + f];
      my_cx = coef[my_r] * x;
      lin += my_cx;
      sq += my_cx * x;
    }
    const int n = (int)min<long long>(G, e - t);
    int j = 0;
    for (; j + kFmU <= n; j += kFmU) {  // kFmU independent gathers in flight
      float sv[kFmU], cs[kFmU];
#pragma unroll
      for (int u = 0; u < kFmU; ++u) {
        const int r = __shfl(my_r, j + u, G);
        cs[u] = __shfl(my_cx, j + u, G);
        sv[u] = f < k ? S[(long long)r * k + f] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kFmU; ++u) gs += cs[u] * sv[u];
    }
    for (; j < n; ++j) {
      const int r = __shfl(my_r, j, G);
      const float cx = __shfl(my_cx, j, G);
      if (f < k) gs += cx * S[(long long)r * k + f];
    }
  }
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) {
    lin += __shfl_xor(lin, off, G);
    sq += __shfl_xor(sq, off, G);
  }
  float* o = part + ch * (long long)(k + 2);
  if (f < k) o[f] = gs;
  if (f == 0) { o[k] = lin; o[k + 1] = sq; }
}


// Hogwild!-style SGD update for linear / FM weights (optimization.optimizer = "sgd").
// One G-lane group per row of a mini-batch (the same mapping as fm_forward, whose S = X V
// rows it reuses): after the batch's loss derivatives c_r are known, every lane f walks
// the row's entries and applies, without locks, the per-sample gradient step
//   w_i  -= lr * (c_r x_i + l2w w_i)                       (lane 0)
//   V_if -= lr * (c_r x_i (S_rf - V_if x_i) + l2v V_if)     (lane f < k)
// with no-return hardware float atomics -- concurrent rows touching the same feature
// race exactly as in Hogwild! (updates are never lost, reads may be stale). reg_skip is
// the bias index (not regularised; its latent row is frozen unless bias_latent);
// upd_w = 0 leaves all linear weights but the bias untouched (k[0] < 1).
// cnt (optional, int32 [F]): the batch's rows per feature (sgd_count_kernel); the step of a
// weight is then divided by its count -- the per-feature mean of the batch's per-sample
// gradients (optimization.sgd.average = feature): with thousands of concurrent rows per
// batch a hot feature (the bias is in every row) otherwise takes the SUM of its rows' steps
// at once and the model diverges.
template <int G>
__global__ __launch_bounds__(256) void fm_sgd_update_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    long long nrows, float* __restrict__ w, float* __restrict__ V, int k, const float* __restrict__ S,
    const float* __restrict__ c, float lr, float l2w, float l2v, int reg_skip, int upd_w, int bias_latent,
    __hip_bfloat16* __restrict__ Vb, const int* __restrict__ cnt) {
  const long long gid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / G;
  const int f = threadIdx.x & (G - 1);
  // the bias weight (reg_skip: in every row) is summed over the block and takes ONE atomic
  // per block: a device atomic per row on one address serialises the whole batch
  float bias_acc = 0.f;
  const float cr = gid < nrows ? c[gid] : 0.f;
  const long long b = cr != 0.f ? indptr[gid] : 0, e = cr != 0.f ? indptr[gid + 1] : 0;  // group-uniform
  const float s = (cr != 0.f && f < k) ? S[gid * k + f] : 0.f;
  for (long long t = b; t < e; t += G) {
    int my_i = 0;
    float my_x = 0.f;
    if (t + f < e) { my_i = idx[t + f]; my_x = val[t + f]; }
    const int n = (int)min<long long>(G, e - t);
    for (int j = 0; j < n; ++j) {
      const int i = __shfl(my_i, j, G);
      const float x = __shfl(my_x, j, G);
      const bool is_bias = i == reg_skip;
      const float lri = cnt ? lr / (float)max(1, cnt[i]) : lr;
      if (f == 0 && (upd_w || is_bias)) {
        const float gw = cr * x + (is_bias ? 0.f : l2w * w[i]);
        if (is_bias) bias_acc += -lri * gw;
        else unsafeAtomicAdd(w + i, -lri * gw);
      }
      if (f < k && (!is_bias || bias_latent)) {
        const long long o = (long long)i * k + f;
        if (Vb) {  // bf16 working copy: gradient from the value the forward used, fp32
                   // master takes the update (returning atomic), mirror re-rounded from it
          const float v = __bfloat162float(Vb[o]);
          const float gv = cr * x * (s - v * x) + (is_bias ? 0.f : l2v * v);
          const float d = -lri * gv;
          const float old = atomicAdd(V + o, d);
          Vb[o] = __float2bfloat16(old + d);  // races with other rows: Hogwild!-tolerant
        } else {
          float* vp = V + o;
          const float v = *vp;
          const float gv = cr * x * (s - v * x) + (is_bias ? 0.f : l2v * v);
          unsafeAtomicAdd(vp, -lri * gv);
        }
      }
    }
  }
  if (reg_skip >= 0) {
    __shared__ float s_bias[256 / kWave];
    bias_acc = wave_sumf(bias_acc);
    if (lane_id() == 0) s_bias[threadIdx.x / kWave] = bias_acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      float tot = 0.f;
      for (int q = 0; q < 256 / kWave; ++q) tot += s_bias[q];
      if (tot != 0.f) unsafeAtomicAdd(w + reg_skip, tot);
    }
  }
}

// Column-ordered mini-batch SGD step (optimization.optimizer = "sgd"): the batch's CSC
// (ops/sgd.py: one SparseMatrix per fixed batch row range, built once) has been reduced
// per chunk by fm_backward_kernel (part[c] = [sum c x S_f (f < k) | sum c x | sum c x^2]) and,
// for FFM, by the streamed pair-gradient kernel (lat[c] = the chunk's [nfield * k] pair
// gradient). One G-lane group per touched feature u (global id ucol[u], cnt[u] batch
// entries, chunks [ucb[u], uce[u])) sums its chunks in chunk order -- deterministic, no
// atomics, no race between the rows of a batch -- and applies the batch step with the
// weights as the batch read them:
//   w_i  -= lri * (g_i + cnt_i * l2w * w_i)
//   V_ij -= lri * (gV_ij + cnt_i * l2v * V_ij),   gV = sum c x S - V sum c x^2 (FM) | lat (FFM)
// lri = lr / cnt_i (avg: the mean of the per-sample steps of the rows holding feature i) or
// lr (the sum). FFM latents (lat != null) take the same l2 decay. reg_skip: bias index (no
// decay; latent row frozen unless bias_latent); upd_w = 0 updates only the bias among the
// linear weights. Vb (bf16 working copy read by the FM forward) and Vt ([nfield][F][k] copy
// read by the FFM backward) are rewritten from the new fp32 values of the touched entries.
template <int G>
__global__ __launch_bounds__(256) void sgd_apply_kernel(
    const int* __restrict__ ucol, const long long* __restrict__ ucb, const long long* __restrict__ uce,
    const int* __restrict__ ucnt, int nu, const float* __restrict__ part, int ldp, const float* __restrict__ lat, int J, float* __restrict__ w,
    float* __restrict__ V, int k, __hip_bfloat16* __restrict__ Vb, float* __restrict__ Vt, long long nfeat,
    float lr, float l2w, float l2v, int reg_skip, int upd_w, int bias_latent, int avg) {
  const long long gid = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / G;
  const int f = threadIdx.x & (G - 1);
  if (gid >= nu) return;
  const int i = ucol[gid];
  const long long c0 = ucb[gid], c1 = uce[gid];
  const float cnt = (float)ucnt[gid];
  const float lri = avg ? lr / fmaxf(cnt, 1.f) : lr;
  const bool is_bias = i == reg_skip;
  const int lin_col = lat ? 0 : k;  // FFM: part = [sum c x | sum c x^2]
  // chunk partials in chunk order, four loads in flight (a hot column has ~N / 64 chunks)
  float glin = 0.f, gsq = 0.f;
  long long c = c0;
  for (; c + 4 <= c1; c += 4) {
    float a[4], q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { a[u] = part[(c + u) * ldp + lin_col]; q[u] = part[(c + u) * ldp + lin_col + 1]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) { glin += a[u]; gsq += q[u]; }
  }
  for (; c < c1; ++c) {
    glin += part[c * ldp + lin_col];
    gsq += part[c * ldp + lin_col + 1];
  }
  if (f == 0 && (upd_w || is_bias)) {
    const float wi = w[i];
    w[i] = wi - lri * (glin + (is_bias ? 0.f : cnt * l2w * wi));
  }
  if (J == 0 || (is_bias && !bias_latent)) return;
  const float dec = is_bias ? 0.f : cnt * l2v;
  for (int j = f; j < J; j += G) {
    float g = 0.f;
    const long long o = (long long)i * J + j;
    const float v = V[o];
    const float* src = lat ? lat + j : part + j;
    const long long ld = lat ? J : ldp;
    long long c = c0;
    for (; c + 4 <= c1; c += 4) {
      float a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = src[(c + u) * ld];
#pragma unroll
      for (int u = 0; u < 4; ++u) g += a[u];
    }
    for (; c < c1; ++c) g += src[c * ld];
    if (!lat) g -= v * gsq;
    const float nv = v - lri * (g + dec * v);
    V[o] = nv;
    if (Vb) Vb[o] = __float2bfloat16(nv);
    if (Vt) Vt[((long long)(j / k) * nfeat + i) * k + (j % k)] = nv;
  }
}

// Rows per feature of a mini-batch (clear = 0: cnt[i] += 1 per entry) and the reset of the
// touched counters afterwards (clear = 1: plain stores of 0), over the batch's entries
// [indptr[0], indptr[nrows]) (device row pointers: no host read). Counting aggregates in
// an LDS hash table per block first (a block takes one contiguous run of entries): one
// global atomic per (block, distinct feature) instead of one per entry -- the bias is in
// every row, and 65536 same-address device atomics per batch serialise (~1 ms per batch).
// Keys that find no slot within kCntProbe probes go straight to the global counter.
constexpr int kCntSlots = 4096;
constexpr int kCntProbe = 8;
__global__ __launch_bounds__(256) void sgd_count_kernel(const long long* __restrict__ indptr,
                                                        const int* __restrict__ idx, long long nrows,
                                                        int* __restrict__ cnt, int clear) {
  const long long b = indptr[0], e = indptr[nrows];
  if (clear) {
    for (long long t = b + blockIdx.x * 256LL + threadIdx.x; t < e; t += (long long)gridDim.x * 256) cnt[idx[t]] = 0;
    return;
  }
  __shared__ int s_key[kCntSlots];
  __shared__ int s_val[kCntSlots];
  for (int i = threadIdx.x; i < kCntSlots; i += 256) {
    s_key[i] = -1;
    s_val[i] = 0;
  }
  __syncthreads();
  const long long per = (e - b + gridDim.x - 1) / gridDim.x;
  const long long r0 = b + blockIdx.x * per, r1 = min(e, r0 + per);
  for (long long t = r0 + threadIdx.x; t < r1; t += 256) {
    const int k = idx[t];
    unsigned h = ((unsigned)k * 2654435761u) >> 20;  // 12 bits: kCntSlots
    bool done = false;
    for (int p = 0; p < kCntProbe; ++p) {
      const int old = atomicCAS(&s_key[h], -1, k);
      if (old == -1 || old == k) {
        atomicAdd(&s_val[h], 1);
        done = true;
        break;
      }
      h = (h + 1) & (kCntSlots - 1);
    }
    if (!done) atomicAdd(cnt + k, 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kCntSlots; i += 256)
    if (s_key[i] >= 0) atomicAdd(cnt + s_key[i], s_val[i]);
}

}  // namespace ytk

using namespace ytk;

static int fm_group(int k) {
  int g = 4;
  while (g < k) g <<= 1;
  return g;
}

extern "C" {

// fx[r] (double) and S[r, k] for every row; w: linear weights [F], V: [F, k] (any alignment).
void ytk_fm_forward(uintptr_t indptr, uintptr_t idx, uintptr_t val, long long nrows, uintptr_t w,
                    uintptr_t V, int k, uintptr_t fx, uintptr_t S, int v_bf16, uintptr_t stream) {
  if (nrows <= 0) return;
  // k == 0: the linear score alone (S unused) -- the SGD optimizer's linear-model forward
  if (k < 0 || k > 64) throw std::invalid_argument("fm_forward: 0 <= k <= 64");
  const int G = fm_group(k);
  const long long threads = nrows * G;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_FM_F(GG)                                                                               \
  if (v_bf16)                                                                                      \
    hipLaunchKernelGGL((fm_forward_kernel<GG, __hip_bfloat16>), grid, dim3(256), 0, s,              \
                       (const long long*)indptr, (const int*)idx, (const float*)val, nrows,         \
                       (const float*)w, (const __hip_bfloat16*)V, k, (double*)fx, (float*)S);       \
  else                                                                                             \
    hipLaunchKernelGGL((fm_forward_kernel<GG, float>), grid, dim3(256), 0, s,                       \
                       (const long long*)indptr, (const int*)idx, (const float*)val, nrows,         \
                       (const float*)w, (const float*)V, k, (double*)fx, (float*)S)
  switch (G) {
    case 4: YTK_FM_F(4); break;
    case 8: YTK_FM_F(8); break;
    case 16: YTK_FM_F(16); break;
    case 32: YTK_FM_F(32); break;
    default: YTK_FM_F(64); break;
  }
#undef YTK_FM_F
  YTK_LAUNCH_CHECK();
}

// part[chunk, k + 2] column sums of the FM gradient (see kernel comment).
// k == 0: part[chunk, 2] = [sum c x | sum c x^2] only (linear gradient; S unused)
void ytk_fm_backward(uintptr_t chunk_beg, uintptr_t chunk_end, long long nch, uintptr_t csc_rows,
                     uintptr_t csc_vals, uintptr_t coef, uintptr_t S, int k, uintptr_t part,
                     uintptr_t stream) {
  if (nch <= 0) return;
  if (k < 0 || k > 64) throw std::invalid_argument("fm_backward: 0 <= k <= 64");
  const int G = fm_group(k);
  const long long threads = nch * G;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_FM_B(GG)                                                                           \
  hipLaunchKernelGGL(fm_backward_kernel<GG>, grid, dim3(256), 0, s,                            \
                     (const long long*)chunk_beg, (const long long*)chunk_end, nch,            \
                     (const int*)csc_rows, (const float*)csc_vals, (const float*)coef,         \
                     (const float*)S, k, (float*)part)
  switch (G) {
    case 4: YTK_FM_B(4); break;
    case 8: YTK_FM_B(8); break;
    case 16: YTK_FM_B(16); break;
    case 32: YTK_FM_B(32); break;
    default: YTK_FM_B(64); break;
  }
#undef YTK_FM_B
  YTK_LAUNCH_CHECK();
}

// indptr: the batch's row pointers (absolute offsets into idx / val); V / S may be null
// when k == 0 (linear model).
void ytk_fm_sgd_update(uintptr_t indptr, uintptr_t idx, uintptr_t val, long long nrows, uintptr_t w,
                       uintptr_t V, int k, uintptr_t S, uintptr_t c, float lr, float l2w, float l2v,
                       int reg_skip, int upd_w, int bias_latent, uintptr_t Vb, uintptr_t cnt, uintptr_t stream) {
  if (nrows <= 0) return;
  if (k < 0 || k > 64) throw std::invalid_argument("fm_sgd_update: 0 <= k <= 64");
  const int G = k == 0 ? 4 : fm_group(k);
  const long long threads = nrows * G;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_FM_S(GG)                                                                            \
  hipLaunchKernelGGL(fm_sgd_update_kernel<GG>, grid, dim3(256), 0, s, (const long long*)indptr, \
                     (const int*)idx, (const float*)val, nrows, (float*)w, (float*)V, k,        \
                     (const float*)S, (const float*)c, lr, l2w, l2v, reg_skip, upd_w, bias_latent,     \
                     (__hip_bfloat16*)Vb, (const int*)cnt)
  switch (G) {
    case 4: YTK_FM_S(4); break;
    case 8: YTK_FM_S(8); break;
    case 16: YTK_FM_S(16); break;
    case 32: YTK_FM_S(32); break;
    default: YTK_FM_S(64); break;
  }
#undef YTK_FM_S
  YTK_LAUNCH_CHECK();
}

// One column-ordered SGD batch step (see sgd_apply_kernel); J latent values per feature
// (FM: k, gradient folded from part; FFM: nfield * k from lat; 0: linear model). Feature u's
// chunks are [ucb[u], uce[u]) (the full touched list: ucb = ucp, uce = ucp + 1).
void ytk_sgd_apply(uintptr_t ucol, uintptr_t ucb, uintptr_t uce, uintptr_t ucnt, int nu, uintptr_t part, int ldp, uintptr_t lat,
                   int J, uintptr_t w, uintptr_t V, int k, uintptr_t Vb, uintptr_t Vt, long long nfeat, float lr,
                   float l2w, float l2v, int reg_skip, int upd_w, int bias_latent, int avg, uintptr_t stream) {
  if (nu <= 0) return;
  if (J < 0 || (J > 0 && k < 1) || (!lat && J != k) || (!lat && ldp != k + 2) || (lat && ldp != 2) ||
      (Vt && !lat))
    throw std::invalid_argument("sgd_apply: inconsistent part / latent layout");
  const int G = J <= 4 ? 4 : J <= 8 ? 8 : J <= 16 ? 16 : J <= 32 ? 32 : 64;
  const long long threads = (long long)nu * G;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_SGD_A(GG)                                                                                   \
  hipLaunchKernelGGL(sgd_apply_kernel<GG>, grid, dim3(256), 0, s, (const int*)ucol, (const long long*)ucb, \
                     (const long long*)uce, (const int*)ucnt, nu, (const float*)part, ldp, (const float*)lat, J, (float*)w,        \
                     (float*)V, k, (__hip_bfloat16*)Vb, (float*)Vt, nfeat, lr, l2w, l2v, reg_skip, upd_w,  \
                     bias_latent, avg)
  switch (G) {
    case 4: YTK_SGD_A(4); break;
    case 8: YTK_SGD_A(8); break;
    case 16: YTK_SGD_A(16); break;
    case 32: YTK_SGD_A(32); break;
    default: YTK_SGD_A(64); break;
  }
#undef YTK_SGD_A
  YTK_LAUNCH_CHECK();
}

// cnt[i] += 1 per entry of the batch rows (clear = 0) or cnt[i] = 0 for them (clear = 1).
void ytk_sgd_count(uintptr_t indptr, uintptr_t idx, long long nrows, long long nnz_hint, uintptr_t cnt, int clear,
                   uintptr_t stream) {
  if (nrows <= 0) return;
  // count: blocks of >= 4096 entries (the hash table pays off per block); clear: 256 per block
  const long long want = (std::max<long long>(nnz_hint, 1) + (clear ? 255 : 4095)) / (clear ? 256 : 4096);
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(want, clear ? 4096 : 1024));
  hipLaunchKernelGGL(sgd_count_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const long long*)indptr, (const int*)idx, nrows, (int*)cnt, clear);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"

