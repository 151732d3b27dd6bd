// MFMA histogram microbenchmark ("settle MFMA with measurements").
//
// The GBDT histogram (J/data/gbdt/HistogramBuilder.java:56-90) written as a matrix product:
//   hist_f[bin][c] = sum_rows onehot(bin_f(row) == bin) * limb_c(row)
// with the exact fixed-point (g, h) split into 8-bit limbs (bf16 holds 0..255 exactly, the
// fp32 accumulator is exact below 2^24 = 65k rows of 255), recombined afterwards. One wave
// owns one feature's 256-bin x 32-column histogram in 8 accumulator tiles of
// v_mfma_f32_32x32x16_bf16 (128 fp32 per lane) and walks the rows 16 at a time:
//   A (16 rows x 32 bins of a tile)  = one-hot built from the 16 bins with VALU compares
//   B (16 rows x 32 columns)         = the rows' limbs (g: 5 bytes of qg + 2^39, h: 5 bytes
//                                      of qh, col 10 = 1 -> the row count)
// 8 MFMAs per 16 rows per feature: 28 features x 10.5M rows = 147M MFMAs of 32K flop =
// 4.8 PFLOP of which 1/256 are non-zero products. Kernel B is the production LDS-atomic
// kernel's algorithm reduced to the same output for a same-machine comparison.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/microbench/mfma_hist.hip -o /tmp/mfma_hist
// Run:   /tmp/mfma_hist [rows]   (validates both kernels bit-exactly on a small case first)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);             \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kF = 28, kStride = 32, kB = 256, kCols = 32, kLimbs = 5;

// limbs of row r: cols 0..4 = bytes of (qg + 2^39), 5..9 = bytes of qh, 10 = 1
__device__ __forceinline__ float limb(long long qg, long long qh, int col) {
  if (col < kLimbs) return (float)(((unsigned long long)(qg + (1ll << 39)) >> (8 * col)) & 255);
  if (col < 2 * kLimbs) return (float)(((unsigned long long)qh >> (8 * (col - kLimbs))) & 255);
  return col == 2 * kLimbs ? 1.f : 0.f;
}

// grid = (row chunks, kF); one wave per block; chunk of rows <= 65536 (fp32-exact sums)
__global__ __launch_bounds__(64) void mfma_hist_kernel(const uint8_t* __restrict__ bins, const long long* __restrict__ q,
                                                       int n, int chunk, float* __restrict__ out /* [chunks][kF][kB][kCols] */) {
  const int f = blockIdx.y;
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  for (int base = beg; base < end; base += 16) {
    int bn[8];
    bf16x8 bfrag;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = base + 8 * h + j;
      const bool ok = row < end;
      bn[j] = ok ? bins[(size_t)row * kStride + f] : -1;
      const long long qg = ok ? q[2 * (size_t)row] : 0, qh = ok ? q[2 * (size_t)row + 1] : 0;
      bfrag[j] = (__bf16)(ok ? limb(qg, qh, r) : 0.f);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      bf16x8 afrag;
#pragma unroll
      for (int j = 0; j < 8; ++j) afrag[j] = (__bf16)(bn[j] == t * 32 + r ? 1.f : 0.f);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afrag, bfrag, acc[t], 0, 0, 0);
    }
  }
  // C/D map (32x32): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
  float* o = out + ((size_t)blockIdx.x * kF + f) * kB * kCols;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
      o[(t * 32 + row) * kCols + r] = acc[t][i];
    }
}

// reference LDS-atomic histogram (the production algorithm, int64 g / h planes)
__global__ __launch_bounds__(1024) void lds_hist_kernel(const uint8_t* __restrict__ bins, const long long* __restrict__ q,
                                                        int n, int chunk, long long* __restrict__ out /* [kF][kB][2] */) {
  __shared__ unsigned long long lg[kB * 32], lh[kB * 32];
  for (int i = threadIdx.x; i < kB * 32; i += 1024) lg[i] = lh[i] = 0;
  __syncthreads();
  const int beg = blockIdx.x * chunk, end = min(n, beg + chunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wr = lane >> 3, qd = lane & 7;
  for (int row = beg + wave * 8 + wr; row < end; row += 128) {
    const unsigned d = *reinterpret_cast<const unsigned*>(bins + (size_t)row * kStride + 4 * qd);
    const unsigned long long g = q[2 * (size_t)row], hh = q[2 * (size_t)row + 1];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int b = (d >> (8 * c)) & 255;
      atomicAdd(&lg[b * 32 + 4 * qd + c], g);
      atomicAdd(&lh[b * 32 + 4 * qd + c], hh);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kB * 32; i += 1024) {
    const int b = i >> 5, ff = i & 31;
    if (ff < kF && (lg[i] | lh[i])) {
      atomicAdd((unsigned long long*)&out[(ff * kB + b) * 2], lg[i]);
      atomicAdd((unsigned long long*)&out[(ff * kB + b) * 2 + 1], lh[i]);
    }
  }
}

int main(int argc, char** argv) {
  const int n_big = argc > 1 ? atoi(argv[1]) : 10500000;
  for (int pass = 0; pass < 2; ++pass) {
    const int n = pass == 0 ? 20000 : n_big;
    std::vector<uint8_t> hb((size_t)n * kStride, 0);
    std::vector<long long> hq(2 * (size_t)n);
    uint64_t s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (int i = 0; i < n; ++i) {
      for (int f = 0; f < kF; ++f) hb[(size_t)i * kStride + f] = (uint8_t)(rnd() % 255);
      hq[2 * i] = (long long)(rnd() % (1ull << 36)) - (1ll << 35);
      hq[2 * i + 1] = (long long)(rnd() % (1ull << 34));
    }
    uint8_t* db;
    long long* dq;
    CK(hipMalloc(&db, hb.size()));
    CK(hipMalloc(&dq, hq.size() * 8));
    CK(hipMemcpy(db, hb.data(), hb.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dq, hq.data(), hq.size() * 8, hipMemcpyHostToDevice));
    const int chunk = 16384;  // 16k rows x 255 < 2^24: exact fp32 sums
    const int nch = (n + chunk - 1) / chunk;
    float* dout;
    CK(hipMalloc(&dout, (size_t)nch * kF * kB * kCols * 4));
    long long* dl;
    CK(hipMalloc(&dl, (size_t)kF * kB * 2 * 8));
    CK(hipMemset(dl, 0, (size_t)kF * kB * 2 * 8));
    const int lchunk = (n + 255) / 256;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms_m = 0, ms_l = 0;
    const int reps = pass == 0 ? 1 : 5;
    for (int it = 0; it < reps + (pass ? 1 : 0); ++it) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(mfma_hist_kernel, dim3(nch, kF), dim3(64), 0, 0, db, dq, n, chunk, dout);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (it > 0 || pass == 0) ms_m += t;
      CK(hipMemset(dl, 0, (size_t)kF * kB * 2 * 8));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(lds_hist_kernel, dim3(256), dim3(1024), 0, 0, db, dq, n, lchunk, dl);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t, e0, e1));
      if (it > 0 || pass == 0) ms_l += t;
    }
    if (pass == 0) {  // exactness: recombine the limbs and compare with the int64 kernel and the CPU
      std::vector<float> ho((size_t)nch * kF * kB * kCols);
      std::vector<long long> hl((size_t)kF * kB * 2), ref((size_t)kF * kB * 2, 0), cnt((size_t)kF * kB, 0);
      CK(hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hl.data(), dl, hl.size() * 8, hipMemcpyDeviceToHost));
      for (int i = 0; i < n; ++i)
        for (int f = 0; f < kF; ++f) {
          const int b = hb[(size_t)i * kStride + f];
          ref[(f * kB + b) * 2] += hq[2 * i];
          ref[(f * kB + b) * 2 + 1] += hq[2 * i + 1];
          cnt[f * kB + b] += 1;
        }
      long long bad = 0;
      for (int f = 0; f < kF; ++f)
        for (int b = 0; b < kB; ++b) {
          long long g = 0, hh = 0, c = 0;
          for (int ch = 0; ch < nch; ++ch) {
            const float* o = &ho[(((size_t)ch * kF + f) * kB + b) * kCols];
            for (int L = 0; L < kLimbs; ++L) {
              g += (long long)o[L] << (8 * L);
              hh += (long long)o[kLimbs + L] << (8 * L);
            }
            c += (long long)o[2 * kLimbs];
          }
          g -= c << 39;  // undo the per-row offset
          bad += (g != ref[(f * kB + b) * 2]) + (hh != ref[(f * kB + b) * 2 + 1]) + (c != cnt[f * kB + b]);
          bad += (hl[(f * kB + b) * 2] != ref[(f * kB + b) * 2]) + (hl[(f * kB + b) * 2 + 1] != ref[(f * kB + b) * 2 + 1]);
        }
      printf("validation n=%d: mismatches=%lld\n", n, bad);
      if (bad) return 2;
    } else {
      const double mfma_tf = 2.0 * 32 * 32 * 16 * 8.0 * ((n + 15) / 16) * kF / (ms_m / reps * 1e-3) / 1e12;
      printf("rows=%d features=%d bins=%d: mfma(bf16 one-hot x limbs) %.3f ms (%.0f dense TFLOP/s), "
             "lds-atomic int64 %.3f ms\n", n, kF, kB, ms_m / reps, mfma_tf, ms_l / reps);
    }
    CK(hipFree(db));
    CK(hipFree(dq));
    CK(hipFree(dout));
    CK(hipFree(dl));
  }
  return 0;
}
