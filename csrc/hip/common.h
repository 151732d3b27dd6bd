// Shared helpers for the ytk-learn-amd HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

#define YTK_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    }                                                                              \
  } while (0)

#define YTK_LAUNCH_CHECK() YTK_HIP_CHECK(hipGetLastError())

namespace ytk {

constexpr int kWave = 64;
// dynamic LDS a kernel may request: 160 KiB per CU on gfx950, minus headroom for the
// kernels' small static __shared__ reduction scratch
constexpr size_t kLdsBudget = 160 * 1024 - 1024;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// 64-lane inclusive prefix sum (double), shuffle based.
__device__ __forceinline__ double wave_incl_scan(double v) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    double o = __shfl_up(v, off, kWave);
    if (l >= off) v += o;
  }
  return v;
}

// 64-lane inclusive max scan (int).
__device__ __forceinline__ int wave_incl_max(int v) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    int o = __shfl_up(v, off, kWave);
    if (l >= off) v = max(v, o);
  }
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ int wave_sumi(int v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace ytk
