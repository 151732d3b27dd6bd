// Histogram ablation #2 (gfx950): integer LDS accumulation + dword row loads.
// Finding of hist_ablate.hip: ds_add_f32 runs ~33x slower than ds_add_u32 on this
// pattern (2.89 ms vs 0.087 ms for 10.5M rows x 28 feats), so accumulate fixed point.
// Mapping here: lane = (row = lane/8, q = lane%8): one dword = 4 features of one row;
// step k handles feature 4q + ((k + row) & 3) -> the 32 lanes of a half-wave hit 32
// distinct banks (conflict free) while each wave-load moves 8 rows x 32 B = 256 B.
//   A: dword loads + 2 x u32 planes            (64 KiB LDS)
//   B: dword loads + 1 packed u64 plane         (64 KiB LDS) [g:int32 hi | h:uint32 lo]
//   C: dword loads + 2 x u64 planes            (128 KiB LDS)
//   D: atomics only, packed u64
//   E: dword loads only
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int T = 1024;
constexpr int U = 4;

template <int V>
__global__ __launch_bounds__(T) void hist_var(const uint8_t* __restrict__ bins, int F,
                                              const float2* __restrict__ ghp, int N, int chunk,
                                              unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long smem64[];
  unsigned* s32 = reinterpret_cast<unsigned*>(smem64);
  const int tid = threadIdx.x;
  const int nwords = (V == 0) ? 256 * 64 : (V == 2 ? 256 * 64 * 2 : 256 * 64);
  for (int i = tid; i < nwords; i += T) s32[i] = 0u;
  __syncthreads();
  const int wrow = (tid & 63) >> 3;  // row within the wave's 8
  const int q = tid & 7;
  const int wave = tid >> 6;
  const int beg = blockIdx.x * chunk;
  const int end = min(N, beg + chunk);
  constexpr int RW = (T / 64) * 8;  // rows per block step
  unsigned acc = 0;
  const float sg = 65536.f, sh = 65536.f;
  for (int base = beg + wave * 8; base < end; base += RW * U) {
    unsigned d[U];
    float2 v[U];
    bool ok[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int r = base + j * RW + wrow;
      ok[j] = r < end;
      if (V == 3) {
        unsigned h = (unsigned)r * 2654435761u + q * 40503u;
        d[j] = h;
        v[j] = make_float2((float)(h & 7) * 0.1f, 0.2f);
      } else {
        d[j] = ok[j] ? *reinterpret_cast<const unsigned*>(bins + (size_t)r * 32 + 4 * q) : 0u;
        v[j] = ok[j] ? ghp[r] : make_float2(0.f, 0.f);
      }
    }
    if (V == 4) {
#pragma unroll
      for (int j = 0; j < U; ++j) acc += d[j] + (unsigned)v[j].x;
      continue;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int gi = __float2int_rn(v[j].x * sg);
      const unsigned hi = (unsigned)__float2int_rn(v[j].y * sh);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = (k + wrow) & 3;
        const int f = 4 * q + c;
        const int bin = (d[j] >> (8 * c)) & 255;
        if (ok[j] && f < F) {
          if (V == 0) {
            atomicAdd(&s32[bin * 32 + f], (unsigned)gi);
            atomicAdd(&s32[256 * 32 + bin * 32 + f], hi);
          } else if (V == 1 || V == 3) {
            atomicAdd(&smem64[bin * 32 + f], ((unsigned long long)(unsigned)gi << 32) + hi);
          } else {
            atomicAdd(&smem64[bin * 32 + f], (unsigned long long)(long long)gi);
            atomicAdd(&smem64[256 * 32 + bin * 32 + f], (unsigned long long)hi);
          }
        }
      }
    }
  }
  __syncthreads();
  if (V == 4) {
    if (acc == 12345u) out[0] = acc;
    return;
  }
  for (int i = tid; i < 256 * 32; i += T) {
    const unsigned long long x = (V == 0) ? s32[i] : smem64[i];
    if (x) atomicAdd(&out[i], x);
  }
}

template <int V>
float run(const uint8_t* bins, const float2* gh, int N, int nblk, unsigned long long* out) {
  const int chunk = (N + nblk - 1) / nblk;
  const size_t lds = (V == 2) ? 256 * 64 * 8 : 256 * 64 * 4;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int it = 0; it < 3; ++it)
    hipLaunchKernelGGL(hist_var<V>, dim3(nblk), dim3(T), lds, 0, bins, 28, gh, N, chunk, out);
  CK(hipEventRecord(a));
  const int R = 10;
  for (int it = 0; it < R; ++it)
    hipLaunchKernelGGL(hist_var<V>, dim3(nblk), dim3(T), lds, 0, bins, 28, gh, N, chunk, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / R;
}

int main() {
  const int N = 10500000;
  uint8_t* bins;
  float2* gh;
  unsigned long long* out;
  CK(hipMalloc(&bins, (size_t)N * 32));
  CK(hipMalloc(&gh, (size_t)N * 8));
  CK(hipMalloc(&out, 256 * 64 * 8));
  std::vector<uint8_t> hb((size_t)N * 32);
  for (size_t i = 0; i < hb.size(); ++i) hb[i] = (uint8_t)((i * 2654435761u) >> 11);
  CK(hipMemcpy(bins, hb.data(), hb.size(), hipMemcpyHostToDevice));
  std::vector<float2> hg(N);
  for (int i = 0; i < N; ++i) hg[i] = make_float2((i % 7) * 0.1f - 0.3f, 0.2f);
  CK(hipMemcpy(gh, hg.data(), (size_t)N * 8, hipMemcpyHostToDevice));
  for (int nblk : {512, 1024, 2048}) {
    printf("nblk=%d  A(2xu32) %.3f ms | B(packed u64) %.3f | C(2xu64,128K) %.3f | D(u64 atom only) %.3f | E(loads only) %.3f\n",
           nblk, run<0>(bins, gh, N, nblk, out), run<1>(bins, gh, N, nblk, out),
           run<2>(bins, gh, N, nblk, out), run<3>(bins, gh, N, nblk, out), run<4>(bins, gh, N, nblk, out));
  }
  return 0;
}
