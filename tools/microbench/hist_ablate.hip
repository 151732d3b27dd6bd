// Ablation microbenchmark for the GBDT histogram kernel (gfx950).
// Variants (same grid/geometry as the production kernel, 10.5M rows x 28 feats):
//   0: production-like: loads + LDS f32 atomics
//   1: loads only (atomics replaced by register sums kept alive)
//   2: atomics only (bins derived from position hash, no global loads)
//   3: loads + LDS u32 atomics (integer add instead of float add)
//   4: loads + ds_add_f32 with one plane (g only)
//   5: atomics only, u32
// Build: hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics hist_ablate.hip -o hist_ablate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int T = 1024;
constexpr int U = 8;

template <int V>
__global__ __launch_bounds__(T) void hist_var(const uint8_t* __restrict__ bins, int stride, int F,
                                              const float2* __restrict__ ghp, int N, int chunk,
                                              float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lg = smem;
  float* lh = smem + 256 * 32;
  unsigned* ug = reinterpret_cast<unsigned*>(smem);
  unsigned* uh = reinterpret_cast<unsigned*>(smem + 256 * 32);
  const int tid = threadIdx.x;
  for (int i = tid; i < 256 * 64; i += T) smem[i] = 0.f;
  __syncthreads();
  const int hw = tid >> 5, fl = tid & 31;
  const bool active = fl < F;
  const uint8_t* bcol = bins + fl;
  const int beg = blockIdx.x * chunk;
  const int end = min(N, beg + chunk);
  float acc = 0.f;
  constexpr int HW = T / 32;
  int pos = beg + hw;
  for (; pos + HW * (U - 1) < end; pos += HW * U) {
    int b[U];
    float2 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int p = pos + HW * j;
      if (V == 2 || V == 5) {
        unsigned h = (unsigned)p * 2654435761u + fl * 40503u;
        b[j] = (h >> 13) & 255;
        v[j] = make_float2((float)(h & 7), 1.f);
      } else {
        b[j] = bcol[(size_t)p * stride];
        v[j] = ghp[p];
      }
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (V == 0 || V == 2) {
          atomicAdd(&lg[b[j] * 32 + fl], v[j].x);
          atomicAdd(&lh[b[j] * 32 + fl], v[j].y);
        } else if (V == 1) {
          acc += v[j].x * b[j] + v[j].y;
        } else if (V == 3 || V == 5) {
          atomicAdd(&ug[b[j] * 32 + fl], (unsigned)(v[j].x * 1000.f));
          atomicAdd(&uh[b[j] * 32 + fl], (unsigned)(v[j].y * 1000.f));
        } else if (V == 4) {
          atomicAdd(&lg[b[j] * 32 + fl], v[j].x + v[j].y);
        }
      }
    }
  }
  __syncthreads();
  if (V == 1) {
    if (acc == 12345.f) out[0] = acc;
    return;
  }
  for (int i = tid; i < 256 * 32; i += T) {
    const float g = lg[i];
    if (g != 0.f) atomicAdd(&out[i], g);
  }
}

template <int V>
float run(const uint8_t* bins, const float2* gh, int N, int nblk, float* out) {
  const int chunk = (N + nblk - 1) / nblk;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int it = 0; it < 3; ++it)
    hipLaunchKernelGGL(hist_var<V>, dim3(nblk), dim3(T), 256 * 64 * 4, 0, bins, 32, 28, gh, N, chunk, out);
  CK(hipEventRecord(a));
  const int R = 10;
  for (int it = 0; it < R; ++it)
    hipLaunchKernelGGL(hist_var<V>, dim3(nblk), dim3(T), 256 * 64 * 4, 0, bins, 32, 28, gh, N, chunk, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / R;
}

int main() {
  const int N = 10500000;
  uint8_t* bins;
  float2* gh;
  float* out;
  CK(hipMalloc(&bins, (size_t)N * 32));
  CK(hipMalloc(&gh, (size_t)N * 8));
  CK(hipMalloc(&out, 256 * 32 * 4));
  std::vector<uint8_t> hb((size_t)N * 32);
  for (size_t i = 0; i < hb.size(); ++i) hb[i] = (uint8_t)((i * 2654435761u) >> 11);
  CK(hipMemcpy(bins, hb.data(), hb.size(), hipMemcpyHostToDevice));
  std::vector<float2> hg(N);
  for (int i = 0; i < N; ++i) hg[i] = make_float2((i % 7) * 0.1f - 0.3f, 0.2f);
  CK(hipMemcpy(gh, hg.data(), (size_t)N * 8, hipMemcpyHostToDevice));
  for (int nblk : {512, 1024, 4096}) {
    printf("nblk=%d  v0(load+f32atom) %.3f ms | v1(load only) %.3f | v2(f32atom only) %.3f | "
           "v3(load+u32atom) %.3f | v4(load+1plane) %.3f | v5(u32atom only) %.3f\n",
           nblk, run<0>(bins, gh, N, nblk, out), run<1>(bins, gh, N, nblk, out),
           run<2>(bins, gh, N, nblk, out), run<3>(bins, gh, N, nblk, out),
           run<4>(bins, gh, N, nblk, out), run<5>(bins, gh, N, nblk, out));
  }
  return 0;
}
