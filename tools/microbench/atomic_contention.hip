// Cost of the per-chunk cursor reservation of the single-pass partition: nblk blocks each
// issue ONE returning device-scope 64-bit atomicAdd (thread 0, like partition_atomic_body)
// onto `naddr` cursors spaced `stride` u64 apart, then a dependent store of the result
// (the scatter needs it). Prints us per launch for each (blocks, addresses, stride).
//   hipcc --offload-arch=gfx950 -O3 atomic_contention.hip -o atomic_contention
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ __launch_bounds__(256) void reserve_kernel(unsigned long long* cur, int naddr, int stride,
                                                      unsigned long long* out, int chunks_per_block) {
  __shared__ unsigned long long s_base;
  for (int c = 0; c < chunks_per_block; ++c) {
    const int chunk = blockIdx.x * chunks_per_block + c;
    const int a = (int)(((long long)chunk * naddr) / ((long long)gridDim.x * chunks_per_block));  // contiguous runs
    if (threadIdx.x == 0) s_base = atomicAdd(&cur[(size_t)a * stride], 0x100000001ull);
    __syncthreads();
    if (threadIdx.x == 0) out[chunk] = s_base;
    __syncthreads();
  }
}

int main() {
  const int max_chunks = 8192;
  unsigned long long *cur, *out;
  CK(hipMalloc(&cur, sizeof(unsigned long long) * 64 * 4096));
  CK(hipMalloc(&out, sizeof(unsigned long long) * max_chunks));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int cfg_chunks[] = {641, 5127};
  const int cfg_addr[] = {1, 2, 8, 32};
  const int cfg_stride[] = {1, 16, 512};
  for (int nc : cfg_chunks)
    for (int cpb : {1, 3})
      for (int na : cfg_addr)
        for (int st : cfg_stride) {
          if (na == 1 && st != 1) continue;
          const int nblk = (nc + cpb - 1) / cpb;
          CK(hipMemset(cur, 0, sizeof(unsigned long long) * 64 * 4096));
          for (int w = 0; w < 3; ++w)
            hipLaunchKernelGGL(reserve_kernel, dim3(nblk), dim3(256), 0, 0, cur, na, st, out, cpb);
          CK(hipDeviceSynchronize());
          const int reps = 20;
          CK(hipEventRecord(e0));
          for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(reserve_kernel, dim3(nblk), dim3(256), 0, 0, cur, na, st, out, cpb);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, e0, e1));
          printf("chunks %5d  chunks/block %d  addresses %3d  stride %4d u64: %7.2f us/launch\n", nc, cpb, na, st,
                 1000.f * ms / reps);
        }
  // empty-launch reference
  CK(hipEventRecord(e0));
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(reserve_kernel, dim3(2048), dim3(256), 0, 0, cur, 1, 1, out, 0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("no atomics (2048 blocks): %7.2f us/launch\n", 1000.f * ms / 20);
  return 0;
}
