// Cost of a grid-wide barrier inside one persistent kernel vs a kernel boundary on MI355X.
// 256 blocks x 1024 threads (128 KiB dynamic LDS each: one block per CU, all co-resident),
// `iters` barriers; between two barriers every block optionally writes `wbytes` and, after
// the barrier, reads (and checks) the next block's bytes -- a histogram-partial exchange. The
// barrier: release fence, one device atomic per block on a counter, the last arrival bumps a
// generation word, the others spin on it with acquire loads (all vector memory ops). Prints
// us per barrier, and us per launch of an empty kernel (the kernel-boundary alternative).
//   hipcc --offload-arch=gfx950 -O3 grid_barrier.hip -o grid_barrier
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ void grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, long long* spins) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nblocks - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long long n = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++n > (1ll << 26)) break;  // bounded: never hang the GPU (reported as spins)
      }
      if (n > (1ll << 26)) atomicAdd((unsigned long long*)spins, 1ull);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void persist_kernel(unsigned* count, unsigned* gen, int iters, int4* buf,
                                                       int wvec, long long* bad) {
  extern __shared__ int4 lds[];
  const unsigned nb = gridDim.x;
  for (int it = 0; it < iters; ++it) {
    int4* mine = buf + (size_t)blockIdx.x * wvec;
    for (int i = threadIdx.x; i < wvec; i += 1024) mine[i] = make_int4(it, blockIdx.x, i, 7);
    if (threadIdx.x == 0) lds[0] = make_int4(it, 0, 0, 0);
    grid_barrier(count, gen, nb, bad + 1);
    const int nbk = (blockIdx.x + 1) % nb;
    const int4* other = buf + (size_t)nbk * wvec;
    int errs = 0;
    for (int i = threadIdx.x; i < wvec; i += 1024) {
      const int4 v = other[i];
      errs += (v.x != it || v.y != nbk || v.z != i);
    }
    if (errs) atomicAdd((unsigned long long*)bad, (unsigned long long)errs);
    grid_barrier(count, gen, nb, bad + 1);  // nobody overwrites before every reader is done
  }
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 1;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int nb = ncu;
  unsigned *count, *gen;
  long long* bad;
  int4* buf;
  const size_t max_w = 131072 / 16;  // 128 KiB per block
  CK(hipMalloc(&count, 256));
  CK(hipMalloc(&gen, 256));
  CK(hipMalloc(&bad, 64));
  CK(hipMalloc(&buf, (size_t)nb * max_w * 16));
  CK(hipMemset(count, 0, 256));
  CK(hipMemset(gen, 0, 256));
  CK(hipFuncSetAttribute((const void*)persist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("CUs %d, blocks %d x 1024 threads, 128 KiB LDS each\n", ncu, nb);
  for (int wkb : {0, 4, 32, 128}) {
    const int wvec = wkb * 1024 / 16;
    for (int rep = 0; rep < 2; ++rep) {
      const int iters = 200;
      CK(hipMemset(bad, 0, 64));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(persist_kernel, dim3(nb), dim3(1024), 128 * 1024, 0, count, gen, iters, buf, wvec, bad);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      long long hb[2];
      CK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
      if (rep)
        printf("write %3d KiB/block: %.2f us per barrier (2 per iteration), errors %lld, timeouts %lld\n", wkb,
               1000.0 * ms / (2 * iters), hb[0], hb[1]);
    }
  }
  for (int rep = 0; rep < 2; ++rep) {
    const int n = 500;
    CK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel, dim3(nb), dim3(1024), 0, 0, (int*)nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) printf("empty kernel (%d x 1024): %.2f us per launch (stream)\n", nb, 1000.0 * ms / n);
  }
  return 0;
}
