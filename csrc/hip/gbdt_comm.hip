// Histogram-sync helpers of the multi-GPU tree engines (gfx950).
//
// Reference: J/data/gbdt/HistogramBuilder.java:95 -- reduceScatterArray of the level's
// histograms by feature ownership (GBDTDataFlow.java:252-272 assigns each worker a
// contiguous feature range), plus the per-level child-count allreduce
// (DataParallelTreeMaker.java:518,538).
//
// Owner-computes sync: the level's built slots are [slot][bin][F][2] int64; rank r owns
// features [r*fr, min(F, (r+1)*fr)). A reduce-scatter needs the P feature blocks as P
// contiguous chunks, so ONE pack kernel writes x[r] = (the slots' block-r columns, zero
// padded to fr, then the level's count words, replicated into every chunk) into a
// persistent buffer, and ONE unpack kernel scatters this rank's reduced chunk back
// (instead of a zero fill plus one strided copy per rank every level).
#include "common.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace ytk {

// i in [0, P * (nb + C)): chunk r = i / (nb + C); inside a chunk, element
// ((slot * B + bin) * fr + fl) * 2 + c of the block, then the C count words.
__global__ __launch_bounds__(256) void owner_pack_kernel(const long long* __restrict__ hist, long long* __restrict__ x,
                                                         int nslots, int B, int F, int fr, int P,
                                                         const long long* __restrict__ cnt, int C) {
  const long long nb = (long long)nslots * B * fr * 2;
  const long long per = nb + C;
  const long long total = per * P;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / per);
    const long long j = i - (long long)r * per;
    long long v = 0;
    if (j < nb) {
      const int c = (int)(j & 1);
      const long long e = j >> 1;  // (slot * B + bin) * fr + fl
      const int fl = (int)(e % fr);
      const long long sb = e / fr;  // slot * B + bin
      const int f = r * fr + fl;
      if (f < F) v = hist[(sb * F + f) * 2 + c];
    } else {
      v = cnt[j - nb];
    }
    x[i] = v;
  }
}

__global__ __launch_bounds__(256) void owner_unpack_kernel(const long long* __restrict__ out, long long* __restrict__ hist,
                                                           int nslots, int B, int F, int fr, int rank,
                                                           long long* __restrict__ cnt, int C) {
  const long long nb = (long long)nslots * B * fr * 2;
  const long long total = nb + C;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < total;
       j += (long long)gridDim.x * blockDim.x) {
    if (j < nb) {
      const int c = (int)(j & 1);
      const long long e = j >> 1;
      const int fl = (int)(e % fr);
      const long long sb = e / fr;
      const int f = rank * fr + fl;
      if (f < F) hist[(sb * F + f) * 2 + c] = out[j];
    } else {
      cnt[j - nb] = out[j];
    }
  }
}

static inline int grid_of(long long n) { return (int)std::min<long long>((n + 255) / 256, 256 * 8); }

}  // namespace ytk

using namespace ytk;

extern "C" {

// hist: the first of the nslots slots (slot stride B * F * 2 int64); cnt: C count words
// (0 when none); x: P * (nslots * B * fr * 2 + C) int64.
void ytk_owner_pack(uintptr_t hist, uintptr_t x, int nslots, int B, int F, int fr, int P, uintptr_t cnt, int C,
                    uintptr_t stream) {
  const long long total = ((long long)nslots * B * fr * 2 + C) * P;
  if (total <= 0) return;
  hipLaunchKernelGGL(owner_pack_kernel, dim3(grid_of(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const long long*)hist, (long long*)x, nslots, B, F, fr, P, (const long long*)cnt, C);
  YTK_LAUNCH_CHECK();
}

void ytk_owner_unpack(uintptr_t out, uintptr_t hist, int nslots, int B, int F, int fr, int rank, uintptr_t cnt, int C,
                      uintptr_t stream) {
  const long long total = (long long)nslots * B * fr * 2 + C;
  if (total <= 0) return;
  hipLaunchKernelGGL(owner_unpack_kernel, dim3(grid_of(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const long long*)out, (long long*)hist, nslots, B, F, fr, rank, (long long*)cnt, C);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"

// ------------------------------------------------------------------ one-shot peer reduce
// Latency-optimised histogram all-reduce over peer memory (xGMI), behind YTK_PEER_REDUCE=1.
// RCCL stays the default until this path is measured on 8 GPUs.
//
// Each rank owns ONE uncached device allocation (hipDeviceMallocUncached: loads and stores
// bypass every cache level, so data handed between processes never meets a stale L2 line on
// any XCD) = [signal words | send slab | recv slab], exported with hipIpcGetMemHandle and
// opened by every other rank. One all-reduce of n int64 (the level's histogram slots +
// count words) is five launches on the compute stream, no host involvement:
//   pack      local: send <- hist
//   barrier   every rank stamps its epoch into every peer's signal word [rank] (system-scope
//             release), then waits until all P words of its own signal array reach the epoch
//   reduce    rank r sums chunk r of all P send slabs (exact int64, rank order) and stores the
//             sum into chunk r of every rank's recv slab (two-shot: reduce-scatter by reads,
//             all-gather by writes; each chunk has exactly one writer)
//   barrier   (next epoch)
//   unpack    local: hist <- recv
// Barrier waits are bounded: a wait that outlives its budget raises an error word (checked by
// the host) and exits, so a missing peer can never hang the GPU.
namespace ytk {
constexpr int kPeerMax = 16;
constexpr int kSigWords = 64;  // int64 signal words (one per rank, 512 B)

struct PeerPtrs {
  long long* send[kPeerMax];
  long long* recv[kPeerMax];
  unsigned long long* sig[kPeerMax];
};

__global__ __launch_bounds__(64) void peer_barrier_kernel(PeerPtrs pp, int P, int rank, unsigned long long epoch,
                                                          int* __restrict__ err, long long max_spins) {
  const int t = threadIdx.x;
  __threadfence_system();  // this rank's earlier stores (previous kernels) are visible first
  if (t < P)
    __hip_atomic_store(pp.sig[t] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < P) {
    const unsigned long long* mine = pp.sig[rank] + t;
    long long spins = 0;
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(4);
      if (++spins > max_spins) {
        atomicExch(err, 1);
        break;
      }
    }
  }
  __threadfence_system();
}

__global__ __launch_bounds__(256) void peer_copy_kernel(const long long* __restrict__ src, long long* __restrict__ dst,
                                                        long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void peer_reduce_kernel(PeerPtrs pp, int P, int rank, long long n) {
  const long long lo = n * rank / P, hi = n * (rank + 1) / P;
  for (long long i = lo + blockIdx.x * 256LL + threadIdx.x; i < hi; i += (long long)gridDim.x * 256) {
    long long s = 0;
#pragma unroll 4
    for (int q = 0; q < P; ++q) s += __builtin_nontemporal_load(pp.send[q] + i);
    for (int q = 0; q < P; ++q) __builtin_nontemporal_store(s, pp.recv[q] + i);
  }
}

struct PeerGroup {
  int P = 0, rank = 0;
  long long cap = 0;  // int64 elements per slab
  char* base = nullptr;  // own allocation
  std::vector<void*> opened;
  PeerPtrs pp{};
  int* err = nullptr;  // device error word (fine to be ordinary device memory)
  unsigned long long epoch = 0;
};
}  // namespace ytk
static std::vector<ytk::PeerGroup> g_peer;
namespace ytk {

static size_t peer_bytes(long long cap) { return (size_t)kSigWords * 8 + 2 * (size_t)cap * 8; }

}  // namespace ytk

extern "C" {

// Allocate this rank's uncached [signal | send | recv] block for slabs of cap int64; returns
// a group handle. The exported IPC handle (64 bytes) goes to out_handle.
int ytk_peer_create(int P, int rank, long long cap, uintptr_t out_handle) {
  if (P < 1 || P > ytk::kPeerMax || rank < 0 || rank >= P || cap <= 0)
    throw std::invalid_argument("peer_create: bad group");
  ytk::PeerGroup g;
  g.P = P;
  g.rank = rank;
  g.cap = cap;
  void* p = nullptr;
  YTK_HIP_CHECK(hipExtMallocWithFlags(&p, ytk::peer_bytes(cap), hipDeviceMallocUncached));
  YTK_HIP_CHECK(hipMemset(p, 0, ytk::peer_bytes(cap)));
  g.base = (char*)p;
  YTK_HIP_CHECK(hipMalloc(&g.err, sizeof(int)));
  YTK_HIP_CHECK(hipMemset(g.err, 0, sizeof(int)));
  YTK_HIP_CHECK(hipDeviceSynchronize());
  hipIpcMemHandle_t h;
  YTK_HIP_CHECK(hipIpcGetMemHandle(&h, p));
  memcpy(reinterpret_cast<void*>(out_handle), &h, sizeof(h));
  g_peer.push_back(g);
  return (int)g_peer.size() - 1;
}

// Open every peer's block (handles: P x 64 bytes in rank order; the own entry is skipped).
void ytk_peer_open(int hnd, uintptr_t handles) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  const char* hs = reinterpret_cast<const char*>(handles);
  for (int q = 0; q < g.P; ++q) {
    char* b = nullptr;
    if (q == g.rank) {
      b = g.base;
    } else {
      hipIpcMemHandle_t h;
      memcpy(&h, hs + (size_t)q * sizeof(h), sizeof(h));
      void* p = nullptr;
      YTK_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      g.opened.push_back(p);
      b = (char*)p;
    }
    g.pp.sig[q] = reinterpret_cast<unsigned long long*>(b);
    g.pp.send[q] = reinterpret_cast<long long*>(b + ytk::kSigWords * 8);
    g.pp.recv[q] = reinterpret_cast<long long*>(b + ytk::kSigWords * 8 + (size_t)g.cap * 8);
  }
}

// hist[0:n] <- the element-wise sum over the group's ranks (n <= cap int64), on `stream`.
void ytk_peer_allreduce(int hnd, uintptr_t data, long long n, long long max_spins, uintptr_t stream) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (n <= 0) return;
  if (n > g.cap) throw std::invalid_argument("peer_allreduce: message larger than the slab");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int grid = (int)std::min<long long>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(ytk::peer_copy_kernel, dim3(grid), dim3(256), 0, s, (const long long*)data, g.pp.send[g.rank], n);
  hipLaunchKernelGGL(ytk::peer_barrier_kernel, dim3(1), dim3(64), 0, s, g.pp, g.P, g.rank, ++g.epoch, g.err, max_spins);
  const int rgrid = (int)std::min<long long>((n / g.P + 255) / 256 + 1, 1024);
  hipLaunchKernelGGL(ytk::peer_reduce_kernel, dim3(rgrid), dim3(256), 0, s, g.pp, g.P, g.rank, n);
  hipLaunchKernelGGL(ytk::peer_barrier_kernel, dim3(1), dim3(64), 0, s, g.pp, g.P, g.rank, ++g.epoch, g.err, max_spins);
  hipLaunchKernelGGL(ytk::peer_copy_kernel, dim3(grid), dim3(256), 0, s, g.pp.recv[g.rank], (long long*)data, n);
  YTK_LAUNCH_CHECK();
}

// device address of the error word (non-zero: a barrier wait timed out)
uintptr_t ytk_peer_err(int hnd) { return reinterpret_cast<uintptr_t>(g_peer.at(hnd).err); }

// the error word, read after the device has drained (host check between trees)
int ytk_peer_check(int hnd) {
  int v = 0;
  YTK_HIP_CHECK(hipMemcpy(&v, g_peer.at(hnd).err, sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

void ytk_peer_destroy(int hnd) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (!g.base) return;
  (void)hipDeviceSynchronize();
  for (void* p : g.opened) (void)hipIpcCloseMemHandle(p);
  g.opened.clear();
  (void)hipFree(g.base);
  (void)hipFree(g.err);
  g.base = nullptr;
}

}  // extern "C"
