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
#include <cstdlib>
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

// ------------------------------------------------------------------ peer-memory exchange
// All-reduce of the tree engines' level / batch messages and of the L-BFGS gradients over
// peer memory (xGMI), in ONE kernel per exchange and without the host: mp4j's collectives
// were latency-optimised recursive-halving / Rabenseifner algorithms for small messages and
// bandwidth-optimal ones for large (docs/gbdt_features.md:36,142-143; HistogramBuilder.java:95;
// HoagOptimizer.java:1038); at a 1/8 shard a level's build is 10-20 us, so the exchange's
// latency sets the multi-GPU tree time, while a 68-628 MB gradient needs every xGMI link.
//
// Every rank owns ONE uncached device allocation (hipDeviceMallocUncached: no cache level
// holds its lines, so data handed between processes never meets a stale line on any XCD)
//   [send flags: kPeerMax x kXchgGrid u64 | result flags: same | send slab 0, 1 | result slab 0, 1]
// exported with hipIpcGetMemHandle and opened by every other rank. A message is n elements
// (int64 histogram / count words, fp64 or fp32 sums) moved in 16-byte units; an exchange runs
// G blocks and, by its size (the same on every rank, so every rank takes the same path):
//  one-shot (small messages: latency): block b copies chunk b of the message into this rank's
//    send slab, releases it and stamps the epoch into send flag [rank][b] of EVERY rank, waits
//    for the peers' flags of chunk b, then sums chunk b of all P slabs in rank order (this
//    rank's own term from its buffer) and writes the sums back in place.
//  two-shot (large messages: bandwidth): rank q owns the q-th 1/P of the units; block b
//    publishes sub-chunk b of EVERY owner's range, waits for the peers' flags, sums sub-chunk
//    b of its OWN range over the P slabs (rank order), writes it in place and into its result
//    slab, stamps result flag [rank][b] everywhere, then copies sub-chunk b of every other
//    owner's result slab in place once that owner's flag is up. Each rank reads
//    2 (P - 1) / P of the message instead of P - 1 messages, spread over every peer's link.
// int64 sums are exact (bitwise the RCCL result); fp64 / fp32 sums are taken in rank order,
// identical on every rank. The two halves of two-shot also run alone (owner-computes sync,
// the message made of P equal segments): reduce-scatter (segment q summed into place on rank
// q only) and all-gather (rank q's segment copied into place on every rank). A message may be described by device words (the leaf-wise batch:
// its built slots + split cursors, counted by the planner) -- no host round trip per batch.
//
// Slab reuse: exchange e writes slab e & 1, exchange e + 2 writes it again. Block 0 takes
// part in every exchange (both phases), so during exchange e + 1 this rank saw a flag e + 1
// of every peer, stamped after that peer's exchange-e kernel (which read our slabs) had
// completed (stream order). Exchanges a rank skips (device-side skip word, e.g. the leaf-wise
// batches queued after the tree finished) advance no epoch; the skip word is identical on
// every rank because every rank takes the identical planning decisions. The epoch lives in
// device memory (advanced by each exchange's last block), so a captured HIP graph replays
// with fresh epochs. Waits are bounded in wall-clock time: a timed-out wait sets the error
// word (host-mapped; checked where rounds land) and the kernel finishes, and every later
// exchange of the group returns at once, so a lost peer never hangs the GPU.
namespace ytk {
constexpr int kPeerMax = 16;
constexpr int kXchgGrid = 256;     // max blocks of one exchange (flag words per rank)
constexpr int kXchgThreads = 256;
enum { XT_I64 = 0, XT_F64 = 1, XT_F32 = 2 };
enum { XM_ALLREDUCE = 0, XM_REDUCE_SCATTER = 1, XM_ALLGATHER = 2 };

struct PeerPtrs {
  char* send[kPeerMax][2];
  char* res[kPeerMax][2];
  unsigned long long* sig[kPeerMax];   // [kPeerMax][kXchgGrid] send flags of each rank
  unsigned long long* rsig[kPeerMax];  // [kPeerMax][kXchgGrid] result flags
};

// The message: contiguous (n >= 0: base[0..n)) or a leaf-wise batch of int64 words (n < 0:
// the *nb_dev slots listed in ids, slot_elems words each, then *k_dev * cur_stride cursors).
struct XchgMsg {
  char* base;
  long long n;
  long long* hist;
  const int* ids;
  const int* nb_dev;
  const int* k_dev;
  long long slot_elems;
  long long* cursor;
  int cur_stride;
  const int* skip;  // non-null and non-zero: no exchange
  int seg_p;        // > 0 (with n < 0): a CONTIGUOUS message at base of seg_p equal segments of
                    // *nb_dev * slot_elems + *k_dev * cur_stride words each (leaf-wise owner sync)
};

typedef long long xv2 __attribute__((ext_vector_type(2)));  // nontemporal builtins need a native vector

// unit u (16 bytes) of the message; gather mode: int64 pairs (slot sizes and cursor strides
// are even, every slot 16-B aligned)
__device__ __forceinline__ xv2* xchg_unit(const XchgMsg& m, long long u, long long nh) {
  if (m.n >= 0 || m.seg_p > 0) return reinterpret_cast<xv2*>(m.base) + u;
  const long long i = 2 * u;
  if (i < nh) {
    const long long kb = i / m.slot_elems;
    return reinterpret_cast<xv2*>(m.hist + (size_t)m.ids[kb] * m.slot_elems + (i - kb * m.slot_elems));
  }
  return reinterpret_cast<xv2*>(m.cursor + (i - nh));
}

template <int kType>
__device__ __forceinline__ xv2 unit_add(xv2 a, xv2 b) {
  if (kType == XT_I64) return a + b;
  if (kType == XT_F64) {
    xv2 r;
    r.x = __double_as_longlong(__longlong_as_double(a.x) + __longlong_as_double(b.x));
    r.y = __double_as_longlong(__longlong_as_double(a.y) + __longlong_as_double(b.y));
    return r;
  }
  float fa[4], fb[4];
  __builtin_memcpy(fa, &a, 16);
  __builtin_memcpy(fb, &b, 16);
#pragma unroll
  for (int k = 0; k < 4; ++k) fa[k] += fb[k];
  xv2 r;
  __builtin_memcpy(&r, fa, 16);
  return r;
}

// one element of the (contiguous) tail, summed in rank order
template <int kType>
__device__ __forceinline__ void tail_sum(char* dst, char* const* src, int P, int rank) {
  if (kType == XT_F32) {
    float s = 0.f;
    for (int q = 0; q < P; ++q) s += q == rank ? *(float*)dst : __builtin_nontemporal_load((const float*)src[q]);
    *(float*)dst = s;
  } else if (kType == XT_F64) {
    double s = 0.0;
    for (int q = 0; q < P; ++q) s += q == rank ? *(double*)dst : __builtin_nontemporal_load((const double*)src[q]);
    *(double*)dst = s;
  } else {
    long long s = 0;
    for (int q = 0; q < P; ++q)
      s += q == rank ? *(long long*)dst : __builtin_nontemporal_load((const long long*)src[q]);
    *(long long*)dst = s;
  }
}

// stamp flag [rank][b] = e into every peer's array; wait for [q][b] >= e of every peer
__device__ __forceinline__ void flag_publish(unsigned long long* const* sig, int P, int rank, int b,
                                             unsigned long long e) {
  const int t = threadIdx.x;
  if (t < P && t != rank)
    __hip_atomic_store(sig[t] + (size_t)rank * kXchgGrid + b, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void flag_wait(unsigned long long* const* sig, int P, int rank, int b, unsigned long long e,
                                          int* err, unsigned long long* ctl, long long timeout_ticks, int only = -1) {
  const int t = threadIdx.x;
  if (t < P && t != rank && (only < 0 || t == only)) {
    const unsigned long long* w = sig[rank] + (size_t)t * kXchgGrid + b;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(1);
      if (__hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;  // aborted
      if ((long long)(wall_clock64() - t0) > timeout_ticks) {
        atomicExch(err, 1);
        atomicExch(ctl + 2, 1ull);
        break;
      }
    }
  }
}

// the block's stores are acknowledged and released before its flags go out
template <bool kSysFence>
__device__ __forceinline__ void publish_fence() {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (kSysFence) {
    if (threadIdx.x == 0) __threadfence_system();
    __syncthreads();
  }
}
template <bool kSysFence>
__device__ __forceinline__ void acquire_fence() {
  __syncthreads();
  if (kSysFence) {
    if (threadIdx.x == 0) __threadfence_system();
    __syncthreads();
  }
}

template <int kType, bool kSysFence>
__global__ __launch_bounds__(kXchgThreads) void peer_xchg_kernel(PeerPtrs pp, int P, int rank, XchgMsg m,
                                                                 long long cap_bytes, unsigned long long* __restrict__ ctl,
                                                                 int* __restrict__ err, long long timeout_ticks,
                                                                 long long two_shot_bytes, int mode) {
  if (m.skip != nullptr && *m.skip != 0) return;
  // after a timed-out wait (ctl[2] != 0) every later exchange returns at once: the job is
  // failing (the host check raises), so nothing waits again
  if (__hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  constexpr int ES = kType == XT_F32 ? 4 : 8;  // element bytes
  constexpr int U = 16 / ES;                   // elements per unit
  __shared__ unsigned long long s_e;
  const int t = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  long long n = m.n, nh = 0;
  if (n < 0) {
    nh = (long long)(*m.nb_dev) * m.slot_elems;
    n = nh + (long long)(*m.k_dev) * m.cur_stride;
    if (m.seg_p > 0) n *= m.seg_p;  // contiguous segments
  }
  if (t == 0) s_e = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  // device-timed exchanges (diagnostics, ytk_peer_timing): block 0's start, read by the last
  // block to finish (which arrived after block 0's start, through the ctl[1] counter)
  if (b == 0 && t == 0) __hip_atomic_store(ctl + 3, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned long long e = s_e;
  if (n * ES > cap_bytes) {  // identical on every rank: nobody exchanges, the host check raises
    if (b == 0 && t == 0) atomicExch(err, 2);
    n = 0;
  }
  const long long nu = n / U;       // 16-byte units
  const int tail = (int)(n - nu * U);  // contiguous messages only (gather messages are even)
  const bool tail_blk = tail > 0 && b == G - 1;
  const int par = (int)(e & 1ull);
  xv2* mine = reinterpret_cast<xv2*>(pp.send[rank][par]);
  // reduce-scatter / all-gather: the owner ranges are the message's P segments (the host
  // checked that they are whole, equal numbers of units: no tail)
  const bool two = mode != XM_ALLREDUCE || (nu * 16 >= two_shot_bytes && P > 1);
  if (!two) {
    const long long lo = nu * b / G, hi = nu * (b + 1) / G;
    if (!(hi > lo || tail_blk || b == 0)) goto done;
    for (long long u = lo + t; u < hi; u += kXchgThreads) __builtin_nontemporal_store(*xchg_unit(m, u, nh), mine + u);
    if (tail_blk && t < tail) {
      const long long off = (nu * U + t) * ES;
      __builtin_memcpy(pp.send[rank][par] + off, m.base + off, ES);
    }
    publish_fence<kSysFence>();
    flag_publish(pp.sig, P, rank, b, e);
    flag_wait(pp.sig, P, rank, b, e, err, ctl, timeout_ticks);
    acquire_fence<kSysFence>();
    for (long long u = lo + t; u < hi; u += kXchgThreads) {
      xv2* dst = xchg_unit(m, u, nh);
      xv2 s = *dst;
      if (rank > 0) s = __builtin_nontemporal_load(reinterpret_cast<const xv2*>(pp.send[0][par]) + u);
      for (int q = 1; q < P; ++q) {
        const xv2 v = q == rank ? *dst : __builtin_nontemporal_load(reinterpret_cast<const xv2*>(pp.send[q][par]) + u);
        s = unit_add<kType>(s, v);
      }
      *dst = s;
    }
  } else {
    // ---- two-shot: owner q's units [nu q / P, nu (q + 1) / P), sub-chunk b of each
    auto sub = [&](int q, long long& lo, long long& hi) {
      const long long a = nu * q / P, z = nu * (q + 1) / P;
      lo = a + (z - a) * b / G;
      hi = a + (z - a) * (b + 1) / G;
    };
    long long lo, hi;
    xv2* rmine = reinterpret_cast<xv2*>(pp.res[rank][par]);
    if (mode == XM_ALLGATHER) {
      // this rank's own segment goes straight to its result slab
      sub(rank, lo, hi);
      for (long long u = lo + t; u < hi; u += kXchgThreads) __builtin_nontemporal_store(*xchg_unit(m, u, nh), rmine + u);
    } else {
      for (int q = 0; q < P; ++q) {  // publish sub-chunk b of every owner's range
        sub(q, lo, hi);
        for (long long u = lo + t; u < hi; u += kXchgThreads) __builtin_nontemporal_store(*xchg_unit(m, u, nh), mine + u);
      }
      if (tail_blk && t < tail) {
        const long long off = (nu * U + t) * ES;
        __builtin_memcpy(pp.send[rank][par] + off, m.base + off, ES);
      }
      publish_fence<kSysFence>();
      flag_publish(pp.sig, P, rank, b, e);
      flag_wait(pp.sig, P, rank, b, e, err, ctl, timeout_ticks);
      acquire_fence<kSysFence>();
      // reduce this rank's sub-chunk b; result in place (+ into the result slab)
      sub(rank, lo, hi);
      for (long long u = lo + t; u < hi; u += kXchgThreads) {
        xv2* dst = xchg_unit(m, u, nh);
        xv2 s = *dst;
        if (rank > 0) s = __builtin_nontemporal_load(reinterpret_cast<const xv2*>(pp.send[0][par]) + u);
        for (int q = 1; q < P; ++q) {
          const xv2 v = q == rank ? *dst : __builtin_nontemporal_load(reinterpret_cast<const xv2*>(pp.send[q][par]) + u);
          s = unit_add<kType>(s, v);
        }
        *dst = s;
        if (mode == XM_ALLREDUCE) __builtin_nontemporal_store(s, rmine + u);
      }
    }
    if (mode == XM_REDUCE_SCATTER) goto done;
    publish_fence<kSysFence>();
    flag_publish(pp.rsig, P, rank, b, e);
    // the other owners' reduced sub-chunks b, each as soon as its owner's flag is up
    for (int q = 0; q < P; ++q) {
      if (q == rank) continue;
      flag_wait(pp.rsig, P, rank, b, e, err, ctl, timeout_ticks, q);
      acquire_fence<kSysFence>();
      sub(q, lo, hi);
      const xv2* rq = reinterpret_cast<const xv2*>(pp.res[q][par]);
      for (long long u = lo + t; u < hi; u += kXchgThreads) *xchg_unit(m, u, nh) = __builtin_nontemporal_load(rq + u);
    }
  }
  if (tail_blk && t < tail) {  // the last < 16 bytes: every rank sums them itself (block G - 1
    const long long off = (nu * U + t) * ES;  // waited for every peer's block G - 1 above)
    char* src[kPeerMax];
    for (int q = 0; q < P; ++q) src[q] = pp.send[q][par] + off;
    tail_sum<kType>(m.base + off, src, P, rank);
  }
done:
  // the last block to finish advances the epoch (the next exchange kernel starts after this
  // one has completed, so every block of it reads the new value)
  __syncthreads();
  if (t == 0) {
    const unsigned long long prev = atomicAdd(ctl + 1, 1ull);
    if (prev == (unsigned long long)(G - 1)) {
      __hip_atomic_store(ctl + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = __hip_atomic_load(ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ctl[4] += wall_clock64() - t0;  // exchange ticks (only this block writes ctl[4], ctl[5])
      ctl[5] += 1;
    }
  }
}

struct PeerGroup {
  int P = 0, rank = 0;
  long long cap = 0;     // bytes per slab
  char* base = nullptr;  // own uncached allocation
  std::vector<void*> opened;
  PeerPtrs pp{};
  unsigned long long* ctl = nullptr;  // device: [0] last epoch, [1] block arrivals, [2] timed out,
                                      // [3] exchange start tick, [4] exchange ticks, [5] exchanges
  long long ticks_per_s = 100000000;  // wall_clock64 rate
  bool sys_fence = true;              // YTK_PEER_SYS_FENCE=0: waitcnt-ordered publishing only
  int block_bytes = 16384;            // YTK_PEER_BLOCK_BYTES: message bytes per block
  long long two_shot_bytes = 1 << 20;  // YTK_PEER_TWO_SHOT_BYTES: two-shot from this size on
  int* err_host = nullptr;            // host-mapped error word
  int* err = nullptr;                 // its device address
  int grid_cap = kXchgGrid;           // blocks per exchange (ytk_peer_set_grid_cap)
};
}  // namespace ytk
static std::vector<ytk::PeerGroup> g_peer;
namespace ytk {

static size_t peer_sig_bytes() { return (size_t)kPeerMax * kXchgGrid * 8; }
static size_t peer_bytes(long long cap) { return 2 * peer_sig_bytes() + 4 * (size_t)cap; }

static void peer_launch(PeerGroup& g, const XchgMsg& m, int grid, int type, double timeout_s, hipStream_t s,
                        int mode = XM_ALLREDUCE) {
  grid = std::max(1, std::min(grid, g.grid_cap));
  const long long ticks = (long long)(timeout_s * (double)g.ticks_per_s);
#define YTK_XCHG(T, S)                                                                                     \
  hipLaunchKernelGGL((peer_xchg_kernel<T, S>), dim3(grid), dim3(kXchgThreads), 0, s, g.pp, g.P, g.rank, m, \
                     g.cap, g.ctl, g.err, ticks, g.two_shot_bytes, mode)
  if (g.sys_fence) {
    if (type == XT_F64) YTK_XCHG(XT_F64, true);
    else if (type == XT_F32) YTK_XCHG(XT_F32, true);
    else YTK_XCHG(XT_I64, true);
  } else {
    if (type == XT_F64) YTK_XCHG(XT_F64, false);
    else if (type == XT_F32) YTK_XCHG(XT_F32, false);
    else YTK_XCHG(XT_I64, false);
  }
#undef YTK_XCHG
  YTK_LAUNCH_CHECK();
}

}  // namespace ytk

extern "C" {

// Allocate this rank's uncached [flags | send 0, 1 | result 0, 1] block for messages of up to
// cap bytes; returns a group handle. The exported IPC handle (64 bytes) goes to out_handle.
int ytk_peer_create(int P, int rank, long long cap, uintptr_t out_handle) {
  if (P < 1 || P > ytk::kPeerMax || rank < 0 || rank >= P || cap <= 0)
    throw std::invalid_argument("peer_create: bad group");
  cap = (cap + 255) & ~255LL;  // every slab 256-B aligned
  ytk::PeerGroup g;
  g.P = P;
  g.rank = rank;
  g.cap = cap;
  void* p = nullptr;
  YTK_HIP_CHECK(hipExtMallocWithFlags(&p, ytk::peer_bytes(cap), hipDeviceMallocUncached));
  YTK_HIP_CHECK(hipMemset(p, 0, 2 * ytk::peer_sig_bytes()));
  g.base = (char*)p;
  YTK_HIP_CHECK(hipMalloc(&g.ctl, 8 * sizeof(unsigned long long)));
  YTK_HIP_CHECK(hipMemset(g.ctl, 0, 8 * sizeof(unsigned long long)));
  int dev = 0, khz = 0;
  YTK_HIP_CHECK(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
    g.ticks_per_s = (long long)khz * 1000;
  if (const char* e = getenv("YTK_PEER_SYS_FENCE")) g.sys_fence = e[0] != '0';
  if (const char* e = getenv("YTK_PEER_BLOCK_BYTES")) g.block_bytes = std::max(1024, atoi(e));
  if (const char* e = getenv("YTK_PEER_TWO_SHOT_BYTES")) g.two_shot_bytes = std::max(0LL, atoll(e));
  YTK_HIP_CHECK(hipHostMalloc(&g.err_host, sizeof(int), hipHostMallocMapped));
  *g.err_host = 0;
  void* dp = nullptr;
  YTK_HIP_CHECK(hipHostGetDevicePointer(&dp, g.err_host, 0));
  g.err = (int*)dp;
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
  const size_t sb = ytk::peer_sig_bytes();
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
    g.pp.rsig[q] = reinterpret_cast<unsigned long long*>(b + sb);
    for (int k = 0; k < 2; ++k) {
      g.pp.send[q][k] = b + 2 * sb + (size_t)k * g.cap;
      g.pp.res[q][k] = b + 2 * sb + (size_t)(2 + k) * g.cap;
    }
  }
}

// data[0:n] <- the element-wise sum over the group's ranks, in place, on `stream`: one kernel
// launch. type: 0 int64, 1 fp64, 2 fp32. n must be identical on every rank.
void ytk_peer_allreduce(int hnd, uintptr_t data, long long n, int type, double timeout_s, uintptr_t stream) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (n <= 0 || g.P == 1) return;  // a one-rank all-reduce is the identity
  const long long bytes = n * (type == ytk::XT_F32 ? 4 : 8);
  if (bytes > g.cap) throw std::invalid_argument("peer_allreduce: message larger than the slab");
  if (data % 16 != 0) throw std::invalid_argument("peer_allreduce: data must be 16-B aligned");
  ytk::XchgMsg m{};
  m.base = reinterpret_cast<char*>(data);
  m.n = n;
  const int grid = (int)std::min<long long>((bytes + g.block_bytes - 1) / g.block_bytes, ytk::kXchgGrid);
  ytk::peer_launch(g, m, grid, type, timeout_s, reinterpret_cast<hipStream_t>(stream));
}

// Owner-computes halves of the exchange over P equal segments of data[0:n] (n a multiple of
// P 16-byte units): reduce-scatter leaves the sum over the ranks of segment `rank` in place
// (the other segments keep this rank's values); all-gather copies every rank's own segment
// into place on every rank. One kernel each; a one-rank group is the identity.
static void peer_segments(int hnd, uintptr_t data, long long n, int type, double timeout_s, uintptr_t stream,
                          int mode, uintptr_t skip) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (n <= 0 || g.P == 1) return;
  const int es = type == ytk::XT_F32 ? 4 : 8;
  const long long bytes = n * es;
  if (bytes > g.cap) throw std::invalid_argument("peer segments: message larger than the slab");
  if (data % 16 != 0 || bytes % (16LL * g.P) != 0)
    throw std::invalid_argument("peer segments: 16-B aligned data of P whole 16-B unit segments needed");
  ytk::XchgMsg m{};
  m.base = reinterpret_cast<char*>(data);
  m.n = n;
  m.skip = reinterpret_cast<const int*>(skip);
  const int grid = (int)std::min<long long>((bytes + g.block_bytes - 1) / g.block_bytes, ytk::kXchgGrid);
  ytk::peer_launch(g, m, grid, type, timeout_s, reinterpret_cast<hipStream_t>(stream), mode);
}

void ytk_peer_reduce_scatter(int hnd, uintptr_t data, long long n, int type, double timeout_s, uintptr_t stream) {
  peer_segments(hnd, data, n, type, timeout_s, stream, ytk::XM_REDUCE_SCATTER, 0);
}

// skip (optional): a device word; non-zero = no exchange (leaf-wise batches past the tree's end)
void ytk_peer_allgather(int hnd, uintptr_t data, long long n, int type, double timeout_s, uintptr_t stream,
                        uintptr_t skip) {
  peer_segments(hnd, data, n, type, timeout_s, stream, ytk::XM_ALLGATHER, skip);
}

// Reduce-scatter of a contiguous int64 message of P equal segments sized on the device: each
// segment is *nb_dev * seg_slot + *k_dev * cur_stride words (leaf-wise owner-computes batch:
// the packed feature blocks of the built slots + the split cursors). Skipped while *skip != 0.
void ytk_peer_reduce_scatter_dev(int hnd, uintptr_t data, long long seg_slot, uintptr_t nb_dev, uintptr_t k_dev,
                                 int cur_stride, uintptr_t skip, double timeout_s, uintptr_t stream) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (g.P == 1) return;
  if ((seg_slot & 1) || (cur_stride & 1) || data % 16 != 0)
    throw std::invalid_argument("peer_reduce_scatter_dev: even segment parts and 16-B aligned data needed");
  ytk::XchgMsg m{};
  m.base = reinterpret_cast<char*>(data);
  m.n = -1;
  m.nb_dev = reinterpret_cast<const int*>(nb_dev);
  m.k_dev = reinterpret_cast<const int*>(k_dev);
  m.slot_elems = seg_slot;
  m.cur_stride = cur_stride;
  m.seg_p = g.P;
  m.skip = reinterpret_cast<const int*>(skip);
  ytk::peer_launch(g, m, ytk::kXchgGrid, ytk::XT_I64, timeout_s, reinterpret_cast<hipStream_t>(stream),
                   ytk::XM_REDUCE_SCATTER);
}

// Leaf-wise batch message counted on the device: the *nb_dev built slots listed in ids
// (slot_elems int64 each, at hist + ids[i] * slot_elems) and the first *k_dev * cur_stride
// cursor words; skipped (no epoch) while *skip != 0. Fixed grid: one launch, no host wait.
void ytk_peer_allreduce_slots(int hnd, uintptr_t hist, long long slot_elems, uintptr_t ids, uintptr_t nb_dev,
                              uintptr_t cursor, uintptr_t k_dev, int cur_stride, uintptr_t skip, double timeout_s,
                              uintptr_t stream) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (g.P == 1) return;  // a one-rank all-reduce is the identity
  if ((slot_elems & 1) || (cur_stride & 1)) throw std::invalid_argument("peer_allreduce_slots: odd slot / stride");
  ytk::XchgMsg m{};
  m.n = -1;
  m.hist = reinterpret_cast<long long*>(hist);
  m.ids = reinterpret_cast<const int*>(ids);
  m.nb_dev = reinterpret_cast<const int*>(nb_dev);
  m.k_dev = reinterpret_cast<const int*>(k_dev);
  m.slot_elems = slot_elems;
  m.cursor = reinterpret_cast<long long*>(cursor);
  m.cur_stride = cur_stride;
  m.skip = reinterpret_cast<const int*>(skip);
  ytk::peer_launch(g, m, ytk::kXchgGrid, ytk::XT_I64, timeout_s, reinterpret_cast<hipStream_t>(stream));
}

// the host-mapped error word (1: a flag wait timed out, 2: a device-counted message exceeded
// the slab); read after the device has drained past the exchanges
int ytk_peer_check(int hnd) { return *(volatile int*)g_peer.at(hnd).err_host; }

// Abort the group (the job is failing): every exchange waiting now and every later one
// returns at once. The word is written from a stream of its own, so it lands while this
// rank's compute stream is still blocked in an exchange.
void ytk_peer_abort(int hnd) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
  (void)hipMemsetAsync(g.ctl + 2, 1, 1, s);
  (void)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
}

// the group's last completed exchange epoch (synchronous copy: diagnostics after a failure)
long long ytk_peer_epoch(int hnd) {
  unsigned long long e = 0;
  (void)hipMemcpy(&e, g_peer.at(hnd).ctl, sizeof(e), hipMemcpyDeviceToHost);
  return (long long)e;
}

// Device-timed exchanges so far (synchronous copy; diagnostics): out[0] = exchanges that ran,
// out[1] = their summed wall time in microseconds (block 0's start to the last block's end).
void ytk_peer_timing(int hnd, uintptr_t out) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  unsigned long long c[8] = {};
  (void)hipMemcpy(c, g.ctl, sizeof(c), hipMemcpyDeviceToHost);
  double* o = reinterpret_cast<double*>(out);
  o[0] = (double)c[5];
  o[1] = 1e6 * (double)c[4] / (double)g.ticks_per_s;
}

// At most `cap` blocks per exchange (every rank of the group must use the same cap). An
// exchange's blocks spin on their peers' flags, so the peers' exchange kernels have to be
// co-resident; ranks that SHARE one GPU must also leave room for each other's earlier
// kernels, which a full 256-block exchange per rank can starve (one process per GPU never
// co-schedules another rank's work).
void ytk_peer_set_grid_cap(int hnd, int cap) {
  g_peer.at(hnd).grid_cap = std::max(1, std::min(cap, ytk::kXchgGrid));
}

void ytk_peer_destroy(int hnd) {
  ytk::PeerGroup& g = g_peer.at(hnd);
  if (!g.base) return;
  (void)hipDeviceSynchronize();
  for (void* p : g.opened) (void)hipIpcCloseMemHandle(p);
  g.opened.clear();
  (void)hipFree(g.base);
  (void)hipFree(g.ctl);
  (void)hipHostFree(g.err_host);
  g.base = nullptr;
}

}  // extern "C"
