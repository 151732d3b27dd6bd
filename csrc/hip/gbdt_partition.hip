// Stable partition of tree-node row segments (gfx950 / CDNA4, wave64).
//
// Reference semantics: J/data/gbdt/SamplePositionData.java:115-165 -- after a
// split every row of the node goes left iff bin <= cond; left rows first, in
// their previous order, then right rows.
//
// Design (two launches per level, all split nodes batched):
//  1. flags: one pass over each node segment: row id (coalesced) + ONE BYTE from the
//     COLUMN-MAJOR copy of the bin matrix (binsT[f][row]: neighbouring positions of a
//     node hit neighbouring bytes of the same column instead of 32-B-strided rows),
//     writes a 1-byte go-left flag per position and a per-block left count.
//  2. scatter: coalesced reads of flags / row ids / (g,h) in position order,
//     4 sub-tiles of 256 positions per step, wave ballots + one LDS scan of the
//     16 (sub-tile, wave) counts -> stable destinations; writes the row id AND the
//     (g,h) pair so the next level's histogram reads (g,h) contiguously.
// items[blk] = {split_idx, begin, end, blk_in_node}; rows == nullptr means the identity
// permutation (root level without instance sampling: no iota copy).
#include "common.h"
#include "gbdt_partition_atomic.h"

#include <algorithm>

namespace ytk {

constexpr int kPartSub = 4;

template <typename BinT>
__global__ __launch_bounds__(kPartThreads) void partition_flags_kernel(
    const BinT* __restrict__ binsT, long long ncol, const int* __restrict__ rows,
    const int4* __restrict__ items, const int* __restrict__ feat, const int* __restrict__ thr,
    uint8_t* __restrict__ flags, int* __restrict__ counts, const int* __restrict__ nitems_dev,
    long long* __restrict__ left_acc) {
  __shared__ int s_cnt[kPartThreads / kWave];
  if (nitems_dev && (int)blockIdx.x >= *nitems_dev) return;
  const int4 it = items[blockIdx.x];
  const BinT* col = binsT + (size_t)feat[it.x] * ncol;
  const int t = thr[it.x] & kThrMask;
  int c = 0;
  int pos = it.y + threadIdx.x;
  for (; pos + 3 * kPartThreads < it.z; pos += 4 * kPartThreads) {
    int r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = rows ? rows[pos + j * kPartThreads] : pos + j * kPartThreads;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint8_t fl = (int)col[(unsigned)r[j]] <= t;
      flags[pos + j * kPartThreads] = fl;
      c += fl;
    }
  }
  for (; pos < it.z; pos += kPartThreads) {
    const uint8_t fl = (int)col[(unsigned)(rows ? rows[pos] : pos)] <= t;
    flags[pos] = fl;
    c += fl;
  }
  c = wave_sumi(c);
  if (lane_id() == 0) s_cnt[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    counts[blockIdx.x] = tot;
    // per-split left total (level engine): one 64-bit atomic per block
    if (left_acc) atomicAdd(reinterpret_cast<unsigned long long*>(&left_acc[it.x]),
                            (unsigned long long)tot);
  }
}

__global__ __launch_bounds__(kPartThreads) void partition_scatter_kernel(
    const uint8_t* __restrict__ flags, const int* __restrict__ rows,
    const float2* __restrict__ ghp, int* __restrict__ rows_out, float2* __restrict__ gh_out,
    const int4* __restrict__ items, const int* __restrict__ node_begin,
    const int* __restrict__ first_blk, const int* __restrict__ nblk,
    const int* __restrict__ counts, int* __restrict__ left_total_out,
    const int* __restrict__ nitems_dev) {
  constexpr int NW = kPartThreads / kWave;
  __shared__ int s_red[2 * NW];
  __shared__ int s_l[kPartSub * NW], s_v[kPartSub * NW];
  if (nitems_dev && (int)blockIdx.x >= *nitems_dev) return;
  const int4 it = items[blockIdx.x];
  const int si = it.x;
  const int nbeg = node_begin[si], fb = first_blk[si], nb = nblk[si];
  const int tid = threadIdx.x, wid = tid >> 6, l = lane_id();

  int before = 0, total = 0;
  for (int j = tid; j < nb; j += kPartThreads) {
    const int c = counts[fb + j];
    total += c;
    if (fb + j < (int)blockIdx.x) before += c;
  }
  before = wave_sumi(before);
  total = wave_sumi(total);
  if (l == 0) { s_red[wid] = before; s_red[NW + wid] = total; }
  __syncthreads();
  before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) { before += s_red[w]; total += s_red[NW + w]; }
  if (left_total_out && it.w == 0 && tid == 0) left_total_out[si] = total;

  int lbase = nbeg + before;
  int rbase = nbeg + total + (it.y - nbeg - before);
  const unsigned long long lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  for (int tile = it.y; tile < it.z; tile += kPartSub * kPartThreads) {
    int r[kPartSub];
    float2 g[kPartSub];
    bool valid[kPartSub], left[kPartSub];
#pragma unroll
    for (int j = 0; j < kPartSub; ++j) {
      const int pos = tile + j * kPartThreads + tid;
      valid[j] = pos < it.z;
      left[j] = false;
      r[j] = 0;
      g[j] = make_float2(0.f, 0.f);
      if (valid[j]) {
        left[j] = flags[pos] != 0;
        r[j] = rows ? rows[pos] : pos;
        if (ghp) g[j] = ghp[pos];
      }
    }
    int lrank[kPartSub], vrank[kPartSub];
#pragma unroll
    for (int j = 0; j < kPartSub; ++j) {
      const unsigned long long lm = __ballot(left[j]);
      const unsigned long long vm = __ballot(valid[j]);
      lrank[j] = __popcll(lm & lt_mask);
      vrank[j] = __popcll(vm & lt_mask);
      if (l == 0) { s_l[j * NW + wid] = __popcll(lm); s_v[j * NW + wid] = __popcll(vm); }
    }
    __syncthreads();
    int tl = 0, tv = 0;
    int pl[kPartSub], pv[kPartSub];
#pragma unroll
    for (int j = 0; j < kPartSub; ++j) { pl[j] = 0; pv[j] = 0; }
#pragma unroll
    for (int k = 0; k < kPartSub * NW; ++k) {
      const int kl = s_l[k], kv = s_v[k];
#pragma unroll
      for (int j = 0; j < kPartSub; ++j) {
        if (k < j * NW + wid) { pl[j] += kl; pv[j] += kv; }
      }
      tl += kl;
      tv += kv;
    }
#pragma unroll
    for (int j = 0; j < kPartSub; ++j) {
      if (valid[j]) {
        int dst;
        if (left[j]) dst = lbase + pl[j] + lrank[j];
        else dst = rbase + (pv[j] - pl[j]) + (vrank[j] - lrank[j]);
        rows_out[dst] = r[j];
        if (gh_out) gh_out[dst] = g[j];
      }
    }
    lbase += tl;
    rbase += tv - tl;
    __syncthreads();  // s_l / s_v reused next tile
  }
}


// Single-pass partition kernel (level engine and host-planned leaf-wise): see
// partition_atomic_body in gbdt_partition_atomic.h.
// kPrefetch (scatter with (g, h) moving: the level engine's multi-GPU levels): the
// software-pipelined body, next chunk's row ids and (g, h) in flight (see
// lv_partition_children_kernel; YTK_PART_PREFETCH=0 turns it off).
template <typename BinT, bool kScatter, bool kPrefetch = false>
__global__ __launch_bounds__(kPartThreads) void partition_atomic_kernel(
    const BinT* __restrict__ binsT, long long ncol, const int* __restrict__ rows,
    const float2* __restrict__ ghp, int* __restrict__ rows_out, float2* __restrict__ gh_out,
    const int* __restrict__ first_blk, const int* __restrict__ nsplit_dev,
    const int* __restrict__ nblocks_dev, const int* __restrict__ feat, const int* __restrict__ thr,
    const int* __restrict__ node_begin, const int* __restrict__ node_count,
    unsigned long long* __restrict__ cursor, const int* __restrict__ out_shift) {
  if constexpr (kScatter && kPrefetch)
    partition_atomic_body_pf<BinT, kAtomSub, true>(binsT, ncol, rows, ghp, rows_out, gh_out, first_blk, nsplit_dev,
                                                   nblocks_dev, feat, thr, node_begin, node_count, cursor,
                                                   out_shift, 1);
  else
    partition_atomic_body<BinT, kScatter>(binsT, ncol, rows, ghp, rows_out, gh_out, first_blk, nsplit_dev,
                                          nblocks_dev, feat, thr, node_begin, node_count, cursor, out_shift, 1);
}

}  // namespace ytk

using namespace ytk;

// Count-only variant (children that become leaves immediately: their rows are never
// read again, only the per-block left counts are needed for the node statistics).
extern "C" void ytk_partition_count(uintptr_t binsT, int bin_bytes, long long ncol,
                                    uintptr_t rows, uintptr_t flags, uintptr_t items, int nitems,
                                    uintptr_t feat, uintptr_t thr, uintptr_t counts,
                                    uintptr_t nitems_dev, uintptr_t left_acc, uintptr_t stream) {
  if (nitems <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(partition_flags_kernel<uint8_t>, dim3(nitems), dim3(kPartThreads), 0, s,
                       (const uint8_t*)binsT, ncol, (const int*)rows, (const int4*)items,
                       (const int*)feat, (const int*)thr, (uint8_t*)flags, (int*)counts,
                       (const int*)nitems_dev, (long long*)left_acc);
  } else {
    hipLaunchKernelGGL(partition_flags_kernel<uint16_t>, dim3(nitems), dim3(kPartThreads), 0, s,
                       (const uint16_t*)binsT, ncol, (const int*)rows, (const int4*)items,
                       (const int*)feat, (const int*)thr, (uint8_t*)flags, (int*)counts,
                       (const int*)nitems_dev, (long long*)left_acc);
  }
  YTK_LAUNCH_CHECK();
}

extern "C" void ytk_partition(uintptr_t binsT, int bin_bytes, long long ncol, uintptr_t rows,
                              uintptr_t rows_out, uintptr_t ghp, uintptr_t gh_out,
                              uintptr_t flags, uintptr_t items, int nitems, uintptr_t feat,
                              uintptr_t thr, uintptr_t node_begin, uintptr_t first_blk,
                              uintptr_t nblk, uintptr_t counts, uintptr_t left_total,
                              uintptr_t nitems_dev, uintptr_t left_acc, uintptr_t stream) {
  if (nitems <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(partition_flags_kernel<uint8_t>, dim3(nitems), dim3(kPartThreads), 0, s,
                       (const uint8_t*)binsT, ncol, (const int*)rows, (const int4*)items,
                       (const int*)feat, (const int*)thr, (uint8_t*)flags, (int*)counts,
                       (const int*)nitems_dev, (long long*)left_acc);
  } else {
    hipLaunchKernelGGL(partition_flags_kernel<uint16_t>, dim3(nitems), dim3(kPartThreads), 0, s,
                       (const uint16_t*)binsT, ncol, (const int*)rows, (const int4*)items,
                       (const int*)feat, (const int*)thr, (uint8_t*)flags, (int*)counts,
                       (const int*)nitems_dev, (long long*)left_acc);
  }
  YTK_LAUNCH_CHECK();
  hipLaunchKernelGGL(partition_scatter_kernel, dim3(nitems), dim3(kPartThreads), 0, s,
                     (const uint8_t*)flags, (const int*)rows, (const float2*)ghp, (int*)rows_out,
                     (float2*)gh_out, (const int4*)items, (const int*)node_begin,
                     (const int*)first_blk, (const int*)nblk, (const int*)counts,
                     (int*)left_total, (const int*)nitems_dev);
  YTK_LAUNCH_CHECK();
}

// Copy-back of partitioned segments (loss-guided batches partition a few node segments
// in place): rows[p] = rows_out[p], ghp[p] = gh_out[p] for p in every chunk [b, e) of
// items (the partition's own chunk list) -- one launch instead of two copies per node.
// Copy the partitioned segments back (leaf-wise growth partitions only the batch's
// segments). An item's range is split over gridDim.y blocks and every thread keeps 4
// independent loads in flight: the item ranges are large (a batch's rows / ~256) and
// one 256-thread block per item left the copy latency bound at ~1/4 of HBM bandwidth.
constexpr int kCopySplit = 16;
constexpr int kCopyUnroll = 4;

__global__ __launch_bounds__(kPartThreads) void segment_copy_kernel(
    const int4* __restrict__ items, const int* __restrict__ src_rows, int* __restrict__ dst_rows,
    const float2* __restrict__ src_gh, float2* __restrict__ dst_gh) {
  const int4 it = items[blockIdx.x];
  const int len = it.z - it.y;
  const int per = (len + (int)gridDim.y - 1) / (int)gridDim.y;
  const int b = it.y + (int)blockIdx.y * per, e = min(it.z, b + per);
  for (int p0 = b; p0 < e; p0 += kPartThreads * kCopyUnroll) {
    int r[kCopyUnroll];
    float2 g[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const int p = p0 + u * kPartThreads + (int)threadIdx.x;
      if (p < e) { r[u] = src_rows[p]; g[u] = src_gh[p]; }
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const int p = p0 + u * kPartThreads + (int)threadIdx.x;
      if (p < e) { dst_rows[p] = r[u]; dst_gh[p] = g[u]; }
    }
  }
}

extern "C" void ytk_segment_copy(uintptr_t items, int nitems, uintptr_t src_rows, uintptr_t dst_rows,
                                 uintptr_t src_gh, uintptr_t dst_gh, uintptr_t stream) {
  if (nitems <= 0) return;
  hipLaunchKernelGGL(segment_copy_kernel, dim3(nitems, kCopySplit), dim3(kPartThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), (const int4*)items,
                     (const int*)src_rows, (int*)dst_rows, (const float2*)src_gh, (float2*)dst_gh);
  YTK_LAUNCH_CHECK();
}

// hist[ids[i]] = 0 for the nslots listed slots (16-byte stores; one launch instead of an
// id conversion + index_fill from the host).
__global__ __launch_bounds__(256) void zero_slots_kernel(longlong2* __restrict__ hist, long long slot_v2,
                                                         const int* __restrict__ ids) {
  longlong2* h = hist + (size_t)ids[blockIdx.y] * slot_v2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < slot_v2; i += (long long)gridDim.x * 256)
    h[i] = make_longlong2(0, 0);
}

extern "C" void ytk_zero_slots(uintptr_t hist, long long slot_bytes, uintptr_t ids, int nslots,
                               uintptr_t stream) {
  if (nslots <= 0) return;
  const long long v2 = slot_bytes / 16;
  const int gx = (int)std::min<long long>(64, (v2 + 255) / 256);
  hipLaunchKernelGGL(zero_slots_kernel, dim3(gx, nslots), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (longlong2*)hist, v2, (const int*)ids);
  YTK_LAUNCH_CHECK();
}

extern "C" void ytk_memset_async(uintptr_t dst, int value, long long bytes, uintptr_t stream) {
  if (bytes <= 0) return;
  if (hipMemsetAsync((void*)dst, value, (size_t)bytes, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
    throw std::runtime_error("hipMemsetAsync failed");
}

// cursor: per split, zeroed by the caller; on return low 32 bits = left rows, high 32 =
// right rows (scatter) or the left rows alone (count_only). first_blk: exclusive scan of
// ceil(node_count / 2048) per split; nsplit_dev / nblocks_dev: device-resident counts;
// grid = max_blocks (blocks past *nblocks_dev exit). out_shift (optional, per split): offset
// added to every destination position (ping-pong halves of the leaf-wise engine).
extern "C" void ytk_partition_atomic(uintptr_t binsT, int bin_bytes, long long ncol, uintptr_t rows,
                                     uintptr_t rows_out, uintptr_t ghp, uintptr_t gh_out,
                                     uintptr_t first_blk, uintptr_t nsplit_dev, uintptr_t nblocks_dev,
                                     int max_blocks, uintptr_t feat, uintptr_t thr, uintptr_t node_begin,
                                     uintptr_t node_count, uintptr_t cursor, int count_only,
                                     uintptr_t out_shift, uintptr_t stream) {
  if (max_blocks <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const char* pf = getenv("YTK_PART_PREFETCH");
  const bool prefetch = ghp && gh_out && !(pf && (pf[0] == '0' || pf[0] == '1'));
#define YTK_PART_ATOMIC(BT, SC) do { if ((SC) && prefetch) YTK_PART_ATOMIC2(BT, SC, true); else YTK_PART_ATOMIC2(BT, SC, false); } while (0)
#define YTK_PART_ATOMIC2(BT, SC, PF)                                                              \
  hipLaunchKernelGGL((partition_atomic_kernel<BT, SC, PF>), dim3(std::min(max_blocks, kPartGrid)), dim3(kPartThreads), 0, s, \
                     (const BT*)binsT, ncol, (const int*)rows, (const float2*)ghp, (int*)rows_out,  \
                     (float2*)gh_out, (const int*)first_blk, (const int*)nsplit_dev,               \
                     (const int*)nblocks_dev, (const int*)feat, (const int*)thr,                   \
                     (const int*)node_begin, (const int*)node_count, (unsigned long long*)cursor,   \
                     (const int*)out_shift)
  if (bin_bytes == 1) {
    if (count_only) YTK_PART_ATOMIC(uint8_t, false); else YTK_PART_ATOMIC(uint8_t, true);
  } else {
    if (count_only) YTK_PART_ATOMIC(uint16_t, false); else YTK_PART_ATOMIC(uint16_t, true);
  }
#undef YTK_PART_ATOMIC
#undef YTK_PART_ATOMIC2
  YTK_LAUNCH_CHECK();
}
