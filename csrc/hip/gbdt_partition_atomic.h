// Single-pass row partition body shared by the level engine's partition kernel
// (gbdt_partition.hip) and the leaf-wise engine's fused partition + children kernel
// (gbdt_leafwise.hip).
#pragma once
#include "common.h"
#include "gbdt_chunk_range.h"

namespace ytk {

constexpr int kPartThreads = 256;
constexpr int kPartGrid = 256 * 8;  // persistent partition blocks: 8 per CU
constexpr int kAtomSub = 8;  // single-pass partition: rows per block = 8 x 256 (one chunk)
// Device-scope atomics on ONE cache line serialise at ~12 ns each on MI355X
// (tools/microbench/atomic_contention.hip: 5127 returning 64-bit adds, one per 2048-row
// chunk = one partition level of Higgs, take 63.5 us on one line, 7 us over 32 lines
// 4 KiB apart). The engines therefore space the split cursors a cache line apart
// (kCurStride u64) and count finished blocks through kDoneGroups line-spaced counters.
constexpr int kCurStride = 16;   // u64 per split cursor (128 B)
constexpr int kDoneGroups = 16;
constexpr int kDoneWords = (kDoneGroups + 1) * kCurStride;  // u64 of counter space

// Split thresholds carry a scatter mask in their top bits (level engine, last scatter level:
// only the child that gets a histogram is ever read again, so only its rows are written;
// the counts and the segment geometry are unchanged): 0 both children, 1 left only, 2 right
// only. Thresholds are bin indices (< 2^16).
constexpr int kKeepShift = 30;
constexpr int kThrMask = (1 << kKeepShift) - 1;
__device__ __forceinline__ bool keep_row(int keep, bool left) { return keep == 0 || (keep == 1) == left; }

// true in exactly one block of the grid: the last to arrive. Block b counts itself in
// group b % G; the block completing its group counts the group at the top counter. All
// counters reset themselves (atomic exchange by their last arriver), so ctr must be zero
// only before the first launch. ctr: kDoneWords u64 (zeroed once).
__device__ __forceinline__ bool last_block_done(unsigned long long* ctr64) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* ctr = reinterpret_cast<unsigned*>(ctr64);
    const unsigned G = min(gridDim.x, (unsigned)kDoneGroups);
    const unsigned g = blockIdx.x % G;
    const unsigned members = (gridDim.x - g + G - 1) / G;
    unsigned* grp = ctr + (size_t)g * kCurStride * 2;
    unsigned* top = ctr + (size_t)kDoneGroups * kCurStride * 2;
    bool last = false;
    if (atomicAdd(grp, 1u) == members - 1) {
      atomicExch(grp, 0u);
      if (atomicAdd(top, 1u) == G - 1) {
        atomicExch(top, 0u);
        last = true;
      }
    }
    s_last = last ? 1 : 0;
  }
  __syncthreads();
  return s_last != 0;
}

// Single-pass partition (level engine): each block holds one <= 2048-row chunk in
// registers, gathers its go-left flags, ranks them with wave ballots, reserves its left
// run at the front and its right run at the BACK of the node segment with ONE 64-bit
// atomic on the split's cursor ((right << 32) | left), and scatters row ids and (g, h). No flag
// array, no count pass, one launch: 25 B/row instead of 31 B/row and two launches.
// Chunks land in arbitrary order inside the left / right runs (rows inside a chunk keep
// their order): positions are a free permutation for everything downstream -- the
// int64 histograms, split counts and leaf values are order independent, so trees are
// bitwise identical to the stable two-pass partition.
// S: rows per thread (chunk = S x 256 rows). The level engine's fused kernel runs S = 16
// (4096-row chunks): half the cursor reservations of S = 8, which is what bounds the top
// levels (one split: every chunk reserves on ONE cursor line, ~12 ns each serialised --
// tools/microbench/part_bench.py: 68 us for a count-only root split vs 17 us over 512
// splits). S * (256 / 64) <= 64: the per-(sub-chunk, wave) left counts are scanned by one wave.
template <typename BinT, bool kScatter, int S = kAtomSub>
__device__ __forceinline__ void partition_atomic_body(
    const BinT* __restrict__ binsT, long long ncol, const int* __restrict__ rows,
    const float2* __restrict__ ghp, int* __restrict__ rows_out, float2* __restrict__ gh_out,
    const int* __restrict__ first_blk, const int* __restrict__ nsplit_dev,
    const int* __restrict__ nblocks_dev, const int* __restrict__ feat, const int* __restrict__ thr,
    const int* __restrict__ node_begin, const int* __restrict__ node_count,
    unsigned long long* __restrict__ cursor, const int* __restrict__ out_shift, int cs) {
  // cs: cursor stride (u64; kCurStride in the engines, 1 for the standalone kernel)
  // one chunk (<= S * 256 rows) per block, held in registers: all loads issued
  // up front, ONE cursor reservation per block, then the scatter. The block finds its
  // (split, chunk) by binary search of first_blk (exclusive scan of the splits' chunk
  // counts) -- no per-block work list. kScatter = false: left counts only (last level).
  constexpr int NW = kPartThreads / kWave;
  static_assert(S * NW <= kWave, "one-wave scan of the sub-chunk counts");
  constexpr int CH = S * kPartThreads;
  constexpr int kSplitLds = 1024;  // splits whose chunk table is staged in LDS
  __shared__ int s_l[S * NW];
  __shared__ int s_first[kSplitLds];
  __shared__ unsigned long long s_base;
  __shared__ int s_tl;
  const int nblocks = *nblocks_dev, nsplit = *nsplit_dev;
  if ((int)blockIdx.x >= nblocks) return;  // uniform per block
  const int tid = threadIdx.x, wid = tid >> 6, l = lane_id();
  // Persistent blocks: the grid is capped (kPartGrid) and each block walks chunks
  // bid, bid + gridDim.x, ... Measured: with one short-lived 4-wave block per 2048-row
  // chunk (~5k blocks per level) the workgroup launch rate, not memory, set the time
  // (~4 us wave lifetime, < 1/8 of the wave slots ever occupied).
  // The chunk table is staged in LDS once per block, so locating a chunk's split costs
  // no dependent global round trips.
  const bool lds_tab = nsplit <= kSplitLds;
  if (lds_tab) {
    for (int i = tid; i < nsplit; i += kPartThreads) s_first[i] = first_blk[i];
    __syncthreads();
  }
  const unsigned long long lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  for (int bid = (int)blockIdx.x; bid < nblocks; bid += (int)gridDim.x) {
  int lo = 0, hi = nsplit - 1;  // last split with first_blk <= bid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((lds_tab ? s_first[mid] : first_blk[mid]) <= bid) lo = mid; else hi = mid - 1;
  }
  const int si = lo;
  // independent loads of the split's parameters (one round trip)
  const int fb = first_blk[si], nbeg = node_begin[si], ncnt = node_count[si], fs = feat[si];
  const int th = thr[si] & kThrMask, keep = (int)((unsigned)thr[si] >> kKeepShift);
  const int beg = nbeg + (bid - fb) * CH;
  const int end = min(beg + CH, nbeg + ncnt);
  const int nend = nbeg + ncnt;
  const BinT* col = binsT + (size_t)fs * ncol;
  // valid rows form a prefix of the chunk in position order: the rank of a valid row
  // among the chunk's rows is simply j * 256 + tid (no ballot needed)
  int r[S];
  float2 g[S];
  bool left[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int pos = beg + j * kPartThreads + tid;
    r[j] = pos < end ? (rows ? rows[pos] : pos) : 0;
  }
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int pos = beg + j * kPartThreads + tid;
    const bool valid = pos < end;
    // ghp == nullptr: (g, h) stays ROW-indexed (leaf-wise engine) -- only row ids move
    g[j] = (kScatter && valid && ghp) ? ghp[pos] : make_float2(0.f, 0.f);
    left[j] = valid && (int)col[(unsigned)r[j]] <= th;
  }
  int lrank[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const unsigned long long lm = __ballot(left[j]);
    lrank[j] = __popcll(lm & lt_mask);
    if (l == 0) s_l[j * NW + wid] = __popcll(lm);
  }
  __syncthreads();
  // exclusive scan of the S * NW (= 32) per-(sub-chunk, wave) left counts by wave 0
  if (wid == 0) {
    const int x = l < S * NW ? s_l[l] : 0;
    int incl = x;
#pragma unroll
    for (int off = 1; off < S * NW; off <<= 1) {
      const int y = __shfl_up(incl, off, kWave);
      if (l >= off) incl += y;
    }
    if (l < S * NW) s_l[l] = incl - x;
    const int tl_all = __shfl(incl, S * NW - 1, kWave);
    if (l == 0) {
      const int tv = end - beg;
      if (!kScatter) {
        atomicAdd(&cursor[(size_t)si * cs], (unsigned long long)tl_all);  // count-only: the left rows
      } else {
        s_base = atomicAdd(&cursor[(size_t)si * cs], ((unsigned long long)(tv - tl_all) << 32) | (unsigned long long)tl_all);
        s_tl = tl_all;
      }
    }
  }
  __syncthreads();
  if (kScatter) {
    const int tl = s_tl;
    const int tv = end - beg;
    const unsigned long long base = s_base;
    const int lofs = (int)(base & 0xffffffffull), rofs = (int)(base >> 32);
    // out_shift (leaf-wise engine): the children land in the OTHER half of a 2N-entry
    // ping-pong buffer (per split: +N or -N), so no copy-back of the partitioned segments
    const int sh = out_shift ? out_shift[si] : 0;
    const int rstart = nend - rofs - (tv - tl) + sh;
    const int lstart = nbeg + lofs + sh;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int rank = j * kPartThreads + tid;  // rank among the chunk's rows
      if (rank < tv) {
        const int lb = s_l[j * NW + wid] + lrank[j];  // left rows before this one
        const int dst = left[j] ? lstart + lb : rstart + (rank - lb);
        if (keep_row(keep, left[j])) {
          rows_out[dst] = r[j];
          if (gh_out) gh_out[dst] = g[j];
        }
      }
    }
  }
  __syncthreads();  // s_l / s_base / s_tl are reused by the next chunk
  }
}

constexpr int kPreLoads = 2;  // kMode 3: unrolled prefix loads per thread (covers 25M-row splits)

// Software-pipelined variant of partition_atomic_body (level engine, scatter levels): the
// persistent block locates its NEXT chunk and issues that chunk's row-id loads before it
// ranks, reserves and scatters the current one, so the row-id round trip of chunk i + 1
// overlaps the ballot / cursor-atomic / scatter phases of chunk i. Same output as the
// unpipelined body (same reservation per chunk, same placement).
// kMode (splits with thousands of chunks each -- the root level: every one of Higgs' 5127
// chunks reserved on ONE cursor line, ~12 ns apiece serialised, 62 of the level's 77 us):
//   0: reserve with the cursor atomic;
//   2: scatter at chunk_io[chunk], the reservation a scan of the chunk counts computed
//      (part_chunk_scan_kernel: the same (right, left) prefix an atomic would have returned
//      in chunk order; the split cursors hold the totals);
//   3: chunk_io holds the raw per-chunk counts and gsum their sums per group of 32 chunks
//      (part_count_lean_body) and the block sums its chunk's prefix itself -- the split's
//      earlier chunks as whole groups plus at most 2 x 31 single counts (ChunkRange: 230
//      values at Higgs' root, one load per thread, issued before the next chunk's row ids and
//      reduced under the rank phase's barrier) -- so no scan launch sits between the count
//      pass and the scatter (the caller's last block writes the split totals and re-zeroes
//      gsum, part_split_totals).
template <typename BinT, int S = kAtomSub, bool kGh = false, bool kCol = false, int kMode = 0>
__device__ __forceinline__ void partition_atomic_body_pf(
    const BinT* __restrict__ binsT, long long ncol, const int* __restrict__ rows,
    const float2* __restrict__ ghp, int* __restrict__ rows_out, float2* __restrict__ gh_out,
    const int* __restrict__ first_blk, const int* __restrict__ nsplit_dev,
    const int* __restrict__ nblocks_dev, const int* __restrict__ feat, const int* __restrict__ thr,
    const int* __restrict__ node_begin, const int* __restrict__ node_count,
    unsigned long long* __restrict__ cursor, const int* __restrict__ out_shift, int cs, int gh_rows = 0,
    unsigned long long* __restrict__ chunk_io = nullptr, const unsigned long long* __restrict__ gsum = nullptr) {
  // ghp == nullptr: (g, h) stays row-indexed (leaf-wise engine); out_shift as in
  // partition_atomic_body (children into the other half of a 2N ping-pong buffer).
  // gh_rows: ghp is indexed by ROW id (the level engine's first gathered level), so the next
  // chunk's (g, h) gather waits for its row ids: it is issued after this chunk's cursor
  // reservation (like the split-feature bytes of kCol) instead of with the row-id loads.
  constexpr int NW = kPartThreads / kWave;
  static_assert(S * NW <= kWave, "one-wave scan of the sub-chunk counts");
  constexpr int CH = S * kPartThreads;
  constexpr int kSplitLds = 1024;
  __shared__ int s_l[S * NW];
  __shared__ int s_first[kSplitLds];
  __shared__ unsigned long long s_base;
  __shared__ int s_tl;
  const int nblocks = *nblocks_dev, nsplit = *nsplit_dev;
  if ((int)blockIdx.x >= nblocks) return;  // uniform per block
  const int tid = threadIdx.x, wid = tid >> 6, l = lane_id();
  const bool lds_tab = nsplit <= kSplitLds;
  if (lds_tab) {
    for (int i = tid; i < nsplit; i += kPartThreads) s_first[i] = first_blk[i];
    __syncthreads();
  }
  const unsigned long long lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  struct Chunk { int si, beg, end, nbeg, nend, fs, th, keep; };
  auto locate = [&](int bid) {
    int lo = 0, hi = nsplit - 1;  // last split with first_blk <= bid
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((lds_tab ? s_first[mid] : first_blk[mid]) <= bid) lo = mid; else hi = mid - 1;
    }
    Chunk c;
    c.si = lo;
    const int fb = first_blk[lo], nbeg = node_begin[lo], ncnt = node_count[lo];
    c.fs = feat[lo];
    const int tr = thr[lo];
    c.th = tr & kThrMask;
    c.keep = (int)((unsigned)tr >> kKeepShift);
    c.beg = nbeg + (bid - fb) * CH;
    c.end = min(c.beg + CH, nbeg + ncnt);
    c.nbeg = nbeg;
    c.nend = nbeg + ncnt;
    return c;
  };
  auto load_rows = [&](const Chunk& c, int (&r)[S]) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int pos = c.beg + j * kPartThreads + tid;
      r[j] = pos < c.end ? (rows ? rows[pos] : pos) : 0;
    }
  };
  auto load_gh = [&](const Chunk& c, const int (&r)[S], float2 (&g)[S]) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int pos = c.beg + j * kPartThreads + tid;
      g[j] = (pos < c.end && ghp) ? ghp[gh_rows ? r[j] : pos] : make_float2(0.f, 0.f);
    }
  };
  int bid = (int)blockIdx.x;
  Chunk c = locate(bid);
  int r[S];
  load_rows(c, r);
  float2 g[S];
  if (kGh) load_gh(c, r, g);
  // kCol: the next chunk's split-feature bytes are gathered before this chunk's scatter
  // (its row ids have arrived by then), so a chunk starts with all its loads done
  int cb[kCol ? S : 1];
  auto load_col = [&](const Chunk& c, const int (&r)[S], int (&cb)[S]) {
    const BinT* col = binsT + (size_t)c.fs * ncol;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int pos = c.beg + j * kPartThreads + tid;
      cb[j] = pos < c.end ? (int)col[(unsigned)r[j]] : 0x7fffffff;
    }
  };
  if constexpr (kCol) load_col(c, r, cb);
  // kMode 3: per-wave partial prefixes of the current chunk
  __shared__ unsigned long long s_red[NW];
  while (true) {
    bool left[S];
    // kMode 3: this thread's share of the chunk's prefix in flight first (the counts and group
    // sums the previous launch wrote); reduced after the next chunk's loads are issued
    unsigned long long pv[kPreLoads];
    if constexpr (kMode == 3) {
      const ChunkRange cr(lds_tab ? s_first[c.si] : first_blk[c.si], bid);
#pragma unroll
      for (int k = 0; k < kPreLoads; ++k) {
        const int t = tid + k * kPartThreads;
        pv[k] = t < cr.ntot ? *cr.item(chunk_io, gsum, t) : 0ull;
      }
      for (int t = tid + kPreLoads * kPartThreads; t < cr.ntot; t += kPartThreads)
        pv[0] += *cr.item(chunk_io, gsum, t);  // splits beyond ~25M rows
    }
    if (!kGh) load_gh(c, r, g);
    if constexpr (kCol) {
#pragma unroll
      for (int j = 0; j < S; ++j) left[j] = cb[j] <= c.th;
    } else {
      const BinT* col = binsT + (size_t)c.fs * ncol;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const int pos = c.beg + j * kPartThreads + tid;
        left[j] = pos < c.end && (int)col[(unsigned)r[j]] <= c.th;
      }
    }
    // next chunk: locate it and put its row-id (kGh: and (g, h)) loads in flight now
    const int nbid = bid + (int)gridDim.x;
    const bool more = nbid < nblocks;  // uniform per block
    Chunk cn = c;
    int rn[S];
    float2 gn[kGh ? S : 1];
    if (more) {
      cn = locate(nbid);
      load_rows(cn, rn);
      if constexpr (kGh) {
        if (!gh_rows) load_gh(cn, rn, gn);
      }
    }
    if constexpr (kMode == 3) {
      unsigned long long part = pv[0];
#pragma unroll
      for (int k = 1; k < kPreLoads; ++k) part += pv[k];
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) part += __shfl_xor(part, off, kWave);
      if (l == 0) s_red[wid] = part;
    }
    int lrank[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const unsigned long long lm = __ballot(left[j]);
      lrank[j] = __popcll(lm & lt_mask);
      if (l == 0) s_l[j * NW + wid] = __popcll(lm);
    }
    __syncthreads();
    if (wid == 0) {
      const int x = l < S * NW ? s_l[l] : 0;
      int incl = x;
#pragma unroll
      for (int off = 1; off < S * NW; off <<= 1) {
        const int y = __shfl_up(incl, off, kWave);
        if (l >= off) incl += y;
      }
      if (l < S * NW) s_l[l] = incl - x;
      const int tl_all = __shfl(incl, S * NW - 1, kWave);
      if (l == 0) {
        const int tv = c.end - c.beg;
        const unsigned long long cnt = ((unsigned long long)(tv - tl_all) << 32) | (unsigned long long)tl_all;
        if constexpr (kMode == 2) s_base = chunk_io[bid];
        else if constexpr (kMode == 3) {
          unsigned long long pre = 0ull;
#pragma unroll
          for (int w = 0; w < NW; ++w) pre += s_red[w];
          s_base = pre;
        }
        else s_base = atomicAdd(&cursor[(size_t)c.si * cs], cnt);
        s_tl = tl_all;
      }
    }
    __syncthreads();
    if constexpr (kCol) {
      if (more) load_col(cn, rn, cb);
    }
    if constexpr (kGh) {
      if (gh_rows && more) load_gh(cn, rn, gn);
    }
    {
      const int tl = s_tl;
      const int tv = c.end - c.beg;
      const unsigned long long base = s_base;
      const int lofs = (int)(base & 0xffffffffull), rofs = (int)(base >> 32);
      const int sh = out_shift ? out_shift[c.si] : 0;
      const int rstart = c.nend - rofs - (tv - tl) + sh;
      const int lstart = c.nbeg + lofs + sh;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const int rank = j * kPartThreads + tid;
        if (rank < tv) {
          const int lb = s_l[j * NW + wid] + lrank[j];
          const int dst = left[j] ? lstart + lb : rstart + (rank - lb);
          if (keep_row(c.keep, left[j])) {
            rows_out[dst] = r[j];
            if (gh_out) gh_out[dst] = g[j];
          }
        }
      }
    }
    __syncthreads();  // s_l / s_base / s_tl are reused by the next chunk
    if (!more) break;
    bid = nbid;
    c = cn;
#pragma unroll
    for (int j = 0; j < S; ++j) r[j] = rn[j];
    if constexpr (kGh) {
#pragma unroll
      for (int j = 0; j < S; ++j) g[j] = gn[j];
    }
  }
}

// Lean count pass (the scan path's first kernel): ONE block per 2048-row chunk, the chunk
// geometry of partition_atomic_body_pf (S = kAtomSub rows per thread), no persistence, no
// prefetch pipeline -- each thread's row ids (or positions) and split-feature bytes in flight
// at once, the left rows popcounted per wave -> chunk_io[chunk] = (right << 32) | left. (The
// partition body in count mode walked ~2.5 chunks per persistent block: 14 us at the root.)
__device__ __forceinline__ void part_count_lean_body(const uint8_t* __restrict__ binsT, long long ncol,
                                                     const int* __restrict__ rows, const int* __restrict__ first_blk,
                                                     const int* __restrict__ nsplit_dev,
                                                     const int* __restrict__ nblocks_dev, const int* __restrict__ feat,
                                                     const int* __restrict__ thr, const int* __restrict__ node_begin,
                                                     const int* __restrict__ node_count,
                                                     unsigned long long* __restrict__ chunk_io,
                                                     unsigned long long* __restrict__ gsum) {
  constexpr int S = kAtomSub, NW = kPartThreads / kWave, CH = S * kPartThreads;
  __shared__ int s_c[NW];
  const int bid = (int)blockIdx.x;
  if (bid >= *nblocks_dev) return;  // uniform per block
  const int nsplit = *nsplit_dev;
  int lo = 0, hi = nsplit - 1;  // last split with first_blk <= bid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first_blk[mid] <= bid) lo = mid; else hi = mid - 1;
  }
  const int nbeg = node_begin[lo], fb = first_blk[lo];
  const int beg = nbeg + (bid - fb) * CH, end = min(beg + CH, nbeg + node_count[lo]);
  const uint8_t* col = binsT + (size_t)feat[lo] * ncol;
  const int th = thr[lo] & kThrMask;
  const int tid = threadIdx.x;
  int r[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int pos = beg + j * kPartThreads + tid;
    r[j] = pos < end ? (rows ? rows[pos] : pos) : -1;
  }
  int cb[S];  // every split-feature byte in flight before the first ballot waits on one
#pragma unroll
  for (int j = 0; j < S; ++j) cb[j] = r[j] >= 0 ? (int)col[(unsigned)r[j]] : 0x7fffffff;
  int nl = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) nl += __popcll(__ballot(cb[j] <= th));
  if (lane_id() == 0) s_c[tid >> 6] = nl;
  __syncthreads();
  if (tid == 0) {
    int tl = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) tl += s_c[w];
    const unsigned long long v = ((unsigned long long)(unsigned)(end - beg - tl) << 32) | (unsigned)tl;
    chunk_io[bid] = v;
    if (gsum) atomicAdd(&gsum[bid >> kGrpShift], v);  // non-returning; 32 blocks per line
  }
}

// The split cursors' (right << 32) | left totals from the raw per-chunk counts (kMode 3: the
// partition kernel's last block, before its children planning reads them). Per split, one
// strided block reduction over its chunks.
template <int kThreads>
__device__ __forceinline__ void part_split_totals(const unsigned long long* __restrict__ chunk_io,
                                                  unsigned long long* __restrict__ gsum,
                                                  const int* __restrict__ first_blk, const int* __restrict__ nsplit_dev,
                                                  const int* __restrict__ nblocks_dev,
                                                  unsigned long long* __restrict__ cursor, int cs) {
  constexpr int NW = kThreads / kWave;
  __shared__ unsigned long long s_t[NW];
  const int nsplit = *nsplit_dev, nblocks = *nblocks_dev;
  const int tid = threadIdx.x, wid = tid >> 6, l = lane_id();
  for (int si = 0; si < nsplit; ++si) {
    const int f0 = first_blk[si], f1 = si + 1 < nsplit ? first_blk[si + 1] : nblocks;
    const ChunkRange cr(f0, f1);
    unsigned long long part = 0ull;
    for (int t = tid; t < cr.ntot; t += kThreads) part += *cr.item(chunk_io, gsum, t);
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) part += __shfl_xor(part, off, kWave);
    if (l == 0) s_t[wid] = part;
    __syncthreads();
    if (tid == 0) {
      unsigned long long t = 0ull;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += s_t[w];
      cursor[(size_t)si * cs] = t;
    }
    __syncthreads();
  }
  // every block has read the group sums: zero them for the next count pass
  for (int g = tid; g <= (nblocks - 1) >> kGrpShift; g += kThreads) gsum[g] = 0ull;
}

// One block: exclusive scan of the lean count pass's chunk counts within each split (chunks of split si:
// [first_blk[si], first_blk[si + 1])), in chunk order -> chunk_io[chunk] = (right rows before
// it << 32) | left rows before it; cursor[si * cs] = the split's (right << 32) | left totals
// (what the atomic mode leaves there). One pass: each thread scans a contiguous run of chunks
// (left and right rows as two packed 32-bit sums in one u64: neither half overflows), the run
// totals are scanned across the block, and every chunk's global prefix is rebased to its
// split's first chunk.
// 256 threads (one small block, not a whole CU: a 1024-thread block at ~120 VGPRs needs a CU
// with no other wave on it, which ranks sharing one GPU -- a peer exchange spinning on every
// CU it was given -- may never leave free: the 2-rank leaf-wise test deadlocked with it)
constexpr int kChunkScanThreads = 256;
constexpr int kChunkScanMaxSplits = 256;  // the caller's levels (a few splits each) stay below
__device__ __forceinline__ void part_chunk_scan_body(unsigned long long* __restrict__ chunk_io,
                                                     const int* __restrict__ first_blk, const int* __restrict__ nsplit_dev,
                                                     const int* __restrict__ nblocks_dev,
                                                     unsigned long long* __restrict__ cursor, int cs) {
  constexpr int NW = kChunkScanThreads / kWave;
  constexpr int kRun = 32;  // chunks per thread held in registers (8K chunks per pass)
  __shared__ unsigned long long s_w[NW + 1];
  __shared__ unsigned long long s_sb[kChunkScanMaxSplits + 1];
  __shared__ int s_sf[kChunkScanMaxSplits + 1];
  const int nblocks = *nblocks_dev, nsplit = *nsplit_dev;
  const int tid = threadIdx.x, wid = tid >> 6, l = lane_id();
  for (int si = tid; si < nsplit; si += kChunkScanThreads) s_sf[si] = first_blk[si];
  if (tid == 0) s_sf[nsplit] = nblocks;
  if (nblocks <= kChunkScanThreads * kRun) {
    // one pass (<= 8K chunks): the run prefixes stay in registers; the owners of each split's
    // first chunk publish its prefix, every chunk is rebased and stored once
    const int i0 = tid * kRun;
    unsigned long long v[kRun], run = 0ull;
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      v[k] = i0 + k < nblocks ? chunk_io[i0 + k] : 0ull;
      run += v[k];
    }
    unsigned long long inc = run;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned long long u = __shfl_up(inc, off, kWave);
      if (l >= off) inc += u;
    }
    if (l == kWave - 1) s_w[wid] = inc;
    __syncthreads();  // also orders s_sf
    unsigned long long pre = 0ull, tot = 0ull;
    for (int w = 0; w < NW; ++w) {
      if (w < wid) pre += s_w[w];
      tot += s_w[w];
    }
    pre += inc - run;
    // v[k] <- the exclusive prefix of chunk i0 + k; publish split first-chunk prefixes
    int lo = 0;  // split of chunk i0 (then advanced along the run)
    {
      int hi = nsplit - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_sf[mid] <= i0) lo = mid; else hi = mid - 1;
      }
    }
    int sk[kRun];
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      const unsigned long long c = v[k];
      v[k] = pre;
      pre += c;
      while (lo + 1 < nsplit && s_sf[lo + 1] <= i0 + k) ++lo;
      sk[k] = lo;
      // the chunk opens split lo -- and every empty split before it that starts here too
      for (int t = lo; t >= 0 && i0 + k < nblocks && s_sf[t] == i0 + k; --t) s_sb[t] = v[k];
    }
    if (tid == 0) s_sb[nsplit] = tot;
    for (int si = tid; si < nsplit; si += kChunkScanThreads)
      if (s_sf[si] >= nblocks) s_sb[si] = tot;  // splits without chunks
    __syncthreads();
    for (int si = tid; si < nsplit; si += kChunkScanThreads)
      cursor[(size_t)si * cs] = s_sb[si + 1] - s_sb[si];
#pragma unroll
    for (int k = 0; k < kRun; ++k)
      if (i0 + k < nblocks) chunk_io[i0 + k] = v[k] - s_sb[sk[k]];
    return;
  }
  unsigned long long carry = 0ull;  // packed (right, left) rows of the chunks before this pass
  for (int base = 0; base < nblocks; base += kChunkScanThreads * kRun) {
    const int i0 = base + tid * kRun;
    unsigned long long v[kRun], run = 0ull;
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      v[k] = i0 + k < nblocks ? chunk_io[i0 + k] : 0ull;
      run += v[k];
    }
    unsigned long long inc = run;  // inclusive wave scan of the runs
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned long long u = __shfl_up(inc, off, kWave);
      if (l >= off) inc += u;
    }
    if (l == kWave - 1) s_w[wid] = inc;
    __syncthreads();
    unsigned long long pre = carry;
    for (int w = 0; w < wid; ++w) pre += s_w[w];
    pre += inc - run;  // exclusive prefix of this thread's run
    unsigned long long tot = carry;
    for (int w = 0; w < NW; ++w) tot += s_w[w];
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      if (i0 + k < nblocks) chunk_io[i0 + k] = pre;
      pre += v[k];
    }
    carry = tot;
    __syncthreads();  // s_w is rewritten by the next pass
  }
  __syncthreads();  // every global prefix is stored
  // per split: the prefix at its first chunk (the rebase value) and its totals (the prefix at
  // the next split's first chunk, the grand totals for the last)
  for (int si = tid; si <= nsplit; si += kChunkScanThreads) {
    const int f0 = s_sf[si];
    s_sb[si] = f0 < nblocks ? chunk_io[f0] : carry;
  }
  __syncthreads();  // every rebase value is read before any chunk is rewritten
  for (int si = tid; si < nsplit; si += kChunkScanThreads)
    cursor[(size_t)si * cs] = s_sb[si + 1] - s_sb[si];  // both halves: no borrow (prefixes grow)
  for (int i = tid; i < nblocks; i += kChunkScanThreads) {
    int lo = 0, hi = nsplit - 1;  // the chunk's split: the last with first_blk <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_sf[mid] <= i) lo = mid; else hi = mid - 1;
    }
    chunk_io[i] -= s_sb[lo];
  }
}

}  // namespace ytk
