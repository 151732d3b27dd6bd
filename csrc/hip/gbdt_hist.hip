// GBDT histogram build (gfx950 / CDNA4, wave64) -- exact int64 fixed point.
//
// Reference semantics: J/data/gbdt/HistogramBuilder.java:56-90 (sum of (g, h) per
// (feature, bin) over the rows of a node; the reference accumulates in double).
//
// Why fixed point: on gfx950 `ds_add_f32` measured ~33x slower than `ds_add_u32`
// for the same conflict-free pattern (profiles/hist_ablation.md). Each (g, h) is
// scaled by a per-tree power of two (2^k chosen so |sum over all rows| < 2^62) and
// rounded to int64 once; sums are then EXACT integers:
//   * deterministic and order independent (bitwise identical on 1 and N GPUs,
//     all-reduce of int64 is exact);
//   * parent - small child = large child exactly;
//   * resolution 2^-k ~ 1e-12 x max|g| -- finer than the fp32 gradients themselves.
//
// Layout / mapping:
//   * LDS: two int64 planes lds[bin][32] (g, h): 128 KiB at 256 bins, 1 block/CU,
//     1024 threads (16 waves).
//   * lane = (row r = lane/8, q = lane%8): one dword load = 4 features of a row, a
//     wave-instruction moves 8 rows x 32 B = 256 B; step k updates feature
//     4q + ((k + r) & 3) so the 32 lanes of each half-wave hit 32 distinct banks.
//   * (g, h) is read in POSITION order (the partition moves it with the row ids).
//   * One launch covers every node of a level: work[blk] = (slot, begin, end, 0).
//   * Block partials -> global int64 atomics (zero entries skipped).
#include "common.h"
#include "gbdt_fx.h"

#include <algorithm>
#include <stdexcept>

namespace ytk {

constexpr int kHistThreads = 1024;

// 8 rows per lane in flight (12 measured: 104-107 VGPRs, root 154.6 -> 160.3 us, gathered
// levels 443.6 -> 450.6 us per tree: the loop is not short of memory-level parallelism)
constexpr int kHistU = 8;
constexpr int kHistUGather = 8;  // gathered rows (pipelined: rows two steps ahead)

// kFW: features per block (32: one 128-KiB LDS plane pair per block, 1 block per CU; 16:
// 64 KiB, 2 blocks per CU with twice the rows in flight -- every row is read by both
// feature-half blocks, 16 B each)
template <bool kIdentity, int kFW = 32>
__global__ __launch_bounds__(kHistThreads) void hist_fx_kernel(
    const uint8_t* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B, int nb_lds,
    float sg, float sh, const int* __restrict__ nwork_dev, const float* __restrict__ scales_dev,
    long long* __restrict__ staging, const int* __restrict__ work_off_dev, int gh_rows) {
  // gh_rows: (g, h) is indexed by ROW id (the level engine's first gathered level: the root
  // partition moved only the row ids), else by position
  // LDS bin rows of 64 words: [32 g words | 32 h words]; the h atomic of a (bin, feature)
  // is the g address + 256 B (instruction offset), both conflict-free (hist_lds_pos)
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm64[];
  // device-resident work count (fixed maximal grid launched by the level engine)
  // work_off_dev (optional): this launch covers work items [*work_off_dev, *nwork_dev) --
  // the second half of a level whose first half is already being all-reduced
  const int bx = (int)blockIdx.x + (work_off_dev ? *work_off_dev : 0);
  if (nwork_dev && bx >= *nwork_dev) return;
  if (scales_dev) {
    sg = scales_dev[0];
    sh = scales_dev[1];
  }
  const int4 w = work[bx];
  const int fg = blockIdx.y;
  const int tid = threadIdx.x;
  constexpr int kRow = 2 * kFW;  // LDS words per bin row: [kFW g | kFW h]
  for (int i = tid; i < nb_lds * kRow; i += kHistThreads) sm64[i] = 0ull;
  __syncthreads();

  const int wave = tid >> 6;
  const int lane = tid & 63;
  constexpr int kQ = kFW / 4;          // lanes per row (one dword = 4 features each)
  const int wr = lane / kQ;             // row within the wave's 64 / kQ
  const int q = lane % kQ;              // dword (4 features) within the group's segment
  constexpr int RW = (kHistThreads / 64) * (64 / kQ);  // rows per block step
  const uint8_t* bseg = bins + fg * kFW + 4 * q;
  // LDS word of local feature 4q + c inside a bin row (hist_lds_pos: bank-conflict-free
  // 64-bit atomics)
  int lpos[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) lpos[c] = kFW == 32 ? hist_lds_pos(4 * q + c) : 4 * q + c;
  // 16-feature blocks hold twice the rows per wave instruction: half the unroll keeps the
  // rows in flight per wave and fits 2 blocks (32 waves) per CU in the VGPR budget
  constexpr int U = (kIdentity ? kHistU : kHistUGather) / (kFW == 16 ? 2 : 1);
  constexpr int STEP = RW * U;
  // Software pipeline: the bin dwords and (g, h) of step i+1 are in flight while step i
  // is accumulated into LDS (measured: the un-pipelined loop left the kernel latency
  // bound at ~2.2 TB/s with LDS only ~36 % busy). Gathered rows are loaded one further
  // step ahead so the dependent bin loads of step i+1 never wait on their row ids.
  auto load_rows = [&](int base, int (&r)[U]) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int pos = base + j * RW + wr;
      const int p = pos < w.z ? pos : w.y;
      r[j] = kIdentity ? p : rows[p];
    }
  };
  auto load_data = [&](int base, const int (&r)[U], unsigned (&d)[U], float2 (&v)[U], bool (&ok)[U]) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int pos = base + j * RW + wr;
      ok[j] = pos < w.z;
      const int p = ok[j] ? pos : w.y;
      d[j] = *reinterpret_cast<const unsigned*>(bseg + (size_t)(unsigned)r[j] * stride);
      const float2 t = ghp[gh_rows ? r[j] : p];
      v[j] = ok[j] ? t : make_float2(0.f, 0.f);  // rows past the end add 0
    }
  };
  const int base0 = w.y + wave * (64 / kQ);
  unsigned d[U];
  float2 v[U];
  bool ok[U];
  int rn[U];
  if (base0 < w.z) {
    int r0[U];
    load_rows(base0, r0);
    load_data(base0, r0, d, v, ok);
    load_rows(base0 + STEP, rn);
  }
  for (int base = base0; base < w.z; base += STEP) {
    unsigned dn[U];
    float2 vn[U];
    bool okn[U];
    const bool more = base + STEP < w.z;  // wave-uniform
    if (more) {
      load_data(base + STEP, rn, dn, vn, okn);
      load_rows(base + 2 * STEP, rn);
    }
    // Branch-free inner body (the VALU, not LDS or memory, bounds this loop: measured
    // ~60 VALU per 8-row step with a guarded body): rows past the end add 0, features
    // >= F (bin-row padding, bin 0) land in LDS columns the flush never reads.
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const unsigned long long gi = fx_round(v[j].x * sg);
      const unsigned long long hi = fx_round(v[j].y * sh);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = (k + wr) & 3;
        const unsigned bin = __builtin_amdgcn_ubfe(d[j], 8 * c, 8);
        unsigned long long* e = sm64 + (bin * kRow + lpos[c]);
        atomicAdd(e, gi);
        atomicAdd(e + kFW, hi);
      }
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        d[j] = dn[j];
        v[j] = vn[j];
        ok[j] = okn[j];
      }
    }
  }
  __syncthreads();

  if (staging && w.w == 1) {
    // the slot's ONLY item (leaf-wise engine, small nodes): store the block's sums straight
    // into the slot -- no staging round trip, no zero fill, no reduce
    long long* out = hist + (size_t)w.x * B * F * 2;
    const int E = nb_lds * kFW;
    for (int i = tid; i < E; i += kHistThreads) {
      const int bin = i / kFW, l = i % kFW, ff = fg * kFW + l;
      if (ff < F && bin < B) {
        const int li = bin * kRow + (kFW == 32 ? hist_lds_pos(l) : l);
        *reinterpret_cast<longlong2*>(&out[((size_t)bin * F + ff) * 2]) =
            make_longlong2((long long)sm64[li], (long long)sm64[li + kFW]);
      }
    }
    return;
  }
  if (staging) {
    // two-stage flush: plain 16-B stores of this block's partial (g, h) pairs; the slot
    // sums are formed by hist_reduce_kernel. Global u64 atomics execute at the memory
    // side at ~1.3 TB/s chip-wide, which made the atomic flush the floor of every
    // launch (~45 us per level at 256 blocks); stores + one ordered read are ~4x cheaper.
    const int E = nb_lds * kFW;
    longlong2* st = reinterpret_cast<longlong2*>(staging) + ((size_t)bx * gridDim.y + fg) * E;
    const int fw = min(kFW, F - fg * kFW);  // features of this group (the reduce reads no padding)
    for (int i = tid; i < E; i += kHistThreads) {
      const int l = i % kFW;
      if (l >= fw) continue;
      const int li = (i / kFW) * kRow + (kFW == 32 ? hist_lds_pos(l) : l);
      st[i] = make_longlong2((long long)sm64[li], (long long)sm64[li + kFW]);
    }
    if (w.w == 2 && fg == 0) {
      // first item of a slot the split-K reduce adds into (leaf-wise engine): zero it
      // here instead of in a separate launch (the reduce runs after this kernel)
      longlong2* hs = reinterpret_cast<longlong2*>(hist + (size_t)w.x * B * F * 2);
      for (int i = tid; i < B * F; i += kHistThreads) hs[i] = make_longlong2(0, 0);
    }
    return;
  }
  long long* out = hist + (size_t)w.x * B * F * 2;
  // Flush order rotated per block: every block of a level flushes into the SAME few
  // thousand addresses at about the same time; starting each block at a different
  // 1024-entry tile spreads the global atomics over the L2 channels instead of
  // serialising hundreds of blocks on one address at a time.
  const int E = nb_lds * kFW;
  const int ntile = (E + kHistThreads - 1) / kHistThreads;
  const int rot = (int)((unsigned)bx % (unsigned)ntile);
  for (int t = 0; t < ntile; ++t) {
    const int i = ((t + rot) % ntile) * kHistThreads + tid;
    if (i >= E) continue;
    const int bin = i / kFW, l = i % kFW, ff = fg * kFW + l;
    if (ff < F) {
      const int li = bin * kRow + (kFW == 32 ? hist_lds_pos(l) : l);
      const unsigned long long g = sm64[li], h = sm64[li + kFW];
      if (g | h) {
        unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)bin * F + ff) * 2]);
        atomicAdd(o, g);
        atomicAdd(o + 1, h);
      }
    }
  }
}

// Second stage of the staged flush: hist[slot][bin][f] = sum over the work items of that
// slot of their block partials. One thread per (entry, slot, feature group); the items of
// the slot are collected into LDS first (<= 1024 items per level). Integer sums: exact and
// order independent. Every slot in [slot_base, slot_base + nslots) is written (zero when
// it has no items), so the built half of a level needs no zero fill.
// Split-K over the slot's items (blockIdx.z of kReduceSplit): each block sums a strided
// subset of the items with 8 independent 16-B loads in flight per thread and adds its
// partial with one int64 atomic per value (exact; kReduceSplit-way contention only).
// The slots must be zero on entry.
constexpr int kReduceSplit = 8;
constexpr int kReduceDirect = 16;  // ranged slots with <= this many items: one block, plain stores

template <int U = 8>  // staged partials in flight per thread (YTK_REDUCE_U = 8 | 16)
__global__ __launch_bounds__(256) void hist_reduce_kernel(
    const long long* __restrict__ staging, const int4* __restrict__ work, int nwork,
    const int* __restrict__ nwork_dev, long long* __restrict__ hist, int B, int F, int nb_lds,
    int groups, int slot_base, const int* __restrict__ slot_ids, const int* __restrict__ nslots_dev,
    const int2* __restrict__ slot_range, int gw, const int* __restrict__ slot_first = nullptr, int one_slot = 0) {
  // slot_first (optional): slot slot_base + k owns the items [slot_first[k], slot_first[k + 1])
  // (the level engine's hist_first); one_slot: every item belongs to the one slot -- either
  // way no scan of the work list
  __shared__ int s_sel[1024];
  __shared__ int s_wcnt[4];
  __shared__ int s_n;
  const int n = nwork_dev ? min(*nwork_dev, nwork) : nwork;
  // nslots_dev (optional): device-resident slot count (leaf-wise engine); the grid's y
  // blocks then stride over the slots. Without it every y block owns one slot.
  const int ny = nslots_dev ? *nslots_dev * groups : (int)gridDim.y;
  __shared__ int s_lo, s_hi, s_cnt;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (slot_range) {
    // ranged slots (leaf-wise engine): items [x, x + y) of each listed slot, no scan, no
    // barriers. Slots with <= kReduceDirect items are summed by the z == 0 block and
    // STORED (zeros included: no zero fill needed); larger ones split-K with atomics into
    // a zeroed slot.
    const int E = nb_lds * gw;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int bin = i / gw;
    if (i >= E || bin >= B) return;
    const longlong2* st = reinterpret_cast<const longlong2*>(staging);
    for (int by = (int)blockIdx.y; by < ny; by += (int)gridDim.y) {
      const int2 r = slot_range[by / groups];
      const int fg = by % groups, ff = fg * gw + (i % gw);
      if (ff >= F) continue;
      const bool direct = r.y <= kReduceDirect;
      if (direct && blockIdx.z != 0) continue;
      const int step = direct ? 1 : (int)gridDim.z;  // split-K factor (launch z extent)
      long long g = 0, h = 0;
      int t = direct ? 0 : (int)blockIdx.z;
      for (; t + (U - 1) * step < r.y; t += U * step) {
        longlong2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = st[((size_t)(r.x + t + u * step) * groups + fg) * E + i];
#pragma unroll
        for (int u = 0; u < U; ++u) { g += v[u].x; h += v[u].y; }
      }
      for (; t < r.y; t += step) {
        const longlong2 v = st[((size_t)(r.x + t) * groups + fg) * E + i];
        g += v.x;
        h += v.y;
      }
      const int slot = slot_ids[by / groups];
      long long* o = hist + (((size_t)slot * B + bin) * F + ff) * 2;
      if (direct) {
        *reinterpret_cast<longlong2*>(o) = make_longlong2(g, h);
      } else if (g | h) {
        atomicAdd(reinterpret_cast<unsigned long long*>(o), (unsigned long long)g);
        atomicAdd(reinterpret_cast<unsigned long long*>(o) + 1, (unsigned long long)h);
      }
    }
    return;
  }
  for (int by = (int)blockIdx.y; by < ny; by += (int)gridDim.y) {
  __syncthreads();  // the previous slot's s_sel / s_lo are still being read
  // slot_ids (optional): explicit, possibly non-contiguous target slots (recycled slot pool)
  const int slot = slot_ids ? slot_ids[by / groups] : slot_base + by / groups;
  const int fg = by % groups;
  // Ordered (stable) compaction of this slot's items: the kReduceSplit blocks of a slot
  // each take a strided subset s_sel[z], s_sel[z + 8], ..., so every block must see the
  // SAME order (an LDS-atomic compaction orders items differently per block whenever a
  // slot's items straddle waves, dropping and double counting items).
  // Fast path: every caller emits a slot's items contiguously -> one pass finds the
  // range [lo, hi] (min/max of matching indices) and the match count; contiguous iff
  // count == hi - lo + 1. Otherwise fall back to the ordered compaction below.
  const bool known = slot_first != nullptr || one_slot;  // uniform
  int known_lo = 0, known_cnt = n;
  if (slot_first) {
    known_lo = slot_first[by / groups];
    known_cnt = slot_first[by / groups + 1] - known_lo;
  }
  if (tid == 0) { s_n = 0; s_lo = 0x7fffffff; s_hi = -1; s_cnt = 0; }
  __syncthreads();
  // slot_range (optional): the slot's items are [x, x + y) -- no scan of the work list
  for (int k0 = 0; !known && k0 < n; k0 += 256) {  // one LDS atomic per wave, not per item
    const int k = k0 + tid;
    const unsigned long long bal = __ballot(k < n && work[k].x == slot);
    if (lane == 0 && bal) {
      const int wbase = k0 + wid * 64;
      atomicMin(&s_lo, wbase + __ffsll((long long)bal) - 1);
      atomicMax(&s_hi, wbase + 63 - __clzll((long long)bal));
      atomicAdd(&s_cnt, __popcll(bal));
    }
  }
  __syncthreads();
  const bool contiguous = known || s_cnt == 0 || s_cnt == s_hi - s_lo + 1;
  if (contiguous && !known) {
    if (tid == 0) s_n = s_cnt;
  }
  for (int k0 = 0; !contiguous && k0 < n; k0 += 256) {
    const int k = k0 + tid;
    const bool m = k < n && work[k].x == slot;
    const unsigned long long bal = __ballot(m);
    if (lane == 0) s_wcnt[wid] = __popcll(bal);
    __syncthreads();
    int off = s_n;
    for (int w = 0; w < wid; ++w) off += s_wcnt[w];
    const int p = off + __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    if (m && p < 1024) s_sel[p] = k;
    __syncthreads();
    if (tid == 0) s_n += s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    __syncthreads();
  }
  __syncthreads();
  const int cnt = known ? known_cnt : contiguous ? s_n : min(s_n, 1024);
  const int lo = known ? known_lo : s_lo;
  // t-th item of the slot
#define YTK_SEL(t) (contiguous ? lo + (t) : s_sel[(t)])
  const int E = nb_lds * gw;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E || cnt == 0) continue;
  const int bin = i / gw, ff = fg * gw + (i % gw);
  if (ff >= F || bin >= B) continue;
  // few items (deep levels: many slots, ~hist_target / slots items each): the z == 0
  // block sums them all and STORES -- no 8-way int64 atomics at the memory side
  const bool direct = cnt <= kReduceDirect;
  if (direct && blockIdx.z != 0) continue;
  const int step = direct ? 1 : (int)gridDim.z;  // split-K factor (launch z extent)
  const longlong2* st = reinterpret_cast<const longlong2*>(staging);
  long long g = 0, h = 0;
  int t = direct ? 0 : (int)blockIdx.z;
  for (; t + (U - 1) * step < cnt; t += U * step) {
    longlong2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = st[((size_t)YTK_SEL(t + u * step) * groups + fg) * E + i];
#pragma unroll
    for (int u = 0; u < U; ++u) { g += v[u].x; h += v[u].y; }
  }
  for (; t < cnt; t += step) {
    const longlong2 v = st[((size_t)YTK_SEL(t) * groups + fg) * E + i];
    g += v.x;
    h += v.y;
  }
  if (direct) {
    *reinterpret_cast<longlong2*>(hist + (((size_t)slot * B + bin) * F + ff) * 2) = make_longlong2(g, h);
  } else if (g | h) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(hist + (((size_t)slot * B + bin) * F + ff) * 2);
    atomicAdd(o, (unsigned long long)g);
    atomicAdd(o + 1, (unsigned long long)h);
  }
  }
}
#undef YTK_SEL

// Generic histogram (uint8 or uint16 bins, any bin count): direct global int64
// atomics. Fallback for > 256 bins (e.g. the 5000-bin communication-stress config).
template <typename BinT>
__global__ __launch_bounds__(256) void hist_fx_global_kernel(
    const BinT* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B, float sg, float sh) {
  const int4 w = work[blockIdx.x];
  const long long n = (long long)(w.z - w.y) * F;
  long long* out = hist + (size_t)w.x * B * F * 2;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const int pos = w.y + (int)(i / F);
    const int f = (int)(i % F);
    const int r = rows ? rows[pos] : pos;
    const int b = bins[(long long)r * stride + f];
    const float2 v = ghp[pos];
    unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)b * F + f) * 2]);
    atomicAdd(o, (unsigned long long)__float2ll_rn(v.x * sg));
    atomicAdd(o + 1, (unsigned long long)__float2ll_rn(v.y * sh));
  }
}

// Wide-bin histogram (B > 256, uint16 bins -- e.g. the 5000-bin communication-stress
// config, docs/gbdt_experiments.md:156-168; reference loop HistogramBuilder.java:56-90).
// The 32-feature x B-bin LDS planes of hist_fx_kernel do not fit, so a block owns a
// GROUP of FG features (FG = floor(LDS budget / (B * 16 B)), >= 1) and reads their
// bins from the COLUMN-major matrix binsT [F][ncol] (2 B per row per feature,
// coalesced for the identity root, monotone row ids inside a node otherwise).
// LDS holds two exact int64 planes g[f_in_group * B + bin], h[...] (separate planes: a
// 64-bit word index e uses bank pair e mod 16, interleaving would leave half unused),
// accumulated with ds_add_u64 (same fixed point as hist_fx_kernel -> bitwise equal to
// the CPU path). Block partials are flushed with global int64 atomics, zero entries
// skipped (deep nodes touch few bins). grid: wide_grid (XCD-local feature groups per item).
constexpr int kWideThreads = 1024;
constexpr int kWideLdsBytes = 160 * 1024;    // one block per CU at the widest groups

// XCD-local (group, item) of a wide-histogram block. The grid is 1-D, groups x (work items
// rounded up to 8): blocks are dealt round-robin over the 8 XCDs, so XCD x = L % 8 runs the
// blocks L = 8 s + x, and s enumerates (item / 8, group) -- every feature group of work item
// 8 (s / groups) + x runs on that one XCD, back to back, and the row ids, (g, h) and row
// lines all groups of an item read are fetched into ONE L2 (with the groups spread over
// all XCDs each line came from HBM / MALL once per XCD). false: padding block.
__device__ __forceinline__ bool wide_block(int groups, int nwork_grid, int& g, int& item) {
  const unsigned L = blockIdx.x, s = L >> 3;
  g = (int)(s % (unsigned)groups);
  item = (int)((s / (unsigned)groups) * 8u + (L & 7u));
  return item < nwork_grid;
}

static inline dim3 wide_grid(int groups, int nwork) {
  return dim3((unsigned)((long long)groups * ((nwork + 7) / 8 * 8)));
}

// kFG features per block (power of two <= 32); every row's kFG bin loads of kU rows are
// issued together before the LDS atomics (kU * kFG = 16 loads in flight per thread).
template <bool kIdentity, int kFG>
__global__ __launch_bounds__(kWideThreads) void hist_wide_kernel(
    const uint16_t* __restrict__ binsT, long long ncol, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B,
    float sg, float sh, const int* __restrict__ nwork_dev, const float* __restrict__ scales_dev,
    const int* __restrict__ work_off_dev, long long* __restrict__ staging, int nwork_grid) {
  constexpr int kU = kFG >= 16 ? 1 : 16 / kFG;
  extern __shared__ __attribute__((aligned(16))) unsigned long long wl[];
  const int groups = (F + kFG - 1) / kFG;
  int grp, item;
  if (!wide_block(groups, nwork_grid, grp, item)) return;
  const int bx = item + (work_off_dev ? *work_off_dev : 0);
  if (nwork_dev && bx >= *nwork_dev) return;
  if (scales_dev) {
    sg = scales_dev[0];
    sh = scales_dev[1];
  }
  const int4 w = work[bx];
  const int f_lo = grp * kFG;
  const int nf = min(kFG, F - f_lo);
  const int tid = threadIdx.x;
  const int E = nf * B;
  for (int i = tid; i < 2 * E; i += kWideThreads) wl[i] = 0ull;
  __syncthreads();
  const uint16_t* col = binsT + (size_t)f_lo * ncol;
  for (int base = w.y + tid; base < w.z; base += kWideThreads * kU) {
    int r[kU];
    float2 v[kU];
    bool ok[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const int pos = base + j * kWideThreads;
      ok[j] = pos < w.z;
      const int p = ok[j] ? pos : w.y;
      r[j] = kIdentity ? p : rows[p];
      const float2 t = ghp[p];
      v[j] = ok[j] ? t : make_float2(0.f, 0.f);  // rows past the end add 0
    }
    int bn[kU][kFG];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const uint16_t* c = col + (size_t)(unsigned)r[j];
#pragma unroll
      for (int fi = 0; fi < kFG; ++fi) bn[j][fi] = (fi < nf) ? (int)c[(size_t)fi * ncol] : 0;
    }
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const unsigned long long gi = fx_round(v[j].x * sg);
      const unsigned long long hi = fx_round(v[j].y * sh);
#pragma unroll
      for (int fi = 0; fi < kFG; ++fi) {
        if (fi >= nf) break;
        const int e = fi * B + bn[j][fi];
        atomicAdd(&wl[e], gi);
        atomicAdd(&wl[E + e], hi);
      }
    }
  }
  __syncthreads();
  if (staging) {  // block partial -> staging item (bx, group), hist_reduce_kernel entry order
    const int Eg = kFG * B;
    longlong2* st = reinterpret_cast<longlong2*>(staging) + ((size_t)bx * groups + grp) * Eg;
    for (int i = tid; i < Eg; i += kWideThreads) {
      const int bin = i / kFG, fi = i - bin * kFG;
      const bool in = fi < nf;
      const int e = fi * B + bin;
      st[i] = in ? make_longlong2((long long)wl[e], (long long)wl[E + e]) : make_longlong2(0, 0);
    }
    return;
  }
  long long* out = hist + (size_t)w.x * B * F * 2;
  for (int i = tid; i < E; i += kWideThreads) {
    const unsigned long long g = wl[i], h = wl[E + i];
    if (g | h) {
      const int fi = i / B, bin = i - fi * B;
      unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)bin * F + f_lo + fi) * 2]);
      atomicAdd(o, g);
      atomicAdd(o + 1, h);
    }
  }
}

// Row-major wide-bin histogram (uint16 bins [N][stride], B > 256). Same feature groups and
// LDS planes as hist_wide_kernel, but every row's kFG bins of the group are ONE vector load
// from the row (2 kFG contiguous bytes) instead of kFG column-major gathers: on the gathered
// (deep) levels a column-major read fetched a separate 64-B sector per (row, feature), while
// the groups of one work item now share each row's 64-B line through L2. Columns past F
// are the row padding (bin 0) and are accumulated branch-free into planes the flush skips.
// staging (optional): block partials -> staging item (bx, fg) with the entry order
// bin * kFG + fi of hist_reduce_kernel (gw = kFG), reduced split-K into zeroed slots;
// otherwise global int64 atomics (zero entries skipped).
template <int kFG>
__device__ __forceinline__ void wide_load_row(const uint16_t* p, int (&b)[kFG]) {
  if constexpr (kFG == 1) {
    b[0] = p[0];
  } else if constexpr (kFG == 2) {
    const unsigned v = *reinterpret_cast<const unsigned*>(p);
    b[0] = v & 0xffff; b[1] = v >> 16;
  } else if constexpr (kFG == 4) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    b[0] = v.x & 0xffff; b[1] = v.x >> 16; b[2] = v.y & 0xffff; b[3] = v.y >> 16;
  } else {
#pragma unroll
    for (int q = 0; q < kFG / 8; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(p)[q];
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) { b[8 * q + 2 * t] = w[t] & 0xffff; b[8 * q + 2 * t + 1] = w[t] >> 16; }
    }
  }
}

template <bool kIdentity, int kFG>
__global__ __launch_bounds__(kWideThreads) void hist_wide_rm_kernel(
    const uint16_t* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B,
    float sg, float sh, const int* __restrict__ nwork_dev, const float* __restrict__ scales_dev,
    const int* __restrict__ work_off_dev, long long* __restrict__ staging, int nwork_grid) {
  constexpr int kU = kFG >= 8 ? 2 : 16 / kFG;  // rows in flight per thread
  extern __shared__ __attribute__((aligned(16))) unsigned long long wl[];
  const int groups = (F + kFG - 1) / kFG;
  int grp, item;
  if (!wide_block(groups, nwork_grid, grp, item)) return;
  const int bx = item + (work_off_dev ? *work_off_dev : 0);
  if (nwork_dev && bx >= *nwork_dev) return;
  if (scales_dev) {
    sg = scales_dev[0];
    sh = scales_dev[1];
  }
  const int4 w = work[bx];
  const int f_lo = grp * kFG;
  const int nf = min(kFG, F - f_lo);
  const int tid = threadIdx.x;
  const int E = kFG * B;
  for (int i = tid; i < 2 * E; i += kWideThreads) wl[i] = 0ull;
  __syncthreads();
  const uint16_t* base_row = bins + f_lo;
  for (int base = w.y + tid; base < w.z; base += kWideThreads * kU) {
    int r[kU];
    float2 v[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const int pos = base + j * kWideThreads;
      const bool ok = pos < w.z;
      const int p = ok ? pos : w.y;
      r[j] = kIdentity ? p : rows[p];
      const float2 t = ghp[p];
      v[j] = ok ? t : make_float2(0.f, 0.f);  // rows past the end add 0
    }
    int bn[kU][kFG];
#pragma unroll
    for (int j = 0; j < kU; ++j) wide_load_row<kFG>(base_row + (size_t)(unsigned)r[j] * stride, bn[j]);
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const unsigned long long gi = fx_round(v[j].x * sg);
      const unsigned long long hi = fx_round(v[j].y * sh);
#pragma unroll
      for (int fi = 0; fi < kFG; ++fi) {
        const int e = fi * B + bn[j][fi];
        atomicAdd(&wl[e], gi);
        atomicAdd(&wl[E + e], hi);
      }
    }
  }
  __syncthreads();
  if (staging && w.w == 1) {
    // the slot's ONLY item (leaf-wise engine): this group's columns straight into the slot
    long long* out = hist + (size_t)w.x * B * F * 2;
    for (int i = tid; i < nf * B; i += kWideThreads) {
      const int fi = i / B, bin = i - fi * B;
      *reinterpret_cast<longlong2*>(&out[((size_t)bin * F + f_lo + fi) * 2]) =
          make_longlong2((long long)wl[i], (long long)wl[E + i]);
    }
    return;
  }
  if (staging) {
    longlong2* st = reinterpret_cast<longlong2*>(staging) + ((size_t)bx * groups + grp) * E;
    for (int i = tid; i < E; i += kWideThreads) {
      const int bin = i / kFG, fi = i - bin * kFG;
      const int e = fi * B + bin;
      st[i] = make_longlong2((long long)wl[e], (long long)wl[E + e]);
    }
    if (w.w == 2) {
      // first item of a slot the split-K reduce adds into (leaf-wise engine): zero this
      // group's columns of the slot (the reduce runs after this kernel)
      long long* out = hist + (size_t)w.x * B * F * 2;
      for (int i = tid; i < nf * B; i += kWideThreads) {
        const int fi = i / B, bin = i - fi * B;
        *reinterpret_cast<longlong2*>(&out[((size_t)bin * F + f_lo + fi) * 2]) = make_longlong2(0, 0);
      }
    }
    return;
  }
  long long* out = hist + (size_t)w.x * B * F * 2;
  for (int i = tid; i < nf * B; i += kWideThreads) {
    const unsigned long long g = wl[i], h = wl[E + i];
    if (g | h) {
      const int fi = i / B, bin = i - fi * B;
      unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)bin * F + f_lo + fi) * 2]);
      atomicAdd(o, g);
      atomicAdd(o + 1, h);
    }
  }
}

}  // namespace ytk

using namespace ytk;

// features per histogram block (32 or 16), process-wide (ytk_hist_set_fw); the staging
// slabs hold groups * fw columns per bin
static int g_hist_fw = 32;
// staged partials in flight per reduce thread (YTK_REDUCE_U, read per launch: tests toggle it)
static int reduce_u() {
  const char* e = getenv("YTK_REDUCE_U");
  return (e && atoi(e) == 16) ? 16 : 8;
}

template <bool kIdentity>
static void launch_hist_fx(dim3 grid, size_t lds_unused, hipStream_t s, const uint8_t* bins, long long stride, int F,
                           const float2* ghp, const int* rows, const int4* work, long long* hist, int B, int nb_lds,
                           float sg, float sh, const int* nwork_dev, const float* scales_dev, long long* staging,
                           const int* work_off_dev, int gh_rows = 0) {
  (void)lds_unused;
  const size_t lds = (size_t)nb_lds * 2 * g_hist_fw * sizeof(unsigned long long);
  if (g_hist_fw == 16)
    hipLaunchKernelGGL((hist_fx_kernel<kIdentity, 16>), grid, dim3(kHistThreads), lds, s, bins, stride, F, ghp,
                       rows, work, hist, B, nb_lds, sg, sh, nwork_dev, scales_dev, staging, work_off_dev, gh_rows);
  else
    hipLaunchKernelGGL((hist_fx_kernel<kIdentity, 32>), grid, dim3(kHistThreads), lds, s, bins, stride, F, ghp,
                       rows, work, hist, B, nb_lds, sg, sh, nwork_dev, scales_dev, staging, work_off_dev, gh_rows);
}

extern "C" {

int ytk_hist_wide_group(int B, int F);

void ytk_hist_set_fw(int fw) {
  if (fw != 16 && fw != 32) throw std::invalid_argument("hist_set_fw: 16 or 32");
  g_hist_fw = fw;
}
int ytk_hist_get_fw() { return g_hist_fw; }

// nwork_dev / scales_dev (optional): device-resident work count (grid = nwork is the
// maximum) and fixed-point scales, used by the GPU-resident level engine.
void ytk_hist_fx(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows,
                 uintptr_t work, int nwork, uintptr_t hist, int B, float sg, float sh,
                 uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t stream) {
  if (nwork <= 0) return;
  const int fw = g_hist_fw;
  const int groups = (F + fw - 1) / fw;
  const int nb_lds = B;  // caller guarantees B <= 256
  dim3 grid(nwork, groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0)
    launch_hist_fx<true>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, nullptr,
                         (const int4*)work, (long long*)hist, B, nb_lds, sg, sh, (const int*)nwork_dev,
                         (const float*)scales_dev, nullptr, nullptr);
  else
    launch_hist_fx<false>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                          (const int4*)work, (long long*)hist, B, nb_lds, sg, sh, (const int*)nwork_dev,
                          (const float*)scales_dev, nullptr, nullptr);
  YTK_LAUNCH_CHECK();
}

// Staged variant: block partials to ``staging`` (>= nwork * groups * B * fw * 16 bytes),
// then accumulated into the slots [slot_base, slot_base + nslots) -- or slot_ids[0..nslots)
// when given -- which must be zero.
void ytk_hist_fx_staged(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows,
                        uintptr_t work, int nwork, uintptr_t hist, int B, float sg, float sh,
                        uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t staging,
                        int slot_base, int nslots, uintptr_t slot_ids, uintptr_t work_off_dev,
                        uintptr_t stream, int gh_rows, uintptr_t slot_first, int one_slot) {
  // slot_first / one_slot (optional): the slots' item ranges are known (hist_reduce_kernel)
  if (nwork <= 0 || nslots <= 0) return;
  const int fw = g_hist_fw;
  const int groups = (F + fw - 1) / fw;
  const int nb_lds = B;
  dim3 grid(nwork, groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0)
    launch_hist_fx<true>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, nullptr,
                         (const int4*)work, (long long*)hist, B, nb_lds, sg, sh, (const int*)nwork_dev,
                         (const float*)scales_dev, (long long*)staging, (const int*)work_off_dev);
  else
    launch_hist_fx<false>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                          (const int4*)work, (long long*)hist, B, nb_lds, sg, sh, (const int*)nwork_dev,
                          (const float*)scales_dev, (long long*)staging, (const int*)work_off_dev, gh_rows);
  YTK_LAUNCH_CHECK();
  const int E = nb_lds * fw;
  // split-K factor (YTK_REDUCE_SPLIT overrides; exact int64 atomics, so the sums do not
  // depend on it). 32 / 16-way on the one- / two-slot top levels measured slower (reduce
  // 66 -> 77 us per tree: more memory-side atomics), so kReduceSplit stays.
  const char* rs = getenv("YTK_REDUCE_SPLIT");
  const int zs = rs ? std::max(1, atoi(rs)) : kReduceSplit;
  hipLaunchKernelGGL(reduce_u() == 16 ? hist_reduce_kernel<16> : hist_reduce_kernel<8>, dim3((E + 255) / 256, nslots * groups, zs), dim3(256), 0, s,
                     (const long long*)staging, (const int4*)work, nwork, (const int*)nwork_dev,
                     (long long*)hist, B, F, nb_lds, groups, slot_base, (const int*)slot_ids,
                     (const int*)nullptr, (const int2*)nullptr, fw, (const int*)slot_first, one_slot);
  YTK_LAUNCH_CHECK();
}

// First stage alone (block partials to ``staging``): the level engine's one-GPU gathered
// levels reduce and split-search the partials in one launch (ytk_lv_reduce_split).
void ytk_hist_fx_stage(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows, uintptr_t work,
                       int nwork, int B, uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t staging,
                       uintptr_t stream, int gh_rows) {
  if (nwork <= 0) return;
  if (g_hist_fw != 32) throw std::invalid_argument("hist_fx_stage: 32-feature groups only");
  const int groups = (F + 31) / 32;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(nwork, groups);
  if (rows == 0)
    launch_hist_fx<true>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, nullptr, (const int4*)work,
                         nullptr, B, B, 1.f, 1.f, (const int*)nwork_dev, (const float*)scales_dev,
                         (long long*)staging, nullptr);
  else
    launch_hist_fx<false>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                          (const int4*)work, nullptr, B, B, 1.f, 1.f, (const int*)nwork_dev, (const float*)scales_dev,
                          (long long*)staging, nullptr, gh_rows);
  YTK_LAUNCH_CHECK();
}

// Fully device-driven staged histogram (leaf-wise engine): work count, slot count and
// slot ids all live on the device; the host passes only upper bounds (max_work items,
// the y-extent of the slot reduce). Items with w == 1 are their slot's only item and are
// stored directly; items with w == 2 (first item of a slot with > kReduceDirect items)
// zero their slot; slot_ids / slot_range / *nslots_dev list the multi-item slots.
// gh_rows: ghp is indexed by row id (the leaf-wise engine's row-indexed (g, h)), else by
// position in rows.
void ytk_hist_fx_staged_dev(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows,
                            uintptr_t work, int max_work, uintptr_t nwork_dev, uintptr_t hist, int B,
                            uintptr_t scales_dev, uintptr_t staging, uintptr_t slot_ids, uintptr_t nslots_dev,
                            uintptr_t slot_range, int reduce_y, uintptr_t stream, int gh_rows) {
  if (max_work <= 0) return;
  const int fw = g_hist_fw;
  const int groups = (F + fw - 1) / fw;
  const int nb_lds = B;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(max_work, groups);
  if (rows == 0)
    launch_hist_fx<true>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, nullptr,
                         (const int4*)work, (long long*)hist, B, nb_lds, 1.f, 1.f, (const int*)nwork_dev,
                         (const float*)scales_dev, (long long*)staging, nullptr);
  else
    launch_hist_fx<false>(grid, 0, s, (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                          (const int4*)work, (long long*)hist, B, nb_lds, 1.f, 1.f, (const int*)nwork_dev,
                          (const float*)scales_dev, (long long*)staging, nullptr, gh_rows);
  YTK_LAUNCH_CHECK();
  const int E = nb_lds * fw;
  hipLaunchKernelGGL(reduce_u() == 16 ? hist_reduce_kernel<16> : hist_reduce_kernel<8>, dim3((E + 255) / 256, std::max(1, reduce_y) * groups, kReduceSplit),
                     dim3(256), 0, s, (const long long*)staging, (const int4*)work, max_work,
                     (const int*)nwork_dev, (long long*)hist, B, F, nb_lds, groups, 0, (const int*)slot_ids,
                     (const int*)nslots_dev, (const int2*)slot_range, fw, (const int*)nullptr, 0);
  YTK_LAUNCH_CHECK();
}

// Second stage alone: staging items [0, nwork) (32-feature groups, work[k].x = slot) summed
// into the zeroed slots [slot_base, slot_base + nslots) (used by the fused gradient + root
// histogram pass, tree_grad_hist).
void ytk_hist_reduce(uintptr_t staging, uintptr_t work, int nwork, uintptr_t hist, int B, int F, int slot_base,
                     int nslots, uintptr_t stream) {
  if (nwork <= 0 || nslots <= 0) return;
  const int fw = 32;
  const int groups = (F + fw - 1) / fw;
  const int E = B * fw;
  hipLaunchKernelGGL(reduce_u() == 16 ? hist_reduce_kernel<16> : hist_reduce_kernel<8>, dim3((E + 255) / 256, nslots * groups, kReduceSplit), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const long long*)staging, (const int4*)work, nwork,
                     (const int*)nullptr, (long long*)hist, B, F, B, groups, slot_base, (const int*)nullptr,
                     (const int*)nullptr, (const int2*)nullptr, fw, (const int*)nullptr, nslots == 1 ? 1 : 0);
  YTK_LAUNCH_CHECK();
}

void ytk_hist_fx_global(uintptr_t bins, int bin_bytes, long long stride, int F, uintptr_t ghp,
                        uintptr_t rows, uintptr_t work, int nwork, uintptr_t hist, int B,
                        float sg, float sh, uintptr_t stream) {
  if (nwork <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(hist_fx_global_kernel<uint8_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (long long*)hist, B, sg, sh);
  } else {
    hipLaunchKernelGGL(hist_fx_global_kernel<uint16_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint16_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (long long*)hist, B, sg, sh);
  }
  YTK_LAUNCH_CHECK();
}

// Wide-bin histogram (uint16 binsT [F][ncol], any B up to the LDS budget of one feature:
// B * 16 <= 160 KiB). Target slots must be zero. Returns the feature-group size used.
int ytk_hist_wide(uintptr_t binsT, long long ncol, int F, uintptr_t ghp, uintptr_t rows,
                  uintptr_t work, int nwork, uintptr_t hist, int B, float sg, float sh,
                  uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t work_off_dev,
                  uintptr_t stream) {
  const int FG = ytk_hist_wide_group(B, F);
  if (FG <= 0) throw std::invalid_argument("hist_wide: one feature's bins exceed the LDS budget");
  if (nwork <= 0) return FG;
  const size_t lds = (size_t)FG * B * 2 * sizeof(unsigned long long);
  const dim3 grid = wide_grid((F + FG - 1) / FG, nwork);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_WIDE(ID, G)                                                                              \
  hipLaunchKernelGGL((hist_wide_kernel<ID, G>), grid, dim3(kWideThreads), lds, s, (const uint16_t*)binsT, \
                     ncol, F, (const float2*)ghp, (const int*)(ID ? 0 : rows), (const int4*)work,     \
                     (long long*)hist, B, sg, sh, (const int*)nwork_dev, (const float*)scales_dev,    \
                     (const int*)work_off_dev, (long long*)nullptr, nwork)
#define YTK_WIDE_G(ID)                  \
  switch (FG) {                         \
    case 1: YTK_WIDE(ID, 1); break;     \
    case 2: YTK_WIDE(ID, 2); break;     \
    case 4: YTK_WIDE(ID, 4); break;     \
    case 8: YTK_WIDE(ID, 8); break;     \
    case 16: YTK_WIDE(ID, 16); break;   \
    default: YTK_WIDE(ID, 32); break;   \
  }
  if (rows == 0) {
    YTK_WIDE_G(true)
  } else {
    YTK_WIDE_G(false)
  }
#undef YTK_WIDE_G
#undef YTK_WIDE
  YTK_LAUNCH_CHECK();
  return FG;
}

// Row-major wide-bin histogram (hist_wide_rm_kernel): bins [N][stride] uint16. staging != 0:
// block partials to staging (>= nwork * groups * FG * B * 16 bytes), then the split-K reduce
// into the zeroed slots [slot_base, slot_base + nslots); else global atomics into zeroed
// slots. Returns the feature-group size.
int ytk_hist_wide_rm(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows, uintptr_t work, int nwork,
                     uintptr_t hist, int B, float sg, float sh, uintptr_t nwork_dev, uintptr_t scales_dev,
                     uintptr_t work_off_dev, uintptr_t staging, int slot_base, int nslots, uintptr_t binsT,
                     long long ncol, uintptr_t stream) {
  const int FG = ytk_hist_wide_group(B, F);
  if (FG <= 0) throw std::invalid_argument("hist_wide_rm: one feature's bins exceed the LDS budget");
  if (nwork <= 0) return FG;
  if (stride % FG != 0 || (bins % 16) != 0) throw std::invalid_argument("hist_wide_rm: row stride / alignment");
  const size_t lds = (size_t)FG * B * 2 * sizeof(unsigned long long);
  const int groups = (F + FG - 1) / FG;
  const dim3 grid = wide_grid(groups, nwork);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0 && binsT != 0) {
    // identity rows (a tree's root): the column-major copy is read coalesced -- 2 B per row
    // and feature of the group instead of every group re-reading each row's 64-B line
    // (measured on the 5000-bin Higgs root: 1145 us row-major)
#define YTK_WCM(G)                                                                                            \
  hipLaunchKernelGGL((hist_wide_kernel<true, G>), grid, dim3(kWideThreads), lds, s, (const uint16_t*)binsT, ncol, F, \
                     (const float2*)ghp, (const int*)nullptr, (const int4*)work, (long long*)hist, B, sg, sh,     \
                     (const int*)nwork_dev, (const float*)scales_dev, (const int*)work_off_dev, (long long*)staging, nwork)
    switch (FG) {
      case 1: YTK_WCM(1); break;
      case 2: YTK_WCM(2); break;
      case 4: YTK_WCM(4); break;
      case 8: YTK_WCM(8); break;
      case 16: YTK_WCM(16); break;
      default: YTK_WCM(32); break;
    }
#undef YTK_WCM
    YTK_LAUNCH_CHECK();
  } else {
#define YTK_WRM(ID, G)                                                                                          \
  hipLaunchKernelGGL((hist_wide_rm_kernel<ID, G>), grid, dim3(kWideThreads), lds, s, (const uint16_t*)bins, stride, \
                     F, (const float2*)ghp, (const int*)(ID ? 0 : rows), (const int4*)work, (long long*)hist, B, sg, \
                     sh, (const int*)nwork_dev, (const float*)scales_dev, (const int*)work_off_dev,              \
                     (long long*)staging, nwork)
#define YTK_WRM_G(ID)                  \
  switch (FG) {                        \
    case 1: YTK_WRM(ID, 1); break;     \
    case 2: YTK_WRM(ID, 2); break;     \
    case 4: YTK_WRM(ID, 4); break;     \
    case 8: YTK_WRM(ID, 8); break;     \
    case 16: YTK_WRM(ID, 16); break;   \
    default: YTK_WRM(ID, 32); break;   \
  }
  if (rows == 0) {
    YTK_WRM_G(true)
  } else {
    YTK_WRM_G(false)
  }
#undef YTK_WRM_G
#undef YTK_WRM
  YTK_LAUNCH_CHECK();
  }
  if (staging && nslots > 0) {
    const int E = B * FG;
    hipLaunchKernelGGL(reduce_u() == 16 ? hist_reduce_kernel<16> : hist_reduce_kernel<8>, dim3((E + 255) / 256, nslots * groups, kReduceSplit), dim3(256), 0, s,
                       (const long long*)staging, (const int4*)work, nwork, (const int*)nwork_dev, (long long*)hist, B,
                       F, B, groups, slot_base, (const int*)nullptr, (const int*)nullptr, (const int2*)nullptr, FG,
                       (const int*)nullptr, 0);
    YTK_LAUNCH_CHECK();
  }
  return FG;
}

// Device-driven wide histogram (leaf-wise engine, uint16 rows): as ytk_hist_fx_staged_dev --
// work count, slot count and slot ids on the device; items with w == 1 store their slot,
// w == 2 zero it; slot_ids / slot_range / *nslots_dev list the multi-item slots.
void ytk_hist_wide_staged_dev(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows, uintptr_t work,
                              int max_work, uintptr_t nwork_dev, uintptr_t hist, int B, uintptr_t scales_dev,
                              uintptr_t staging, uintptr_t slot_ids, uintptr_t nslots_dev, uintptr_t slot_range,
                              int reduce_y, uintptr_t stream) {
  // (the column-major root kernel has no sole-item / first-item slot handling: row-major here)
  if (max_work <= 0) return;
  const int FG = ytk_hist_wide_group(B, F);
  if (FG <= 0) throw std::invalid_argument("hist_wide_staged_dev: one feature's bins exceed the LDS budget");
  ytk_hist_wide_rm(bins, stride, F, ghp, rows, work, max_work, hist, B, 1.f, 1.f, nwork_dev, scales_dev, 0, staging,
                   0, 0, 0, 0, stream);
  const int groups = (F + FG - 1) / FG;
  const int E = B * FG;
  hipLaunchKernelGGL(reduce_u() == 16 ? hist_reduce_kernel<16> : hist_reduce_kernel<8>, dim3((E + 255) / 256, std::max(1, reduce_y) * groups, kReduceSplit),
                     dim3(256), 0, reinterpret_cast<hipStream_t>(stream), (const long long*)staging, (const int4*)work,
                     max_work, (const int*)nwork_dev, (long long*)hist, B, F, B, groups, 0, (const int*)slot_ids,
                     (const int*)nslots_dev, (const int2*)slot_range, FG, (const int*)nullptr, 0);
  YTK_LAUNCH_CHECK();
}

// Features per block of hist_wide_kernel: the largest power of two <= 32 whose (g, h)
// planes fit the LDS budget (0: a single feature does not fit).
int ytk_hist_wide_group(int B, int F) {
  const long long per = (long long)B * 16;
  if (B <= 0 || per > kWideLdsBytes) return 0;
  const long long fit = std::min<long long>(32, kWideLdsBytes / per);
  int g = 1;
  while (2 * g <= fit) g *= 2;
  return g;
}

}  // extern "C"
