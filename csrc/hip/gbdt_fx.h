// Fixed-point (g, h) rounding and the conflict-free LDS feature positions shared by the
// histogram kernels (gbdt_hist.hip) and the leaf-wise small-node subtree kernel
// (gbdt_leafwise.hip) -- both must quantise identically for the exact int64 sums to match.
#pragma once
#include "common.h"

namespace ytk {

// Exact float -> int64 round-half-even for the fixed-point (g, h): y = x * 2^k is an
// exact float; rint makes it integral. On its magnitude a, hi = floor(a / 2^32) and
// lo = a - hi * 2^32 are exact (lo < 2^32 is a multiple of ulp(a), so it has <= 24
// significant bits) and 32-bit convertible; the sign is applied to the 64-bit value
// ((u ^ m) - m). ~10 VALU instead of the generic __float2ll_rn sequence; bitwise equal
// to it (and to torch.round(x * s).to(int64) on the CPU) for |y| < 2^63.
__device__ __forceinline__ unsigned long long fx_round(float y) {
  const float r = __builtin_rintf(y);
  const float a = fabsf(r);
  const float hi = floorf(a * 0x1p-32f);
  const float lo = __builtin_fmaf(hi, -0x1p32f, a);
  const unsigned long long u = ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
  const unsigned long long m = r < 0.f ? ~0ull : 0ull;
  return (u ^ m) - m;
}

// Position of local feature fl (0..31) inside the 32 g (or h) words of an LDS bin row. ds_add_u64 is
// serviced in four 16-lane groups with bank = (byte address / 4) mod 32, so a 64-bit
// word w occupies banks 2(w mod 16), 2(w mod 16)+1. A 16-lane group updates the
// features {4q + c0, 4q + c1 : q = 0..7}: features fl and fl + 16 would share banks
// (2-way conflict, measured SQ_LDS_BANK_CONFLICT = 50 % of SQ_LDS_IDX_ACTIVE). Rotating
// the upper 16 features by 2 words makes the 16 lanes hit 16 distinct bank pairs.
__device__ __forceinline__ int hist_lds_pos(int fl) {
  return fl < 16 ? fl : 16 + ((fl - 14) & 15);
}

}  // namespace ytk
