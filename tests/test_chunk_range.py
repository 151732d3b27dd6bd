"""Index math of the partition's in-block prefix sums (CPU).

The partition kernel's kMode 3 (csrc/hip/gbdt_partition_atomic.h) sums a chunk's (right,
left) prefix over its split's earlier chunk counts as whole 32-chunk group sums plus the
partial groups at both ends (``ChunkRange``, csrc/hip/gbdt_chunk_range.h; the count pass adds
every chunk's count into its group's sum). The GPU tests compare the resulting trees with the
cursor-atomic partition; this test checks the geometry itself: a host-only build of the same
header sums every (f0, f1) range of random packed counts and compares with a brute-force sum,
and checks that every item address lies inside the split's chunks or the whole groups
between its ends, and the item-count bound the kernel's unrolled loads assume.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIP_DIR = os.path.join(ROOT, "csrc", "hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

pytestmark = pytest.mark.skipif(not shutil.which(HIPCC), reason="hipcc not available")

HARNESS = r"""
#include "gbdt_chunk_range.h"
#include <cstdio>
#include <random>
#include <vector>

int main() {
  std::mt19937_64 rng(7);
  long long checks = 0;
  const int sizes[] = {1, 2, 31, 32, 33, 63, 64, 65, 95, 96, 97, 160, 161, 200, 5127, 40000};
  for (int n : sizes) {
    std::vector<unsigned long long> cnt(n);
    for (auto& c : cnt) c = ((rng() % 2049ull) << 32) | (rng() % 2049ull);  // (right << 32) | left
    const int ng = (n + 31) >> ytk::kGrpShift;
    std::vector<unsigned long long> gsum(ng, 0ull);
    for (int i = 0; i < n; ++i) gsum[i >> ytk::kGrpShift] += cnt[i];
    auto check = [&](int f0, int f1) -> bool {
      const ytk::ChunkRange cr(f0, f1);
      unsigned long long got = 0ull, want = 0ull;
      for (int i = f0; i < f1; ++i) want += cnt[i];
      for (int t = 0; t < cr.ntot; ++t) {
        const unsigned long long* p = cr.item(cnt.data(), gsum.data(), t);
        if (p >= cnt.data() && p < cnt.data() + n) {
          const long i = p - cnt.data();
          if (i < f0 || i >= f1) { std::printf("FAIL n=%d [%d,%d) t=%d: count %ld outside\n", n, f0, f1, t, i); return false; }
        } else {
          const long g = p - gsum.data();
          if (g < 0 || g >= ng || (g << ytk::kGrpShift) < f0 || ((g + 1) << ytk::kGrpShift) > f1) {
            std::printf("FAIL n=%d [%d,%d) t=%d: group %ld not inside\n", n, f0, f1, t, g);
            return false;
          }
        }
        got += *p;
      }
      // <= 31 leading + 31 trailing single counts (a group-aligned f0 reads its first group
      // count by count: 32) plus the whole groups between
      const int bound = 63 + (f1 - f0) / 32;
      if (got != want || cr.ntot > bound || (f1 == f0 && cr.ntot != 0)) {
        std::printf("FAIL n=%d [%d,%d): sum %llu vs %llu, items %d (bound %d)\n", n, f0, f1, got, want, cr.ntot, bound);
        return false;
      }
      ++checks;
      return true;
    };
    if (n <= 200) {
      for (int f0 = 0; f0 <= n; ++f0)
        for (int f1 = f0; f1 <= n; ++f1)
          if (!check(f0, f1)) return 1;
    } else {
      for (int k = 0; k < 20000; ++k) {
        int a = (int)(rng() % (n + 1)), b = (int)(rng() % (n + 1));
        if (a > b) { const int t = a; a = b; b = t; }
        if (!check(a, b)) return 1;
      }
      if (!check(0, n) || !check(31, n) || !check(32, n - 1) || !check(33, 33)) return 1;
    }
  }
  std::printf("ok %lld\n", checks);
  return 0;
}
"""


def test_chunk_range_sums_and_bounds(tmp_path):
    src = tmp_path / "chunk_range_check.hip"
    exe = tmp_path / "chunk_range_check"
    src.write_text(HARNESS)
    # host-only build: the header's __host__ __device__ members, no device code object
    r = subprocess.run([HIPCC, "-O2", "-std=c++17", "--offload-host-only", "-I" + HIP_DIR, str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.startswith("ok ")
    assert int(r.stdout.split()[1]) > 100000
