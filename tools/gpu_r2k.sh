#!/bin/bash
# Partition (g, h) prefetch A/B: variant-identity GPU tests, level-wise bench
# YTK_PART_PREFETCH=1 (default) vs 2, interleaved twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2k
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants or device_builder_matches"
tail -1 $O/pytest_var.log
for i in 1 2; do
  step 300 b_pf1_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_pf1_$i.log | cut -c1-140
  YTK_PART_PREFETCH=2 step 300 b_pf2_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_pf2_$i.log | cut -c1-140
done
echo r2k ok
