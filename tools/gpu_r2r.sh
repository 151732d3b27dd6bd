#!/bin/bash
# Partition split-feature-byte prefetch A/B: variant-identity GPU tests, level-wise bench
# YTK_PART_PREFETCH=2 (default) vs 3, interleaved twice, plus the 1/8 shard.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2r
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants or device_builder_matches"
tail -1 $O/pytest_var.log
E="--train-rows 1312500 --test-rows 62500"
for i in 1 2; do
  step 300 b_pf2_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_pf2_$i.log | cut -c1-130
  YTK_PART_PREFETCH=3 step 300 b_pf3_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_pf3_$i.log | cut -c1-130
done
step 300 b8_pf2.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
tail -1 $O/b8_pf2.log | cut -c1-130
YTK_PART_PREFETCH=3 step 300 b8_pf3.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
tail -1 $O/b8_pf3.log | cut -c1-130
echo r2r ok
