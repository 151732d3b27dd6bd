#!/bin/bash
# Leaf-wise partition prefetch (row ids + (g, h)) A/B: identity GPU test, leaf-wise 255
# bench YTK_LW_PART_PREFETCH=0 (default) vs 2, interleaved twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2q
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "prefetch_identical"
tail -1 $O/pytest_var.log
for i in 1 2; do
  step 300 bl_pf0_$i.log python bench.py --steps 20 --warmup 3 --policy loss
  tail -1 $O/bl_pf0_$i.log | cut -c1-130
  YTK_LW_PART_PREFETCH=2 step 300 bl_pf2_$i.log python bench.py --steps 20 --warmup 3 --policy loss
  tail -1 $O/bl_pf2_$i.log | cut -c1-130
done
echo r2q ok
