#!/bin/bash
# GPU tests, level-wise bench (prefetch partition default), leaf-wise bench A/B of the
# pipelined partition body (YTK_LW_PART_PREFETCH), interleaved twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2j
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -1 $O/pytest_gpu.log
step 300 b_level.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
tail -1 $O/b_level.log | cut -c1-140
for i in 1 2; do
  step 300 b_leaf$i.log python bench.py --steps 20 --warmup 3 --policy loss
  tail -1 $O/b_leaf$i.log | cut -c1-140
  YTK_LW_PART_PREFETCH=1 step 300 b_leafpf$i.log python bench.py --steps 20 --warmup 3 --policy loss
  tail -1 $O/b_leafpf$i.log | cut -c1-140
done
echo r2j ok
