#!/bin/bash
# GPU tests; leaf-wise 255 bench with split feature groups 1 vs 4 (default), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2n
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -1 $O/pytest_gpu.log
for i in 1 2; do
  YTK_SPLIT_GROUPS=1 step 300 bl_g1_$i.log python bench.py --steps 20 --warmup 3 --policy loss
  tail -1 $O/bl_g1_$i.log | cut -c1-130
  step 300 bl_g4_$i.log python bench.py --steps 20 --warmup 3 --policy loss
  tail -1 $O/bl_g4_$i.log | cut -c1-130
done
echo r2n ok
