#!/bin/bash
# Leaf-wise iteration: GPU tests (SKIP_TESTS=1 skips), leaf-wise 255-leaf bench, one-round
# kernel timeline. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2g
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
if [ -z "$SKIP_TESTS" ]; then
  step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  tail -1 $O/pytest_gpu.log
fi
step 300 bench_leaf.log python bench.py --steps 30 --warmup 3 --policy loss
tail -1 $O/bench_leaf.log | cut -c1-200
cd /tmp
step 300 prof_leaf.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_leaf -o run -- python $R/bench.py --steps 6 --warmup 2 --policy loss
cd $R
python tools/prof_summary.py $(ls $O/prof_leaf/*kernel_trace.csv | head -1) > $O/leaf_round.txt
head -16 $O/leaf_round.txt
echo r2g ok
