#!/bin/bash
# leaf-wise 255: bench (20 trees) + kernel timeline of one steady-state round + host cProfile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/leaf2; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
if [ -z "$SKIP_TESTS" ]; then
  step 400 pytest.log python -u -m pytest tests/test_gbdt_kernels.py tests/test_gbdt_train.py -m gpu -x -q --timeout 120 --timeout-method thread
  tail -1 $O/pytest.log
fi
step 300 b_leaf.log python bench.py --steps 20 --warmup 3 --policy loss
tail -1 $O/b_leaf.log | cut -c1-400
cd /tmp
step 300 p.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 4 --warmup 1 --policy loss
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/summary.txt; head -24 $O/summary.txt
echo leaf2 ok
