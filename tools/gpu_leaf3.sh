#!/bin/bash
# device leaf-wise engine: equivalence tests, then GBDT GPU tests, bench, kernel timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/leaf3; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
step 400 t_dev.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k device_leafwise
tail -3 $O/t_dev.log
if [ -n "$FULL" ]; then
  step 600 t_gbdt.log python -u -m pytest tests/test_gbdt_train.py tests/test_gbdt_kernels.py tests/test_gbdt_materialize.py -m gpu -x -q --timeout 150 --timeout-method thread
  tail -2 $O/t_gbdt.log
fi
step 300 b_leaf.log python bench.py --steps 20 --warmup 3 --policy loss --leafwise-steps 0
tail -1 $O/b_leaf.log | cut -c1-300
YTK_LW_PROF=1 step 300 b_leaf_prof.log python bench.py --steps 20 --warmup 3 --policy loss --leafwise-steps 0
grep "planner profile" $O/b_leaf_prof.log
cd /tmp
step 300 p.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 4 --warmup 1 --policy loss
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/summary.txt; head -24 $O/summary.txt
echo leaf3 ok
