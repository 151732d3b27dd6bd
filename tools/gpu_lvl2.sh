#!/bin/bash
# level engine + multi-rank GPU tests, headline bench, timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/level; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
step 900 t_gbdt.log python -u -m pytest tests/test_gbdt_train.py tests/test_gbdt_kernels.py tests/test_gbdt_materialize.py tests/test_models_e2e.py tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 $O/t_gbdt.log
step 300 bench.log python bench.py --leafwise-steps 0
tail -1 $O/bench.log | cut -c1-200
cd /tmp
step 300 p.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/summary.txt; head -24 $O/summary.txt
echo level ok
