#!/bin/bash
# 1/8-shard level-wise tree on one GPU (the per-GPU compute of the 8-GPU strong-scaling run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/eighth; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
step 300 b.log python bench.py --train-rows 1312500 --test-rows 62500 --leafwise-steps 0
tail -1 $O/b.log | cut -c1-200
cd /tmp
step 300 p.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --train-rows 1312500 --test-rows 62500 --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/summary.txt; head -24 $O/summary.txt
echo eighth ok
