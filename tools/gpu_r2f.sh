#!/bin/bash
# Split-kernel A/B: node-resident split_node_kernel vs (node, feature)-parallel split_feat_kernel
# on the full and the 1/8-shard level-wise bench, plus a 1/8-shard kernel timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2f
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
E="--train-rows 1312500 --test-rows 62500"
step 300 b_full.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
tail -1 $O/b_full.log | cut -c1-200
YTK_SPLIT_NODE=0 step 300 b_full_feat.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
tail -1 $O/b_full_feat.log | cut -c1-200
step 300 b_8.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
tail -1 $O/b_8.log | cut -c1-200
YTK_SPLIT_NODE=0 step 300 b_8_feat.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
tail -1 $O/b_8_feat.log | cut -c1-200
cd /tmp
step 300 p8.log rocprofv3 --kernel-trace --output-format csv -d $O/prof8 -o run -- python $R/bench.py --steps 6 --warmup 2 --leafwise-steps 0 $E
cd $R
python tools/prof_summary.py $(ls $O/prof8/*kernel_trace.csv | head -1) > $O/p8_summary.txt
head -20 $O/p8_summary.txt
echo r2f ok
