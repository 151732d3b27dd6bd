#!/bin/bash
# Final round-5 evidence: r5_ev.sh (GPU suite, smoke, default bench, 500-tree level / leaf,
# 1/8 shard, 5000 bins, sparse L-BFGS, SGD), then rocprofv3 kernel statistics + one-round
# timelines of the default level-wise bench and the 1/8 shard. Usage: tools/r5_final.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
O=$R/gpurun_out/$TAG
bash $R/tools/r5_ev.sh $TAG suite bench b500 eighth b5k sparse sgd || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_full -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 > $O/prof_full.log 2>&1 || { tail -20 $O/prof_full.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e8 -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 --train-rows 1312500 --test-rows 62500 > $O/prof_e8.log 2>&1 || { tail -20 $O/prof_e8.log; exit 1; }
cd $R
python tools/prof_summary.py $O/prof_full/run_kernel_trace.csv > $O/full_round.txt
python tools/prof_summary.py $O/prof_e8/run_kernel_trace.csv > $O/eighth_round.txt
python tools/prof_timeline.py $O/prof_e8/run_kernel_trace.csv > $O/eighth_timeline.txt
cp $O/prof_full/run_kernel_stats.csv $O/full_kernel_stats.csv
cp $O/prof_e8/run_kernel_stats.csv $O/eighth_kernel_stats.csv
rm -rf $O/prof_full $O/prof_e8
head -12 $O/full_round.txt
echo "final $TAG ok"
