#!/bin/bash
# Leaf-wise per-launch timeline of a late tree (rocprofv3 kernel trace, 60 trees) and the
# planner phase counters. Usage: tools/r5_leafprof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-leafprof}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --policy loss --steps 60 --warmup 2 --leafwise-steps 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
python tools/prof_timeline.py $O/prof/run_kernel_trace.csv > $O/late_timeline.txt
python tools/prof_summary.py $O/prof/run_kernel_trace.csv > $O/late_round.txt
rm -rf $O/prof
head -14 $O/late_round.txt
echo "leafprof ok"
