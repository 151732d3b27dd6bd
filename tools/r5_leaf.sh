#!/bin/bash
# Leaf-wise 255-leaf late-tree profile: rocprofv3 kernel trace over 300 trees, the last round's
# breakdown and timeline, plus the 500-tree bench average.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-leaf}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pl -o run -- python3 $R/bench.py --policy loss --steps 300 --warmup 2 > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
cd $R
python3 tools/prof_summary.py $O/pl/run_kernel_trace.csv > $O/late_round.txt
python3 tools/prof_timeline.py $O/pl/run_kernel_trace.csv > $O/late_timeline.txt
head -14 $O/late_round.txt
timeout -k 10 400 python bench.py --policy loss --steps 500 --warmup 5 > $O/leaf500.json 2> $O/leaf500.err || { tail -20 $O/leaf500.err; exit 1; }
cat $O/leaf500.json
echo "leaf ok"
