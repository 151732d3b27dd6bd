#!/bin/bash
# Quick level-wise iteration: GPU tests (SKIP_TESTS=1 skips), level-wise bench under two
# partition chunk sizes, one-round kernel timeline. Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2e
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
if [ -z "$SKIP_TESTS" ]; then
  step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  tail -1 $O/pytest_gpu.log
fi
step 300 bench.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
tail -1 $O/bench.log | cut -c1-260
YTK_PART_CHUNK=2048 step 300 bench_c2048.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
tail -1 $O/bench_c2048.log | cut -c1-260
cd /tmp
step 300 prof_level.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_level -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof_level/*kernel_trace.csv | head -1) > $O/level_round.txt
head -22 $O/level_round.txt
echo r2e ok
