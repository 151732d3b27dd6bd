#!/bin/bash
# Split feature-group A/B: GPU tests, level-wise bench YTK_SPLIT_GROUPS=1 / 4 (default) / 7
# on the full and the 1/8-shard Higgs, one-round timeline with the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2m
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -1 $O/pytest_gpu.log
E="--train-rows 1312500 --test-rows 62500"
for g in 1 4 7; do
  YTK_SPLIT_GROUPS=$g step 300 b_g$g.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_g$g.log | cut -c1-130
  YTK_SPLIT_GROUPS=$g step 300 b8_g$g.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
  tail -1 $O/b8_g$g.log | cut -c1-130
done
cd /tmp
step 300 prof.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/round.txt
head -10 $O/round.txt
echo r2m ok
