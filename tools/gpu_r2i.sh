#!/bin/bash
# Partition prefetch A/B: variant-identity GPU test, then level-wise bench default vs
# YTK_PART_PREFETCH=1 (twice each, interleaved), one-round timeline with the prefetch on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2i
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants or device_builder_matches"
tail -1 $O/pytest_var.log
for i in 1 2; do
  step 300 b_def$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_def$i.log | cut -c1-140
  YTK_PART_PREFETCH=1 step 300 b_pf$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_pf$i.log | cut -c1-140
done
cd /tmp
YTK_PART_PREFETCH=1 step 300 prof.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/round.txt
head -8 $O/round.txt
echo r2i ok
