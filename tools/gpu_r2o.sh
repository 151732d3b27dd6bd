#!/bin/bash
# Slot-reduce split-K A/B: variant-identity GPU tests, level-wise bench (full + 1/8 shard)
# YTK_REDUCE_SPLIT=8 vs the default (32 / 16 on one / two slots), one-round timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2o
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants or device_builder_matches or leafwise"
tail -1 $O/pytest_var.log
E="--train-rows 1312500 --test-rows 62500"
for i in 1 2; do
  YTK_REDUCE_SPLIT=8 step 300 b_z8_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_z8_$i.log | cut -c1-130
  step 300 b_zd_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_zd_$i.log | cut -c1-130
done
YTK_REDUCE_SPLIT=8 step 300 b8_z8.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
tail -1 $O/b8_z8.log | cut -c1-130
step 300 b8_zd.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
tail -1 $O/b8_zd.log | cut -c1-130
cd /tmp
step 300 prof.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/round.txt
head -10 $O/round.txt
echo r2o ok
