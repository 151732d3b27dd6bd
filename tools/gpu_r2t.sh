#!/bin/bash
# tree_grad LDS-staged walk A/B: variant-identity GPU tests, level-wise and leaf-wise benches
# with YTK_TG_LDS_WALK=0 (default) vs 1, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2t
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants or device_builder_matches or leafwise_matches"
tail -1 $O/pytest_var.log
for i in 1 2; do
  step 300 b_w0_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_w0_$i.log | cut -c100-135
  YTK_TG_LDS_WALK=1 step 300 b_w1_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  tail -1 $O/b_w1_$i.log | cut -c100-135
done
step 300 bl_w0.log python bench.py --steps 20 --warmup 3 --policy loss
tail -1 $O/bl_w0.log | cut -c100-135
YTK_TG_LDS_WALK=1 step 300 bl_w1.log python bench.py --steps 20 --warmup 3 --policy loss
tail -1 $O/bl_w1.log | cut -c100-135
cd /tmp
YTK_TG_LDS_WALK=1 step 300 prof.log rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/round.txt
grep tree_grad $O/round.txt
echo r2t ok
