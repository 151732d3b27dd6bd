#!/bin/bash
# histogram feature-group width A/B: tests at fw 16, level + leaf benches at fw 32 / 16
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fw; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
YTK_HIST_FW=16 step 600 t16.log python -u -m pytest tests/test_gbdt_train.py tests/test_gbdt_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread
tail -1 $O/t16.log
for fw in 32 16; do
  YTK_HIST_FW=$fw step 300 lvl_$fw.log python bench.py --leafwise-steps 0
  echo "fw=$fw level: $(tail -1 $O/lvl_$fw.log | cut -c100-160)"
  YTK_HIST_FW=$fw step 300 leaf_$fw.log python bench.py --steps 20 --warmup 3 --policy loss --leafwise-steps 0
  echo "fw=$fw leaf: $(tail -1 $O/leaf_$fw.log | cut -c100-160)"
done
cd /tmp
YTK_HIST_FW=16 step 300 p16.log rocprofv3 --kernel-trace --output-format csv -d $O/prof16 -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof16/*kernel_trace.csv | head -1) > $O/summary16.txt; head -8 $O/summary16.txt
echo fw ok
