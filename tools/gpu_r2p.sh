#!/bin/bash
# Partition chunk A/B for small shards: variant-identity GPU tests, 1/8-shard and full
# level-wise bench with YTK_PART_CHUNK=1024 vs the default 2048, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2p
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 300 pytest_var.log python -u -m pytest tests/test_gbdt_train.py -m gpu -x -v --timeout 120 --timeout-method thread -k "variants"
tail -1 $O/pytest_var.log
E="--train-rows 1312500 --test-rows 62500"
for i in 1 2; do
  step 300 b8_c2048_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
  tail -1 $O/b8_c2048_$i.log | cut -c1-130
  YTK_PART_CHUNK=1024 step 300 b8_c1024_$i.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E
  tail -1 $O/b8_c1024_$i.log | cut -c1-130
done
YTK_PART_CHUNK=1024 step 300 b_c1024.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0
tail -1 $O/b_c1024.log | cut -c1-130
echo r2p ok
