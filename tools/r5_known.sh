#!/bin/bash
# Slot reduce with known item ranges (YTK_REDUCE_KNOWN 1, default) vs the work-list scan (0):
# GBDT + multi-rank GPU tests, full / 1/8 / forced-dist 1/8 benches, two repeats.
# Usage: tools/r5_known.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-known}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"), d.get("test_loss"))')"
}
timeout -k 10 900 python -u -m pytest tests/test_gbdt_train.py tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for k in 1 0; do
    YTK_REDUCE_KNOWN=$k run full_k${k}_r$r 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
    YTK_REDUCE_KNOWN=$k run eighth_k${k}_r$r 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  done
done
YTK_FORCE_DIST=1 MASTER_PORT=29661 run eighthdist_k1 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
echo "known ok"
