#!/bin/bash
# Leaf-wise batches queued ahead of the planner: YTK_LW_POLL_LAG 1 vs 2 (20 and 200 trees,
# two repeats). Usage: tools/r5_lag.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-lag}
mkdir -p $O
cd $R
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
for r in 1 2; do
  for lag in 1 2; do
    YTK_LW_POLL_LAG=$lag run leaf_lag${lag}_r$r 300 python bench.py --policy loss --steps 20 --warmup 3
    YTK_LW_POLL_LAG=$lag run leaf200_lag${lag}_r$r 300 python bench.py --policy loss --steps 200 --warmup 3
  done
done
echo "lag ok"
