#!/bin/bash
# Leaf-wise launch-pipeline A/B (255 leaves, Higgs shape): batches queued ahead of the planner
# (YTK_LW_POLL_LAG) x kernel arguments in device memory (HIP_FORCE_DEV_KERNARG), two repeats.
# Usage: tools/r5_leaf_ab.sh <tag> [steps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-leafab}
STEPS=${2:-20}
mkdir -p $O
cd $R
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
for rep in 1 2; do
  for lag in 2 4 8; do
    for k in 0 1; do
      HIP_FORCE_DEV_KERNARG=$k YTK_LW_POLL_LAG=$lag run leaf_lag${lag}_k${k}_r$rep 300 python bench.py --policy loss --steps $STEPS --warmup 3
    done
  done
done
echo "leafab ok"
