#!/bin/bash
# A/B of the leaf-wise small-node subtree knobs (500-tree leaf-wise bench, one GPU):
#   tools/ab_leaf_sub.sh <tag> "ROWS:MAX:ALPHA" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for cfg in "$@"; do
  IFS=: read -r rows mx al <<< "$cfg"
  YTK_LW_SUB_ROWS=$rows YTK_LW_SUB_MAX=$mx YTK_LW_SUB_ALPHA=$al YTK_LW_PROF=${PROF:-0} \
    timeout -k 10 300 python bench.py --policy loss --steps ${STEPS:-500} --warmup ${WARM:-5} \
    > "$O/l_${rows}_${mx}_${al}.json" 2> "$O/l_${rows}_${mx}_${al}.err" || { tail -20 "$O/l_${rows}_${mx}_${al}.err"; exit 1; }
  echo "$cfg $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss'])" "$O/l_${rows}_${mx}_${al}.json")"
  grep -h "planner profile" "$O/l_${rows}_${mx}_${al}.err" | cut -c1-600 || true
done
