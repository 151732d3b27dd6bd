#!/bin/bash
# Split-search feature groups per node (YTK_SPLIT_GROUPS 2 / 4 / 7 / 14) at the full and the 1/8
# shard. Usage: tools/r5_sg.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sg}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
for g in 4 7 14 2; do
  YTK_SPLIT_GROUPS=$g run full_g$g 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  YTK_SPLIT_GROUPS=$g run eighth_g$g 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  YTK_SPLIT_GROUPS=$g run leaf_g$g 300 python bench.py --policy loss --steps 20 --warmup 3
done
echo "sg ok"
