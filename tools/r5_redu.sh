#!/bin/bash
# Slot-reduce loads in flight A/B (YTK_REDUCE_U 8 / 16): level-wise full and 1/8 shard,
# leaf-wise 255 leaves; then the leaf-wise late-tree timeline. Usage: tools/r5_redu.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-redu}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
for u in 16 8; do
  YTK_REDUCE_U=$u run full_u$u 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  YTK_REDUCE_U=$u run eighth_u$u 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  YTK_REDUCE_U=$u run leaf_u$u 300 python bench.py --policy loss --steps 20 --warmup 3
done
bash tools/r5_leafprof.sh ${1:-redu}/leafprof || exit 1
echo "redu ok"
