#!/bin/bash
# Split-K factor of the staged slot reduce (YTK_REDUCE_SPLIT 4 / 8 / 16) at the full and the
# 1/8 shard. Usage: tools/r5_zs.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-zs}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
for z in 4 8 16; do
  YTK_REDUCE_SPLIT=$z run full_z$z 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  YTK_REDUCE_SPLIT=$z run eighth_z$z 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
done
echo "zs ok"
