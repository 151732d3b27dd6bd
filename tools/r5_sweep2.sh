#!/bin/bash
# 1/8-shard knobs after the planner fast paths: histogram blocks per level (YTK_HIST_TARGET),
# the fused reduce + split (YTK_FUSE_REDUCE_SPLIT=1), partition chunk 1024. Usage: tools/r5_sweep2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sweep2}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
run base 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
YTK_HIST_TARGET=128 run ht128 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
YTK_HIST_TARGET=192 run ht192 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
YTK_FUSE_REDUCE_SPLIT=1 YTK_RS_GROUP=8 run rs8 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
YTK_PART_CHUNK=1024 run pc1024 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
run base2 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
echo "sweep2 ok"
