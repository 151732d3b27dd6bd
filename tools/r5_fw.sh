#!/bin/bash
# Histogram feature width A/B (YTK_HIST_FW 32 vs 16: 16-feature blocks, 2 per CU) for leaf-wise
# (20 / 200 trees) and level-wise (full, 1/8). Usage: tools/r5_fw.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-fw}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
for fw in 16 32; do
  YTK_HIST_FW=$fw run leaf_fw$fw 300 python bench.py --policy loss --steps 20 --warmup 3
  YTK_HIST_FW=$fw run leaf200_fw$fw 300 python bench.py --policy loss --steps 200 --warmup 3
  YTK_HIST_FW=$fw run full_fw$fw 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  YTK_HIST_FW=$fw run eighth_fw$fw 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
done
echo "fw ok"
