#!/bin/bash
# Leaf-wise children fast path: identity tests, then 255-leaf benches (20 and 200 trees) with
# YTK_PLAN_FAST on / off. Usage: tools/r5_lwc.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-lwc}
mkdir -p $O
cd $R
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
timeout -k 10 900 python -u -m pytest tests/test_gbdt_train.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "leafwise or variants_identical or matches_host" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for f in 1 0; do
  YTK_PLAN_FAST=$f run leaf_p$f 300 python bench.py --policy loss --steps 20 --warmup 3
  YTK_PLAN_FAST=$f run leaf200_p$f 300 python bench.py --policy loss --steps 200 --warmup 3
  YTK_PLAN_FAST=$f run leafe8_p$f 300 python bench.py --policy loss --steps 50 --warmup 3 --train-rows 1312500 --test-rows 62500
done
echo "lwc ok"
