#!/bin/bash
# Fused split + plan (YTK_FUSE_SPLIT_PLAN=1, the planner's fast path in the split kernel's last
# block) vs the two launches: identity tests, full and 1/8-shard benches. Usage: tools/r5_fsp.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-fsp}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
timeout -k 10 600 python -u -m pytest tests/test_gbdt_train.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "variants_identical or fused_reduce_split or matches_host" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for f in 1 0; do
    YTK_FUSE_SPLIT_PLAN=$f run full_f${f}_r$r 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
    YTK_FUSE_SPLIT_PLAN=$f run eighth_f${f}_r$r 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  done
done
echo "fsp ok"
