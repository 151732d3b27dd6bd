#!/bin/bash
# Rounds left in flight by the host after each round (YTK_ROUND_LAG 1 / 2 / 3): level-wise full
# and 1/8 shard, leaf-wise 20 trees, two repeats; one-round 1/8 timeline at lag 3.
# Usage: tools/r5_rlag.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rlag}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"), d.get("test_loss"))')"
}
for r in 1 2; do
  for k in 1 2 3; do
    YTK_ROUND_LAG=$k run full_l${k}_r$r 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
    YTK_ROUND_LAG=$k run eighth_l${k}_r$r 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  done
done
for k in 1 3; do
  YTK_ROUND_LAG=$k run leaf_l$k 300 python bench.py --policy loss --steps 20 --warmup 3
done
export TMPDIR=/tmp
cd /tmp
YTK_ROUND_LAG=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_e8 -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 $E8 > $O/prof_e8.log 2>&1 || { tail -20 $O/prof_e8.log; exit 1; }
cd $R
python tools/prof_timeline.py $O/prof_e8/run_kernel_trace.csv > $O/eighth_timeline_lag3.txt
rm -rf $O/prof_e8
head -5 $O/eighth_timeline_lag3.txt
echo "rlag ok"
