#!/bin/bash
# Level planner fast path: identity tests (kernel variants, host builder, multi-rank on one
# GPU), then full / 1/8-shard / forced-dist benches with YTK_PLAN_FAST on and off, and a
# one-round timeline. Usage: tools/r5_plan.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-plan}
mkdir -p $O
export TMPDIR=/tmp
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("train_loss"))')"
}
timeout -k 10 900 python -u -m pytest tests/test_gbdt_train.py tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for f in 1 0; do
  YTK_PLAN_FAST=$f run full_p$f 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  YTK_PLAN_FAST=$f run eighth_p$f 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  YTK_PLAN_FAST=$f YTK_FORCE_DIST=1 MASTER_PORT=2964$f run eighthdist_p$f 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_e8 -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 $E8 > $O/prof_e8.log 2>&1 || { tail -20 $O/prof_e8.log; exit 1; }
cd $R
python tools/prof_summary.py $O/prof_e8/run_kernel_trace.csv > $O/eighth_round.txt
rm -rf $O/prof_e8
head -8 $O/eighth_round.txt
echo "plan ok"
