#!/bin/bash
# Fused reduce + split A/B: identity tests, full / 1/8-shard benches with the fused kernel on
# and off, one-round timelines (rocprofv3 kernel trace) of the fused path.
# Usage: tools/r5_rs.sh <tag> [stages]; stages: test ab prof
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-rs}
shift
STAGES=${*:-test ab prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
E8="--train-rows 1312500 --test-rows 62500"
has() { [[ " $STAGES " == *" $1 "* ]]; }
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | cut -c1-200
}
if has test; then
  timeout -k 10 600 python -u -m pytest tests/test_gbdt_train.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "variants_identical or fused_reduce_split or matches_host" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if has ab; then
  for f in 1 0; do
    YTK_FUSE_REDUCE_SPLIT=$f run full_f$f 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
    YTK_FUSE_REDUCE_SPLIT=$f run eighth_f$f 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  done
fi
if has groups; then
  for g in 2 8; do
    YTK_FUSE_REDUCE_SPLIT=1 YTK_RS_GROUP=$g run full_g$g 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
    YTK_FUSE_REDUCE_SPLIT=1 YTK_RS_GROUP=$g run eighth_g$g 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  done
fi
if has prof; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_full -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 > $O/prof_full.log 2>&1 || { tail -20 $O/prof_full.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_e8 -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 $E8 > $O/prof_e8.log 2>&1 || { tail -20 $O/prof_e8.log; exit 1; }
  cd $R
  python tools/prof_summary.py $O/prof_full/run_kernel_trace.csv > $O/full_round.txt
  python tools/prof_summary.py $O/prof_e8/run_kernel_trace.csv > $O/eighth_round.txt
  head -16 $O/full_round.txt; head -16 $O/eighth_round.txt
  rm -rf $O/prof_full $O/prof_e8
fi
echo "r5_rs $TAG ok"
