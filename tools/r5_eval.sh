#!/bin/bash
# Round-5 evidence run on one MI355X: headline bench, 1/8-shard plain + forced-dist (every
# multi-GPU code path on a world-1 group) benches, and one-round rocprofv3 timelines of the
# 1/8 shard. Usage: tools/r5_eval.sh <tag> [stages...]; stages: bench eighth prof leafprof
# full-prof tests. Outputs under gpurun_out/<tag>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5}
shift
STAGES=${*:-bench eighth prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
E8="--train-rows 1312500 --test-rows 62500"
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
if has bench; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
if has eighth; then
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 > $O/eighth_plain.json 2> $O/eighth_plain.err || { tail -30 $O/eighth_plain.err; exit 1; }
  cat $O/eighth_plain.json
  YTK_FORCE_DIST=1 MASTER_PORT=29611 timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 > $O/eighth_forced.json 2> $O/eighth_forced.err || { tail -30 $O/eighth_forced.err; exit 1; }
  cat $O/eighth_forced.json
fi
if has prof; then
  cd /tmp
  YTK_FORCE_DIST=1 MASTER_PORT=29612 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8f -o run -- python3 $R/bench.py --steps 10 --warmup 2 $E8 --leafwise-steps 0 > $O/prof8f.log 2>&1 || { tail -20 $O/prof8f.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8 -o run -- python3 $R/bench.py --steps 10 --warmup 2 $E8 --leafwise-steps 0 > $O/prof8.log 2>&1 || { tail -20 $O/prof8.log; exit 1; }
  cd $R
  python tools/prof_summary.py $O/prof8f/run_kernel_trace.csv > $O/eighth_forced_round.txt
  python tools/prof_summary.py $O/prof8/run_kernel_trace.csv > $O/eighth_plain_round.txt
  head -40 $O/eighth_forced_round.txt
fi
if has leafprof; then
  cd /tmp
  YTK_FORCE_DIST=1 MASTER_PORT=29613 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8lf -o run -- python3 $R/bench.py --steps 4 --warmup 1 $E8 --policy loss > $O/prof8lf.log 2>&1 || { tail -20 $O/prof8lf.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8l -o run -- python3 $R/bench.py --steps 4 --warmup 1 $E8 --policy loss > $O/prof8l.log 2>&1 || { tail -20 $O/prof8l.log; exit 1; }
  cd $R
  python tools/prof_summary.py $O/prof8lf/run_kernel_trace.csv > $O/eighth_leaf_forced_round.txt
  python tools/prof_summary.py $O/prof8l/run_kernel_trace.csv > $O/eighth_leaf_plain_round.txt
fi
if has full-prof; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/proffull -o run -- python3 $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0 > $O/proffull.log 2>&1 || { tail -20 $O/proffull.log; exit 1; }
  cd $R
  python tools/prof_summary.py $O/proffull/run_kernel_trace.csv > $O/full_round.txt
fi
echo "r5_eval $TAG ok"
