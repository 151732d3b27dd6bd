#!/bin/bash
# GPU round: kernel/numerics tests, bench, rocprofv3 kernel stats. Every GPU step
# runs under its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-30}
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ -n "$PROF" ]; then
  rm -rf $OUT/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 2 > $OUT/prof_bench.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_bench.log; exit 1; }
  echo prof ok
fi
