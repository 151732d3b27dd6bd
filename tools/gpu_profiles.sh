#!/bin/bash
# Full evidence run on one MI355X: GPU tests, GBDT bench + kernel profile, sparse-model
# benches + kernel profiles. Outputs under gpurun_out/evidence/; copy into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/evidence
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for m in linear fm ffm; do
  timeout -k 10 400 python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o run -- python $R/bench.py --steps 10 --warmup 2 > $O/prof_gbdt.log 2>&1 || { tail -20 $O/prof_gbdt.log; exit 1; }
for m in linear fm ffm; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python $R/bench_sparse.py --model $m --rows 4000000 --steps 3 --warmup 1 > $O/prof_$m.log 2>&1 || { tail -20 $O/prof_$m.log; exit 1; }
done
echo evidence ok
