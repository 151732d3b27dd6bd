#!/bin/bash
# Full evidence run on one MI355X: GPU tests, GBDT benches (level-wise depth 6 = the
# BASELINE metric, 1/8 row shard = the per-GPU work at N=8, leaf-wise 255 leaves = the
# reference's own Higgs config) with rocprofv3 kernel stats and one-round timelines,
# sparse-model benches + kernel stats. Outputs under gpurun_out/evidence/; copy the
# summaries into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/evidence
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --train-rows 1312500 --test-rows 62500 > $O/bench_eighth.log 2>&1 || { tail -30 $O/bench_eighth.log; exit 1; }
tail -1 $O/bench_eighth.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --policy loss > $O/bench_leafwise.log 2>&1 || { tail -30 $O/bench_leafwise.log; exit 1; }
tail -1 $O/bench_leafwise.log
for m in linear fm ffm; do
  timeout -k 10 400 python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o run -- python $R/bench.py --steps 10 --warmup 2 > $O/prof_gbdt.log 2>&1 || { tail -20 $O/prof_gbdt.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt8 -o run -- python $R/bench.py --steps 10 --warmup 2 --train-rows 1312500 --test-rows 62500 > $O/prof_gbdt8.log 2>&1 || { tail -20 $O/prof_gbdt8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_leaf -o run -- python $R/bench.py --steps 4 --warmup 1 --policy loss > $O/prof_leaf.log 2>&1 || { tail -20 $O/prof_leaf.log; exit 1; }
for m in linear fm ffm; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python $R/bench_sparse.py --model $m --rows 4000000 --steps 3 --warmup 1 > $O/prof_$m.log 2>&1 || { tail -20 $O/prof_$m.log; exit 1; }
done
cd $R
python tools/prof_summary.py $O/prof_gbdt/run_kernel_trace.csv > $O/gbdt_round.txt
python tools/prof_summary.py $O/prof_gbdt8/run_kernel_trace.csv > $O/gbdt_eighth_round.txt
python tools/prof_summary.py $O/prof_leaf/run_kernel_trace.csv > $O/gbdt_leafwise_round.txt
echo evidence ok
