#!/bin/bash
# Leaf-wise row-indexed (g, h) (YTK_LW_GH_ROWS) + FFM SGD ecol prefetch: GBDT / SGD GPU
# tests, FFM SGD bench, leaf-wise 500-tree A/B, late-tree profile with the new default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-lwgh}
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gbdt_train.py tests/test_gbdt_objectives_gpu.py tests/test_gbdt_materialize.py tests/test_native_planner.py tests/test_sgd_column.py tests/test_gbdt_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench_sparse.py --model ffm --optimizer sgd --rows 4000000 --steps 3 --warmup 1 > $O/ffm.json 2> $O/ffm.err || { tail -30 $O/ffm.err; exit 1; }
cat $O/ffm.json
for g in 1 0; do
  YTK_LW_GH_ROWS=$g timeout -k 10 400 python bench.py --policy loss --steps 500 --warmup 5 > $O/leaf500_gh$g.json 2> $O/leaf500_gh$g.err || { tail -20 $O/leaf500_gh$g.err; exit 1; }
  cat $O/leaf500_gh$g.json
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pl -o run -- python3 $R/bench.py --policy loss --steps 300 --warmup 2 > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
cd $R
python3 tools/prof_summary.py $O/pl/run_kernel_trace.csv > $O/late_round.txt
python3 tools/prof_timeline.py $O/pl/run_kernel_trace.csv > $O/late_timeline.txt
head -14 $O/late_round.txt
echo "lwgh ok"
