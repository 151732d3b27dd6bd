# leaf-wise iteration: GBDT GPU tests + leaf-wise bench + one-round kernel timeline
set -o pipefail
O=gpurun_out/leaf; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gbdt_kernels.py tests/test_gbdt_train.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --policy loss > $O/b_leaf.log 2>&1 && tail -1 $O/b_leaf.log | cut -c1-220 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python $R/bench.py --steps 3 --warmup 1 --policy loss > $R/$O/p.log 2>&1 || exit 1
cd $R && python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/summary.txt; head -12 $O/summary.txt
