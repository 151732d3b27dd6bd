# quick GPU iteration: gpu tests, full + 1/8-shard bench, 1/8-shard one-round kernel timeline
set -o pipefail
O=gpurun_out/iter; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --steps 30 --warmup 3 > $O/b_full.log 2>&1 && tail -1 $O/b_full.log | cut -c1-200 || exit 1
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --train-rows 1312500 --test-rows 62500 > $O/b_eighth.log 2>&1 && tail -1 $O/b_eighth.log | cut -c1-200 || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof8 -o run -- python $R/bench.py --steps 6 --warmup 2 --train-rows 1312500 --test-rows 62500 > $R/$O/p8.log 2>&1 || exit 1
cd $R && python tools/prof_summary.py $(ls $O/prof8/*kernel_trace.csv | head -1) > $O/p8_summary.txt; cat $O/p8_summary.txt
