# leaf-wise (reference-identical 255-leaf) GBDT bench + host profile + kernel timeline
set -o pipefail
O=gpurun_out/g4; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gbdt_train.py tests/test_gbdt_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --policy loss > $O/b_loss.log 2>&1 && tail -1 $O/b_loss.log | cut -c1-300 || exit 1
timeout -k 10 300 python -m cProfile -o $O/cprof.out bench.py --steps 8 --warmup 1 --policy loss > $O/b_cprof.log 2>&1 || exit 1
python -c "import pstats; pstats.Stats('$O/cprof.out').sort_stats('tottime').print_stats(25)" > $O/cprof.txt; head -60 $O/cprof.txt | tail -35
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python $R/bench.py --steps 4 --warmup 1 --policy loss > $R/$O/p.log 2>&1 || exit 1
cd $R && python tools/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) | head -12
