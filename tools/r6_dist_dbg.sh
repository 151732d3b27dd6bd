set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dd; mkdir -p $O; cd $GRAFT_REPO_ROOT
for v in 4000000 0; do
  echo "scan_min_rows=$v"
  YTK_TEST_PART_SCAN_MIN_ROWS=$v timeout -k 10 200 python -u -m pytest "tests/test_distributed.py::test_gpu_builders_multi_rank_one_gpu[gbdt_loss-2-peer]" -x -v --timeout 150 --timeout-method thread --basetemp=$O/pt$v > $O/t$v.log 2>&1
  rc=$?; tail -3 $O/t$v.log; [ $rc -ne 0 ] && exit $rc
done
