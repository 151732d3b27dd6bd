set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lws}; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gbdt_train.py tests/test_distributed.py -x -q --timeout 200 --timeout-method thread -m gpu -k "leafwise or kernel_variants" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for L in 0 2 0 2; do
  YTK_LW_PART_SCAN=$L timeout -k 10 300 python bench.py --policy loss --steps 500 --warmup 5 > $O/l$L.json 2> $O/l$L.err || { tail -20 $O/l$L.err; exit 1; }
  echo "lw_scan=$L $(tail -1 $O/l$L.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["train_loss"])')"
done
