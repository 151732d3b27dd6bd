set -o pipefail
O=gpurun_out/g5; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/dbg_spec.py 1000000 2 0,1 > $O/spec.log 2>&1 || { tail -20 $O/spec.log; exit 1; }
grep -E "booster|identical|batches" $O/spec.log
timeout -k 10 200 python tools/dbg_cmp.py 1000000 level 1 > $O/cmp.log 2>&1 && grep identical $O/cmp.log
timeout -k 10 200 python bench.py --steps 30 --warmup 3 > $O/b_full.log 2>&1 && tail -1 $O/b_full.log | cut -c1-400 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --policy loss > $O/b_loss.log 2>&1 && tail -1 $O/b_loss.log | cut -c1-400 || exit 1
