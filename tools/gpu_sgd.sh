# SGD extension on one MI355X: GPU tests + Criteo-shape epoch throughput (linear / FM / FFM)
set -o pipefail
O=gpurun_out/sgd; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_models_e2e.py -m gpu -x -q -k sgd --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in linear fm ffm; do
  timeout -k 10 300 python bench_sparse.py --model $m --rows 4000000 --steps 2 --warmup 1 --optimizer sgd > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | cut -c1-260
done
