set -o pipefail
O=gpurun_out/bf1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sgd_column.py tests/test_models_e2e.py -x -q --timeout 200 --timeout-method thread -m gpu -k "sgd or bf16" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "ffm fp32" "ffm bf16" "fm fp32" "fm bf16"; do set -- $cfg
  timeout -k 10 300 python bench_sparse.py --model $1 --optimizer sgd --dtype $2 --steps 3 --warmup 1 > $O/sgd_$1_$2.json 2> $O/sgd_$1_$2.err || { tail -20 $O/sgd_$1_$2.err; exit 1; }
  tail -1 $O/sgd_$1_$2.json | cut -c1-330
done
