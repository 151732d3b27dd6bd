#!/bin/bash
# Round-5 checks: grid-barrier microbench, new GPU tests (column SGD, soft-tree epilogue, peer
# fault), SGD epoch benches (fp32 / bf16 FM, FFM, linear) and the GBMLR / GBHSDT evaluations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sgd}
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -x tools/microbench/grid_barrier ]; then
  timeout -k 10 60 tools/microbench/grid_barrier > $O/grid_barrier.txt 2>&1 || { cat $O/grid_barrier.txt; exit 1; }
  cat $O/grid_barrier.txt
fi
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sgd_column.py tests/test_gbst_kernel.py "tests/test_distributed.py::test_lbfgs_peer_dropped_exchange_raises" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in "fm fp32" "fm bf16" "ffm fp32" "linear fp32"; do
  set -- $cfg
  timeout -k 10 300 python bench_sparse.py --model $1 --optimizer sgd --dtype $2 --rows 4000000 --steps 3 --warmup 1 > $O/sgd_$1_$2.json 2> $O/sgd_$1_$2.err || { tail -30 $O/sgd_$1_$2.err; exit 1; }
  cat $O/sgd_$1_$2.json
done
for m in gbmlr gbhsdt; do
  timeout -k 10 300 python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1 > $O/lbfgs_$m.json 2> $O/lbfgs_$m.err || { tail -30 $O/lbfgs_$m.err; exit 1; }
  cat $O/lbfgs_$m.json
done
echo "r5_sgd ok"
