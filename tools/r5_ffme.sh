#!/bin/bash
# FFM SGD pair terms: tests, then A/B of the forward-written pair terms (YTK_SGD_FFM_E_GB=16)
# against the gather kernel (=0), then a kernel-stats profile of the E path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ffme}
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_sgd_column.py tests/test_sparse_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for eg in 16 0; do
  YTK_SGD_FFM_E_GB=$eg timeout -k 10 300 python bench_sparse.py --model ffm --optimizer sgd --rows 4000000 --steps 3 --warmup 1 > $O/ffm_e$eg.json 2> $O/ffm_e$eg.err || { tail -30 $O/ffm_e$eg.err; exit 1; }
  cat $O/ffm_e$eg.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench_sparse.py --model ffm --optimizer sgd --rows 4000000 --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
echo "ffme ok"
