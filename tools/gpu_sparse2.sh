#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sparse2; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
step 400 t.log python -u -m pytest tests/test_sparse_kernels.py tests/test_models_e2e.py tests/test_gbst_kernel.py -m gpu -x -q --timeout 150 --timeout-method thread
tail -2 $O/t.log
for m in linear fm ffm; do
  step 400 b_$m.log python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1
  tail -1 $O/b_$m.log | cut -c1-200
done
for m in gbmlr gbhsdt; do
  step 300 b_$m.log python bench_sparse.py --model $m --rows 2000000 --steps 5 --warmup 1
  tail -1 $O/b_$m.log | cut -c1-200
done
cd /tmp
step 300 p_fm.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fm -o run -- python $R/bench_sparse.py --model fm --rows 4000000 --steps 3 --warmup 1
step 300 p_lin.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_linear -o run -- python $R/bench_sparse.py --model linear --rows 4000000 --steps 3 --warmup 1
echo sparse2 ok
