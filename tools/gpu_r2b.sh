#!/bin/bash
# GPU tests + soft-tree sparse benches (fused vs torch epilogue) + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2b
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 700 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
tail -1 $O/pytest_gpu.log
for m in linear fm ffm; do
  step 400 bench_$m.log python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1
  tail -1 $O/bench_$m.log | cut -c1-300
done
for m in gbmlr gbhsdt; do
  step 300 bench_$m.log python bench_sparse.py --model $m --rows 2000000 --steps 5 --warmup 1
  tail -1 $O/bench_$m.log | cut -c1-300
  YTK_GBST_FUSED=0 step 300 bench_${m}_torch.log python bench_sparse.py --model $m --rows 2000000 --steps 3 --warmup 1
  tail -1 $O/bench_${m}_torch.log | cut -c1-300
done
for dt in fp32 bf16; do
  step 300 bench_fm_sgd_$dt.log python bench_sparse.py --model fm --optimizer sgd --dtype $dt --rows 4000000 --steps 3 --warmup 1
  tail -1 $O/bench_fm_sgd_$dt.log | cut -c1-300
done
step 120 mfma_hist.log ./tools/microbench/mfma_hist
cat $O/mfma_hist.log
cd /tmp
for m in linear fm ffm; do
  step 400 prof_$m.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python $R/bench_sparse.py --model $m --rows 4000000 --steps 3 --warmup 1
done
step 300 prof_gbmlr.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbmlr -o run -- python $R/bench_sparse.py --model gbmlr --rows 2000000 --steps 3 --warmup 1
cd $R
echo r2b ok
