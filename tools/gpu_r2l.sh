#!/bin/bash
# GPU tests; partition microbench (standalone kernel, pipelined by default) vs
# YTK_PART_PREFETCH=0; 2-rank gloo bench on the one GPU (the multi-GPU level path uses the
# standalone partition) with and without the prefetch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2l
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -1 $O/pytest_gpu.log
step 200 part_pf.log python tools/microbench/part_bench.py
YTK_PART_PREFETCH=0 step 200 part_nopf.log python tools/microbench/part_bench.py
paste $O/part_nopf.log $O/part_pf.log | cut -c1-160
for v in 0 2; do
  YTK_PART_PREFETCH=$v YTK_DIST_BACKEND=gloo step 300 dist2_pf$v.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$v bench.py --gpus 2 --steps 10 --warmup 2 --leafwise-steps 0 --train-rows 4000000 --test-rows 200000
  tail -1 $O/dist2_pf$v.log | cut -c1-160
done
echo r2l ok
