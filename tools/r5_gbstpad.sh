#!/bin/bash
# Soft-tree rows padded to line multiples (YTK_GBST_PAD): GBST GPU tests + L-BFGS evaluation
# A/B for gbmlr / gbhmlr k=16 + kernel stats of gbmlr with the padding.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gbstpad}
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gbst_kernel.py tests/test_models_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in gbmlr gbhmlr; do
  for pad in 1 0; do
    YTK_GBST_PAD=$pad timeout -k 10 300 python bench_sparse.py --model $m --steps 10 --warmup 2 > $O/${m}_pad$pad.json 2> $O/${m}_pad$pad.err || { tail -30 $O/${m}_pad$pad.err; exit 1; }
    tail -1 $O/${m}_pad$pad.json
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench_sparse.py --model gbmlr --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo "gbstpad ok"
