#!/bin/bash
# FFM SGD A/B (pair-gradient gathers from V vs the field-major copy Vt) + the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-vt}
mkdir -p $O
export TMPDIR=/tmp
cd $R
for vt in 0 1; do
  YTK_SGD_FFM_VT=$vt timeout -k 10 300 python bench_sparse.py --model ffm --optimizer sgd --rows 4000000 --steps 3 --warmup 1 > $O/ffm_vt$vt.json 2> $O/ffm_vt$vt.err || { tail -30 $O/ffm_vt$vt.err; exit 1; }
  cat $O/ffm_vt$vt.json
done
if [ "${2:-}" = "suite" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
echo "vt ok"
