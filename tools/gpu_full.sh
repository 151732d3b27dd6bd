#!/bin/bash
# full GPU test suite + headline bench (level-wise 6 + leaf-wise 255 extra keys)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/full; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
tail -2 $O/pytest_gpu.log
step 400 bench.log python bench.py
tail -1 $O/bench.log | cut -c1-900
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
tail -2 $O/smoke.log
echo full ok
