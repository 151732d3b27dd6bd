#!/bin/bash
# Exact greedy with float (g, h) moved per position: tests (HIP == tensor engine), bench,
# kernel stats of one round.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-exact}
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_exact_greedy.py tests/test_exact_maker.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python tools/bench_exact.py > $O/bench_exact.json 2> $O/bench_exact.err || { tail -30 $O/bench_exact.err; exit 1; }
tail -1 $O/bench_exact.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/bench_exact.py --rounds 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
python3 tools/prof_summary.py $O/prof/run_kernel_trace.csv > $O/round.txt 2>/dev/null || true
head -14 $O/round.txt
echo "exact ok"
