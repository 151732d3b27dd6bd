#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ffm2; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -60 $O/$log; exit 1; }; }
step 300 t.log python -u -m pytest tests/test_sparse_kernels.py tests/test_models_e2e.py -m gpu -x -q --timeout 150 --timeout-method thread
tail -2 $O/t.log
step 400 b_ffm.log python bench_sparse.py --model ffm --rows 4000000 --steps 5 --warmup 1
tail -1 $O/b_ffm.log | cut -c1-250
step 300 b_fm.log python bench_sparse.py --model fm --rows 4000000 --steps 5 --warmup 1
tail -1 $O/b_fm.log | cut -c1-250
cd /tmp
step 400 p_ffm.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ffm -o run -- python $R/bench_sparse.py --model ffm --rows 4000000 --steps 3 --warmup 1
step 300 p_fm.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fm -o run -- python $R/bench_sparse.py --model fm --rows 4000000 --steps 3 --warmup 1
cd $R
python - <<'PY'
import csv, glob
for name in ("ffm", "fm"):
    f = glob.glob(f"gpurun_out/ffm2/prof_{name}/*kernel_stats.csv")[0]
    print(name)
    for r in list(csv.DictReader(open(f)))[:6]:
        print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1000:9.1f}")
PY
echo ffm2 ok
