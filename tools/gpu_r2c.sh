#!/bin/bash
# Higgs-scale load + preprocess benchmark (11M-line text file: parse, dictionary, dense,
# missing fill, binning) -- cold-ish and warm page cache runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2c
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
ROWS=${ROWS:-10500000}
step 600 load_1.log python tools/bench_load.py --rows $ROWS --test-rows 500000 --dir /tmp/higgs_load --out $O/load_1.json
cat $O/load_1.json
step 300 load_2.log python tools/bench_load.py --rows $ROWS --test-rows 500000 --dir /tmp/higgs_load --out $O/load_2.json
cat $O/load_2.json
rm -rf /tmp/higgs_load
echo r2c ok
