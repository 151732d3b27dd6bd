#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ffmpmc; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
step() { local t=$1; shift; local log=$1; shift; timeout -s KILL $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -30 $O/$log; exit 1; }; }
step 200 pmc1.log rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python $R/bench_sparse.py --model ffm --rows 4000000 --steps 1 --warmup 0
step 200 pmc2.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc2 -o run -- python $R/bench_sparse.py --model ffm --rows 4000000 --steps 1 --warmup 0
cd $R
python tools/pmc_summary.py $(ls $O/pmc1/*counter_collection.csv | head -1) > $O/pmc1.txt
python tools/pmc_summary.py $(ls $O/pmc2/*counter_collection.csv | head -1) > $O/pmc2.txt
grep -E "ffm_" $O/pmc1.txt; grep -E "ffm_" $O/pmc2.txt
