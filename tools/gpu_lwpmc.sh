#!/bin/bash
# PMC passes over the leaf-wise 255 bench (partition / histogram / planner kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lwpmc; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
step() { local t=$1; shift; local log=$1; shift; timeout -s KILL $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -30 $O/$log; exit 1; }; }
step 150 pmc1.log rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python $R/bench.py --steps 2 --warmup 1 --policy loss --leafwise-steps 0
step 150 pmc2.log rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $O/pmc2 -o run -- python $R/bench.py --steps 2 --warmup 1 --policy loss --leafwise-steps 0
cd $R
python tools/pmc_summary.py $(ls $O/pmc1/*counter_collection.csv | head -1) > $O/pmc1.txt
python tools/pmc_summary.py $(ls $O/pmc2/*counter_collection.csv | head -1) > $O/pmc2.txt
head -8 $O/pmc1.txt; head -8 $O/pmc2.txt
