#!/bin/bash
# Round-2 final evidence: GPU tests, headline bench (level-wise + leaf-wise keys), 1/8-shard
# bench, one-round kernel timelines (level, leaf), two PMC passes for the roofline table.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2h
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -1 $O/pytest_gpu.log
step 300 bench.log python bench.py --steps 50 --warmup 5
tail -1 $O/bench.log
step 300 bench_eighth.log python bench.py --steps 50 --warmup 5 --leafwise-steps 0 --train-rows 1312500 --test-rows 62500
tail -1 $O/bench_eighth.log | cut -c1-200
cd /tmp
step 300 prof_level.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_level -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
step 300 prof_leaf.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_leaf -o run -- python $R/bench.py --steps 6 --warmup 2 --policy loss
step 120 pmc1.log rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python $R/bench.py --steps 2 --warmup 1 --leafwise-steps 0
step 120 pmc2.log rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $O/pmc2 -o run -- python $R/bench.py --steps 2 --warmup 1 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof_level/*kernel_trace.csv | head -1) > $O/level_round.txt
python tools/prof_summary.py $(ls $O/prof_leaf/*kernel_trace.csv | head -1) > $O/leaf_round.txt
head -8 $O/level_round.txt
head -8 $O/leaf_round.txt
echo r2h ok
