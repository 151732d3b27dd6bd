#!/bin/bash
# Round-2 GPU pass: GPU tests, whole-round bench (+ leaf-wise extra keys), 5000-bin
# benches, kernel trace of one level-wise round, and PMC counter passes for the
# roofline table. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2
rm -rf $O && mkdir -p $O
export TMPDIR=/tmp
cd $R
step() { local t=$1; shift; local log=$1; shift; timeout -k 10 $t "$@" > $O/$log 2>&1 || { echo "FAILED: $log"; tail -40 $O/$log; exit 1; }; }
if [ -z "$SKIP_TESTS" ]; then
  step 500 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  tail -1 $O/pytest_gpu.log
fi
step 300 bench.log python bench.py --steps 50 --warmup 5
tail -1 $O/bench.log
step 300 bench_5000_level.log python bench.py --steps 20 --warmup 3 --bins 5000 --leafwise-steps 0
tail -1 $O/bench_5000_level.log | cut -c1-400
step 300 bench_5000_loss.log python bench.py --steps 10 --warmup 2 --bins 5000 --policy loss
tail -1 $O/bench_5000_loss.log | cut -c1-400
cd /tmp
step 300 prof_level.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_level -o run -- python $R/bench.py --steps 10 --warmup 2 --leafwise-steps 0
step 300 prof_w5000.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w5000 -o run -- python $R/bench.py --steps 4 --warmup 1 --bins 5000 --leafwise-steps 0
step 120 pmc1.log rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python $R/bench.py --steps 2 --warmup 1 --leafwise-steps 0
step 120 pmc2.log rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $O/pmc2 -o run -- python $R/bench.py --steps 2 --warmup 1 --leafwise-steps 0
cd $R
python tools/prof_summary.py $(ls $O/prof_level/*kernel_trace.csv | head -1) > $O/level_round.txt
python tools/prof_summary.py $(ls $O/prof_w5000/*kernel_trace.csv | head -1) > $O/w5000_round.txt
head -20 $O/level_round.txt
head -20 $O/w5000_round.txt
echo r2 ok
