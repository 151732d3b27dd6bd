#!/bin/bash
# PMC roofline of one level-wise bench (full shard by default): three counter passes, each its
# own run (no tracing domains), then tools/roofline.py. Usage: tools/r5_roofline.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-roof}
shift
ARGS=${*:---steps 4 --warmup 2 --leafwise-steps 0}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d $O/pmc$i -o run -- python3 $R/bench.py $ARGS > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
done
cd $R
python3 tools/roofline.py $O/pmc1/run_counter_collection.csv $O/pmc2/run_counter_collection.csv $O/pmc3/run_counter_collection.csv > $O/roofline.md
python3 tools/pmc_summary.py $O/pmc3/run_counter_collection.csv > $O/wave_states.txt
head -20 $O/roofline.md
echo "roofline ok"
