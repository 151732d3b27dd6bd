#!/bin/bash
# Evidence run on the GPU box (one parameterised script for the round's validation):
#   tools/evidence.sh <tag> [stages]
# stages (default: suite bench b500 eighth b5k sparse sgd prof):
#   suite   GPU test suite + smoke()
#   bench   the default headline line (bench.py)
#   b500    500-tree level-wise and leaf-wise runs
#   eighth  the 1/8 shard (plain, forced-dist, leaf-wise)
#   b5k     5000 bins (level, leaf)
#   sparse  L-BFGS evaluations (linear, fm, ffm, multiclass, gbmlr, gbhsdt)
#   sgd     SGD epochs (linear, fm fp32 / bf16, ffm)
#   prof    rocprofv3 kernel statistics + one-round breakdowns (full data, 1/8 shard, leaf-wise)
#   roof    PMC roofline of the level-wise bench (full data and 1/8 shard): three counter passes,
#           each its own run with no tracing domains, then tools/roofline.py
# Every GPU step runs under its own timeout; the first failure ends the script (nothing more
# runs on the GPU in that call). Output: gpurun_out/<tag>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-ev}
shift
STAGES=${*:-suite bench b500 eighth b5k sparse sgd prof}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
E8="--train-rows 1312500 --test-rows 62500"
has() { [[ " $STAGES " == *" $1 "* ]]; }
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -30 "$O/$n.err"; exit 1; }
  tail -1 "$O/$n.json" | cut -c1-400
}
prof() {  # name timeout python-args...
  local n=$1 t=$2; shift 2
  (cd /tmp && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$n.d" -o run -- \
      python "$R/bench.py" "$@") > "$O/$n.log" 2>&1 || { tail -20 "$O/$n.log"; exit 1; }
  python tools/prof_summary.py "$O/$n.d/run_kernel_trace.csv" > "$O/${n}_round.txt"
  cp "$O/$n.d/run_kernel_stats.csv" "$O/${n}_kernel_stats.csv"
  rm -rf "$O/$n.d"
  head -12 "$O/${n}_round.txt"
}
if has suite; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
      > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
  tail -1 "$O/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
      || { tail -30 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
if has bench; then run bench 300 python bench.py --steps 20 --warmup 5; fi
if has b500; then
  run level500 400 python bench.py --steps 500 --warmup 5 --leafwise-steps 0
  run leaf500 600 python bench.py --policy loss --steps 500 --warmup 5
fi
if has eighth; then
  run eighth_plain 300 python bench.py --steps 50 --warmup 5 $E8
  YTK_FORCE_DIST=1 MASTER_PORT=29641 run eighth_forced 300 python bench.py --steps 50 --warmup 5 $E8
  run eighth_leaf 300 python bench.py --policy loss --steps 50 --warmup 5 $E8
fi
if has b5k; then
  run bins5000 300 python bench.py --bins 5000 --steps 20 --warmup 3 --leafwise-steps 0
  run bins5000_leaf 300 python bench.py --bins 5000 --policy loss --steps 20 --warmup 3
fi
if has sparse; then
  for m in linear fm ffm multiclass gbmlr gbhsdt; do
    run lbfgs_$m 300 python bench_sparse.py --model $m --steps 10 --warmup 2
  done
fi
if has sgd; then
  for m in linear fm ffm; do run sgd_$m 300 python bench_sparse.py --model $m --optimizer sgd --steps 3 --warmup 1; done
  run sgd_fm_bf16 300 python bench_sparse.py --model fm --optimizer sgd --dtype bf16 --steps 3 --warmup 1
  run sgd_ffm_bf16 300 python bench_sparse.py --model ffm --optimizer sgd --dtype bf16 --steps 3 --warmup 1
fi
if has prof; then
  prof prof_full 300 --steps 10 --warmup 2 --leafwise-steps 0
  prof prof_e8 300 --steps 10 --warmup 2 --leafwise-steps 0 $E8
  prof prof_leaf 300 --policy loss --steps 10 --warmup 40 --leafwise-steps 0
fi
roof() {  # name bench-args...
  local n=$1; shift
  local i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
      "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d "$O/${n}_pmc$i" -o run -- \
        python3 "$R/bench.py" "$@") > "$O/${n}_pmc$i.log" 2>&1 || { tail -20 "$O/${n}_pmc$i.log"; exit 1; }
  done
  python3 tools/roofline.py "$O/${n}_pmc1/run_counter_collection.csv" "$O/${n}_pmc2/run_counter_collection.csv" \
      "$O/${n}_pmc3/run_counter_collection.csv" > "$O/${n}.md"
  python3 tools/pmc_summary.py "$O/${n}_pmc3/run_counter_collection.csv" > "$O/${n}_wave_states.txt"
  rm -rf "$O/${n}_pmc1" "$O/${n}_pmc2" "$O/${n}_pmc3"
  head -12 "$O/${n}.md"
}
if has roof; then
  roof roofline_full --steps 4 --warmup 2 --leafwise-steps 0
  roof roofline_eighth --steps 4 --warmup 2 --leafwise-steps 0 $E8
fi
echo "evidence $TAG ok"
