#!/bin/bash
# One-GPU A/B and debugging runs on the GPU box (one parameterised script; tools/evidence.sh is
# the round's validation run):
#   tools/ab.sh <tag> <stage> [args...]
# stages:
#   head [bench-args]        two 50-tree level-wise benches
#   stride                   20-tree headline + 1/8 shard + one-round rocprofv3 breakdown/timeline
#   ident                    partition-path identity tests (kernel variants, part scan, pool
#                            ping-pong, multi-rank one-GPU), then head + stride
#   scan [levels...]         YTK_PART_SCAN_LEVELS sweep of the 50-tree level-wise bench
#   leafscan [values...]     YTK_LW_PART_SCAN sweep of the 500-tree leaf-wise bench
#   leafsub ROWS:MAX:ALPHA.. leaf-wise small-node subtree knobs (500-tree leaf-wise bench;
#                            STEPS / WARM / PROF=1 from the environment)
#   env VAR "v1 v2 .." [bench-args]  the bench once per value of the environment variable VAR
#   sgd                      SGD GPU tests + fp32 / bf16 FM and FFM epochs
#   sgdprof                  rocprofv3 kernel statistics of the FFM SGD epoch, fp32 and bf16
#   distdbg                  two ranks on one GPU (gloo + peer exchange), gbdt_loss, verbose log
# Every GPU step runs under its own timeout; the first failure ends the script.
# Output: gpurun_out/<tag>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:?tag}
STAGE=${2:?stage}
shift 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
E8="--train-rows 1312500 --test-rows 62500"
ms() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d.get("train_loss"))' "$1"; }
bench() {  # name timeout bench-args...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; exit 1; }
}
head2() {
  for i in 1 2; do bench b$i 200 --steps 50 --warmup 5 --leafwise-steps 0 "$@"; echo "run$i $(ms "$O/b$i.json")"; done
}
stride() {
  bench s_bench 200 --steps 20 --warmup 5 --leafwise-steps 10
  echo "level+leaf $(ms "$O/s_bench.json")"
  bench s_e8 200 --steps 20 --warmup 5 --leafwise-steps 0 $E8
  echo "eighth $(ms "$O/s_e8.json")"
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/pf" -o run -- \
      python "$R/bench.py" --steps 10 --warmup 2 --leafwise-steps 0) > "$O/pf.log" 2>&1 || { tail -20 "$O/pf.log"; exit 1; }
  python tools/prof_timeline.py "$O/pf/run_kernel_trace.csv" > "$O/timeline.txt" 2>/dev/null || true
  python tools/prof_summary.py "$O/pf/run_kernel_trace.csv" > "$O/round.txt"
  rm -rf "$O/pf"
  head -8 "$O/round.txt"
}
case "$STAGE" in
  head) head2 "$@" ;;
  stride) stride ;;
  ident)
    timeout -k 10 900 python -u -m pytest tests/test_gbdt_train.py tests/test_distributed.py -m gpu -x -q \
        --timeout 300 --timeout-method thread \
        -k "kernel_variants or part_scan or pingpong or multi_rank_one_gpu" > "$O/tests.log" 2>&1 \
        || { tail -40 "$O/tests.log"; exit 1; }
    tail -1 "$O/tests.log"
    head2 && stride ;;
  scan)
    for L in ${*:-2 3 4 5}; do
      YTK_PART_SCAN_LEVELS=$L bench l$L 200 --steps 50 --warmup 5 --leafwise-steps 0
      echo "levels=$L $(ms "$O/l$L.json")"
    done ;;
  leafscan)
    for v in ${*:-2 0 2 0}; do
      YTK_LW_PART_SCAN=$v bench leaf_s$v 300 --policy loss --steps 500 --warmup 5
      echo "lw_scan=$v $(ms "$O/leaf_s$v.json")"
    done ;;
  leafsub)
    for cfg in "$@"; do
      IFS=: read -r rows mx al <<< "$cfg"
      n=l_${rows}_${mx}_${al}
      YTK_LW_SUB_ROWS=$rows YTK_LW_SUB_MAX=$mx YTK_LW_SUB_ALPHA=$al YTK_LW_PROF=${PROF:-0} \
        bench "$n" 300 --policy loss --steps "${STEPS:-500}" --warmup "${WARM:-5}"
      echo "$cfg $(ms "$O/$n.json")"
      grep -h "planner profile" "$O/$n.err" | cut -c1-600 || true
    done ;;
  env)
    var=$1 vals=$2
    shift 2
    i=0
    for v in $vals; do
      i=$((i + 1))
      (export "$var=$v"; timeout -k 10 300 python bench.py "$@" > "$O/e$i.json" 2> "$O/e$i.err") \
          || { tail -20 "$O/e$i.err"; exit 1; }
      echo "$var=$v $(ms "$O/e$i.json")"
    done ;;
  sgd)
    timeout -k 10 300 python -u -m pytest tests/test_sgd_column.py tests/test_models_e2e.py -x -q --timeout 200 \
        --timeout-method thread -m gpu -k "sgd or bf16" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
    tail -1 "$O/pytest.log"
    for cfg in "ffm fp32" "ffm bf16" "fm fp32" "fm bf16"; do
      set -- $cfg
      timeout -k 10 300 python bench_sparse.py --model "$1" --optimizer sgd --dtype "$2" --steps 3 --warmup 1 \
          > "$O/sgd_$1_$2.json" 2> "$O/sgd_$1_$2.err" || { tail -20 "$O/sgd_$1_$2.err"; exit 1; }
      tail -1 "$O/sgd_$1_$2.json" | cut -c1-330
    done ;;
  sgdprof)
    for dt in fp32 bf16; do
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p_$dt" -o run -- \
          python "$R/bench_sparse.py" --model ffm --optimizer sgd --dtype $dt --steps 2 --warmup 1) > "$O/p_$dt.log" 2>&1 \
          || { tail -20 "$O/p_$dt.log"; exit 1; }
      cp "$O/p_$dt/run_kernel_stats.csv" "$O/stats_$dt.csv"
      rm -rf "$O/p_$dt"
      python tools/kstats.py "$O/stats_$dt.csv" 8 2>/dev/null || head -9 "$O/stats_$dt.csv"
    done ;;
  distdbg)
    mkdir -p "$O/w2"
    HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=2 YTK_DIST_BACKEND=gloo YTK_HIST_SYNC=allreduce YTK_TEST_FSAMPLE=1.0 \
    YTK_PEER_REDUCE=1 YTK_COMM_LOG=1 YTK_HIST_OVERLAP_MIN_ROWS=0 YTK_PEER_OVERLAP=0 YTK_PART_SCAN_MIN_ROWS=0 \
    YTK_PEER_TIMEOUT_S=40 timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
        --master-addr 127.0.0.1 --master-port 29533 tests/dist_worker.py gbdt_loss "$O/w2" cuda > "$O/out.log" 2> "$O/err.log"
    echo "rc=$?"
    tail -40 "$O/err.log" ;;
  *) echo "unknown stage $STAGE" >&2; exit 2 ;;
esac
