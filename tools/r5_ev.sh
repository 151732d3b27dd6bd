#!/bin/bash
# Round-5 evidence: full GPU suite, smoke, default bench line, 500-tree level / leaf-wise,
# 1/8 shard (plain, forced-dist, leaf-wise), 5000 bins, sparse L-BFGS evaluations and SGD
# epochs. Usage: tools/r5_ev.sh <tag> [stages]; stages: suite bench b500 eighth b5k sparse sgd
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ev}
shift
STAGES=${*:-suite bench b500 eighth b5k sparse sgd}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
E8="--train-rows 1312500 --test-rows 62500"
has() { [[ " $STAGES " == *" $1 "* ]]; }
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | cut -c1-400
}
if has suite; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if has bench; then run bench 300 python bench.py; fi
if has b500; then
  run level500 400 python bench.py --steps 500 --warmup 5 --leafwise-steps 0
  run leaf500 400 python bench.py --policy loss --steps 500 --warmup 5
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
  for m in linear fm ffm gbmlr gbhsdt; do run lbfgs_$m 300 python bench_sparse.py --model $m --steps 10 --warmup 2; done
fi
if has sgd; then
  for m in linear fm ffm; do run sgd_$m 300 python bench_sparse.py --model $m --optimizer sgd --steps 3 --warmup 1; done
  run sgd_fm_bf16 300 python bench_sparse.py --model fm --optimizer sgd --dtype bf16 --steps 3 --warmup 1
fi
echo "r5_ev $TAG ok"
