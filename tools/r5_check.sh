#!/bin/bash
# Round-5 check run: selected GPU tests, SGD / soft-tree benches, GBDT benches (full, 1/8
# plain + forced-dist) with a YTK_TGH_VBLOCKS sweep. Usage: tools/r5_check.sh <tag> [stages]
# stages: tests sgd gbdt sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-chk}
shift
STAGES=${*:-tests sgd ghrows gbdt sweep}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
has() { [[ " $STAGES " == *" $1 "* ]]; }
E8="--train-rows 1312500 --test-rows 62500"
if has tests; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sgd_column.py tests/test_gbst_kernel.py \
    "tests/test_distributed.py::test_lbfgs_peer_dropped_exchange_raises" "tests/test_distributed.py::test_leafwise_rccl_loop_fixed_messages" \
    "tests/test_distributed.py::test_rccl_world1_forced_dist" "tests/test_distributed.py::test_peer_world1_forced_dist" \
    "tests/test_distributed.py::test_rccl_world1_capture_failure_falls_back" > $O/tests.log 2>&1 || { tail -80 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
if has sgdtests; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sgd_column.py > $O/sgdtests.log 2>&1 || { tail -80 $O/sgdtests.log; exit 1; }
  tail -2 $O/sgdtests.log
fi
if has tests2; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    "tests/test_distributed.py::test_lbfgs_peer_dropped_exchange_raises" "tests/test_distributed.py::test_leafwise_rccl_loop_fixed_messages" \
    "tests/test_distributed.py::test_rccl_world1_forced_dist" "tests/test_distributed.py::test_peer_world1_forced_dist" \
    "tests/test_distributed.py::test_rccl_world1_capture_failure_falls_back" "tests/test_distributed.py::test_lbfgs_peer_gradient_allreduce_one_gpu" \
    "tests/test_distributed.py::test_peer_primitives_one_gpu" > $O/tests2.log 2>&1 || { tail -80 $O/tests2.log; exit 1; }
  tail -2 $O/tests2.log
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_distributed.py \
    -k "test_gpu_builders_multi_rank_one_gpu and (peer_overlap or gbdt_loss-3-allreduce or gbdt_loss-2-owner or gbdt-2-peer])" \
    > $O/tests3.log 2>&1 || { tail -80 $O/tests3.log; exit 1; }
  cp $O/tests3.log $O/tests2b.log
  tail -2 $O/tests2.log
fi
if has sgd; then
  for cfg in "fm fp32" "fm bf16" "ffm fp32" "linear fp32"; do
    set -- $cfg
    timeout -k 10 300 python bench_sparse.py --model $1 --optimizer sgd --dtype $2 --rows 4000000 --steps 3 --warmup 1 > $O/sgd_$1_$2.json 2> $O/sgd_$1_$2.err || { tail -30 $O/sgd_$1_$2.err; exit 1; }
    cat $O/sgd_$1_$2.json
  done
  for m in gbmlr gbhsdt; do
    timeout -k 10 300 python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1 > $O/lbfgs_$m.json 2> $O/lbfgs_$m.err || { tail -30 $O/lbfgs_$m.err; exit 1; }
    cat $O/lbfgs_$m.json
  done
fi
if has gbdt; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 > $O/eighth_plain.json 2> $O/eighth_plain.err || { tail -30 $O/eighth_plain.err; exit 1; }
  cat $O/eighth_plain.json
  YTK_FORCE_DIST=1 MASTER_PORT=29621 timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 > $O/eighth_forced.json 2> $O/eighth_forced.err || { tail -30 $O/eighth_forced.err; exit 1; }
  cat $O/eighth_forced.json
fi
if has ghrows; then
  for gm in 1 2; do
    YTK_GH_ROWS=$gm timeout -k 10 300 python bench.py --steps 30 --warmup 5 --leafwise-steps 0 > $O/full_gh$gm.json 2> $O/full_gh$gm.err || { tail -30 $O/full_gh$gm.err; exit 1; }
    cat $O/full_gh$gm.json
    YTK_GH_ROWS=$gm timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 --leafwise-steps 0 > $O/eighth_gh$gm.json 2> $O/eighth_gh$gm.err || { tail -30 $O/eighth_gh$gm.err; exit 1; }
    cat $O/eighth_gh$gm.json
  done
fi
if has sweep; then
  for vb in 1024 512; do
    YTK_TGH_VBLOCKS=$vb timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 --leafwise-steps 0 > $O/eighth_vb$vb.json 2> $O/eighth_vb$vb.err || { tail -30 $O/eighth_vb$vb.err; exit 1; }
    cat $O/eighth_vb$vb.json
    YTK_TGH_VBLOCKS=$vb timeout -k 10 300 python bench.py --steps 20 --warmup 5 --leafwise-steps 0 > $O/full_vb$vb.json 2> $O/full_vb$vb.err || { tail -30 $O/full_vb$vb.err; exit 1; }
    cat $O/full_vb$vb.json
  done
fi
echo "r5_check $TAG ok"
