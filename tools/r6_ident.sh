# partition-path identity tests + headline A/B + one-round profile: tools/r6_ident.sh <tag>
set -o pipefail
T=${1:-id}; O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gbdt_train.py tests/test_distributed.py -m gpu -x -q \
    --timeout 300 --timeout-method thread \
    -k "kernel_variants or part_scan or pingpong or multi_rank_one_gpu" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r6_head.sh $T/hd && bash tools/r6_stride.sh $T/sc
