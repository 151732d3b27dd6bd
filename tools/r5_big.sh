#!/bin/bash
# Round-5 combined run: SGD tests + benches + sparse kernel stats, full-shard PMC roofline,
# full / 1/8 round timelines, and a 2-rank shared-GPU peer bench (exchange diagnostics).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-big}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/r5_check.sh $TAG sgdtests sgd || exit 1
CFGS=1 bash tools/r5_prof_sparse.sh ${TAG}_psp || exit 1
bash tools/r5_eval.sh ${TAG}_ev full-prof prof || exit 1
bash tools/r5_roofline.sh ${TAG}_roof || exit 1
export TMPDIR=/tmp
YTK_DIST_BACKEND=gloo YTK_PEER_REDUCE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --steps 10 --warmup 3 --train-rows 2625000 \
  --test-rows 125000 --leafwise-steps 4 > $O/w2_shared.json 2> $O/w2_shared.err || { tail -30 $O/w2_shared.err; exit 1; }
cat $O/w2_shared.json
echo "big ok"
