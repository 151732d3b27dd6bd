#!/bin/bash
# Exchange-overlap A/B on two ranks sharing the one GPU (gloo host group, peer-memory exchange):
# full Higgs rows and 1/4 of them, YTK_PEER_OVERLAP 0 / 1. Two processes on one device contend
# for it, so this checks the path and the JSON line rather than xGMI timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ovl}
mkdir -p $O
export TMPDIR=/tmp
cd $R
port=29671
for rows in "10500000 500000" "2625000 125000"; do
  set -- $rows
  for ov in 0 1; do
    port=$((port + 1))
    YTK_DIST_BACKEND=gloo YTK_PEER_REDUCE=1 YTK_PEER_OVERLAP=$ov timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node=2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 10 --warmup 3 \
      --train-rows $1 --test-rows $2 --leafwise-steps 0 > $O/w2_r$1_ov$ov.json 2> $O/w2_r$1_ov$ov.err || { tail -30 $O/w2_r$1_ov$ov.err; exit 1; }
    cat $O/w2_r$1_ov$ov.json
  done
done
echo "overlap ok"
