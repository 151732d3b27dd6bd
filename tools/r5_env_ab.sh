#!/bin/bash
# Runtime-environment A/B of the level-wise bench (full and 1/8 shard): HIP_FORCE_DEV_KERNARG
# (kernel arguments in device memory) on / off. Usage: tools/r5_env_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-envab}
mkdir -p $O
cd $R
E8="--train-rows 1312500 --test-rows 62500"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | cut -c1-120
}
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k run full_k$k 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0
  HIP_FORCE_DEV_KERNARG=$k run eighth_k$k 300 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 $E8
  HIP_FORCE_DEV_KERNARG=$k run leaf_k$k 300 python bench.py --policy loss --steps 20 --warmup 3
done
echo "envab ok"
