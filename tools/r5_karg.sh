#!/bin/bash
# Device kernargs A/B on the default bench line (level-wise + the leaf-wise extra key) and a
# 200-tree leaf-wise run. Usage: tools/r5_karg.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-karg}
mkdir -p $O
cd $R
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("leafwise_s_per_tree"), d.get("train_loss"))')"
}
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k run bench_k$k 300 python bench.py
  HIP_FORCE_DEV_KERNARG=$k run leaf200_k$k 300 python bench.py --policy loss --steps 200 --warmup 3
done
echo "karg ok"
