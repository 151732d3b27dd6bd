#!/usr/bin/env bash
# Multi-node training (reference: bin/cluster_optimizer.sh, which ssh-launched one JVM per
# host). Here every node runs this script with its NODE_RANK; ranks rendezvous at MASTER_ADDR.
#   usage: NODE_RANK=r NNODES=n MASTER_ADDR=host bin/cluster_optimizer.sh MODEL CONF GPUS_PER_NODE [TRANSFORM]
set -euo pipefail
cd "$(dirname "$0")/.."
model_name=${1:?model}; conf=${2:?conf}; gpus=${3:-8}; transform=${4:-}
targs=(); [ -n "${transform}" ] && targs+=(--transform-script "${transform}")
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
python -m torch.distributed.run --nnodes "${NNODES:?}" --node-rank "${NODE_RANK:?}" --nproc-per-node "${gpus}" \
  --master-addr "${MASTER_ADDR:?}" --master-port "${MASTER_PORT:-29517}" \
  -m ytk_learn_amd.cli.train "${model_name}" "${conf}" "${targs[@]}"
