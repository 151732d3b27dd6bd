#!/usr/bin/env bash
# Single-node training launcher (reference: bin/local_optimizer.sh).
# One process per GPU over RCCL; the reference's CommMaster + thread ranks collapse to
# torch.distributed ranks.
#   usage: bin/local_optimizer.sh MODEL [CONF] [NUM_GPUS] [TRANSFORM_SCRIPT] [-- --set key=value ...]
#   MODEL: linear | multiclass_linear | fm | ffm | gbdt | gbmlr | gbsdt | gbhmlr | gbhsdt
set -euo pipefail
cd "$(dirname "$0")/.."
model_name=${1:?"model name required (linear, fm, ffm, gbdt, gbmlr, gbsdt, gbhmlr, gbhsdt, multiclass_linear)"}
conf=${2:-config/model/${model_name}.conf}
gpus=${3:-1}
transform=${4:-}
shift $(( $# < 4 ? $# : 4 ))
[ "${1:-}" = "--" ] && shift
extra=("$@")
targs=()
[ -n "${transform}" ] && targs+=(--transform-script "${transform}")
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
mkdir -p log
echo "model name:${model_name}, config:${conf}, gpus:${gpus}"
if [ "${gpus}" -gt 1 ]; then
  python -m torch.distributed.run --nnodes=1 --nproc-per-node "${gpus}" --master-addr 127.0.0.1 \
    --master-port "${MASTER_PORT:-29517}" -m ytk_learn_amd.cli.train "${model_name}" "${conf}" "${targs[@]}" "${extra[@]}" \
    2>&1 | tee -a log/master.log
else
  python -m ytk_learn_amd.cli.train "${model_name}" "${conf}" "${targs[@]}" "${extra[@]}" 2>&1 | tee -a log/master.log
fi
