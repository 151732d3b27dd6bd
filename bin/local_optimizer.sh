#!/usr/bin/env bash
# Single-node training launcher (reference: bin/local_optimizer.sh).
# One process per GPU over RCCL; the reference's CommMaster + thread ranks collapse to
# torch.distributed ranks.
#   usage: bin/local_optimizer.sh MODEL [CONF] [NUM_GPUS] [TRANSFORM_SCRIPT] [-- --set key=value ...]
#   env:   MAX_RESTARTS (default 0), MASTER_PORT, YTK_COMM_TIMEOUT, YTK_PROFILE, YTK_METRICS_JSONL
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
# Failure handling: torchrun tears the whole group down when any rank exits non-zero (or
# the RCCL watchdog times out, YTK_COMM_TIMEOUT seconds). With MAX_RESTARTS=n the job is
# relaunched up to n times with model.continue_train=true, resuming from the last dump
# (model.dump_freq) -- the reference's spark/hadoop restart loop plus resume.
run_once() {
  if [ "${gpus}" -gt 1 ]; then
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "${gpus}" --master-addr 127.0.0.1 \
      --master-port "${MASTER_PORT:-29517}" -m ytk_learn_amd.cli.train "${model_name}" "${conf}" "${targs[@]}" \
      "${extra[@]}" "$@" 2>&1 | tee -a log/master.log
  else
    python -m ytk_learn_amd.cli.train "${model_name}" "${conf}" "${targs[@]}" "${extra[@]}" "$@" 2>&1 \
      | tee -a log/master.log
  fi
}
restarts=${MAX_RESTARTS:-0}
attempt=0
until run_once $([ "${attempt}" -gt 0 ] && echo --set model.continue_train=true); do
  attempt=$((attempt + 1))
  if [ "${attempt}" -gt "${restarts}" ]; then
    echo "training failed after ${attempt} attempt(s)" | tee -a log/master_error.log
    exit 1
  fi
  echo "training failed, restart ${attempt}/${restarts} with model.continue_train=true" | tee -a log/master_warn.log
done
