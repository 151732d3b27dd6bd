#!/usr/bin/env bash
# Cygwin launcher (reference: bin/cygwin_local_optimizer.sh): same as bin/local_optimizer.sh
# with Windows-style python on PATH; single process.
#   usage: bin/cygwin_local_optimizer.sh MODEL [CONF] [TRANSFORM_SCRIPT]
set -euo pipefail
cd "$(dirname "$0")/.."
model_name=${1:?model}
conf=${2:-config/model/${model_name}.conf}
mkdir -p log
if [ -n "${3:-}" ]; then
  python -m ytk_learn_amd.cli.train "${model_name}" "${conf}" --transform-script "$3" 2>&1 | tee -a log/master.log
else
  python -m ytk_learn_amd.cli.train "${model_name}" "${conf}" 2>&1 | tee -a log/master.log
fi
