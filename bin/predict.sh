#!/usr/bin/env bash
# Offline batch prediction (reference: bin/predict.sh -> Predicts).
#   usage: bin/predict.sh MODEL FILE_OR_DIR [CONF] [SAVE_MODE] [PREDICT_TYPE] [EVAL_METRICS] [TRANSFORM_SCRIPT]
#   SAVE_MODE: PREDICT_RESULT_ONLY | LABEL_AND_PREDICT | PREDICT_AS_FEATURE ; PREDICT_TYPE: value | leafid
set -euo pipefail
cd "$(dirname "$0")/.."
model_name=${1:?model}; file_name=${2:?file or dir}
conf=${3:-config/model/${model_name}.conf}
mode=${4:-PREDICT_RESULT_ONLY}; ptype=${5:-value}; metrics=${6:-auc,mae}; transform=${7:-}
need_py=false; [ -n "${transform}" ] && need_py=true
mkdir -p log
python -m ytk_learn_amd.cli.predict "${conf}" "${model_name}" "${file_name}" "${need_py}" "${transform}" \
  "${mode}" "_${model_name}_${mode}" 100 "${metrics}" "${ptype}" --device "${YTK_DEVICE:-cpu}" 2>&1 | tee -a log/info.log
