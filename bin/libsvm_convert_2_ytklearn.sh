#!/usr/bin/env bash
# LibSVM -> ytk-learn format (reference: bin/libsvm_convert_2_ytklearn.sh).
#   usage: bin/libsvm_convert_2_ytklearn.sh MODE IN OUT [FS_SCHEME]
#   MODE: binary_classification@neg,pos | multi_classification@l0,l1,... | regression
set -euo pipefail
cd "$(dirname "$0")/.."
python -m ytk_learn_amd.tools.libsvm_convert "${1:?mode}" "###" "," "," ":" "${4:-local}" "${2:?in}" "${3:?out}"
