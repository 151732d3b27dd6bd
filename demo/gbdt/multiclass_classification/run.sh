#!/usr/bin/env bash
# demo: gbdt/multiclass_classification (gbdt). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbdt demo/gbdt/multiclass_classification/gbdt.conf 1 
bash bin/predict.sh gbdt demo/data/ytklearn/dermatology.test.ytklearn demo/gbdt/multiclass_classification/gbdt.conf LABEL_AND_PREDICT value confusion_matrix 
