#!/usr/bin/env bash
# demo: multiclass_linear (multiclass_linear). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh multiclass_linear demo/multiclass_linear/multiclass_linear.conf 1 
bash bin/predict.sh multiclass_linear demo/data/ytklearn/dermatology.test.ytklearn demo/multiclass_linear/multiclass_linear.conf LABEL_AND_PREDICT value confusion_matrix 
