#!/usr/bin/env bash
# demo: linear/binary_classification (linear). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh linear demo/linear/binary_classification/linear.conf 1 
bash bin/predict.sh linear demo/data/ytklearn/agaricus.test.ytklearn demo/linear/binary_classification/linear.conf LABEL_AND_PREDICT value auc 
