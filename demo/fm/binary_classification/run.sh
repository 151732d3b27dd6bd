#!/usr/bin/env bash
# demo: fm/binary_classification (fm). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh fm demo/fm/binary_classification/fm.conf 1 
bash bin/predict.sh fm demo/data/ytklearn/agaricus.test.ytklearn demo/fm/binary_classification/fm.conf LABEL_AND_PREDICT value auc 
