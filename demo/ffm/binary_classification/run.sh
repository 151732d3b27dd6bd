#!/usr/bin/env bash
# demo: ffm/binary_classification (ffm). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh ffm demo/ffm/binary_classification/ffm.conf 1 
bash bin/predict.sh ffm demo/data/ytklearn/agaricus.test.ytklearn demo/ffm/binary_classification/ffm.conf LABEL_AND_PREDICT value auc 
