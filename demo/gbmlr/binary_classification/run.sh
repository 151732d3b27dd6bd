#!/usr/bin/env bash
# demo: gbmlr/binary_classification (gbmlr). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbmlr demo/gbmlr/binary_classification/gbmlr.conf 1 
bash bin/predict.sh gbmlr demo/data/ytklearn/agaricus.test.ytklearn demo/gbmlr/binary_classification/gbmlr.conf LABEL_AND_PREDICT value auc 
