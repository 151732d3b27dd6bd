#!/usr/bin/env bash
# demo: gbsdt/binary_classification (gbsdt). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbsdt demo/gbsdt/binary_classification/gbsdt.conf 1 
bash bin/predict.sh gbsdt demo/data/ytklearn/agaricus.test.ytklearn demo/gbsdt/binary_classification/gbsdt.conf LABEL_AND_PREDICT value auc 
