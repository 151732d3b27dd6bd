#!/usr/bin/env bash
# demo: gbhmlr/binary_classification (gbhmlr). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbhmlr demo/gbhmlr/binary_classification/gbhmlr.conf 1 
bash bin/predict.sh gbhmlr demo/data/ytklearn/agaricus.test.ytklearn demo/gbhmlr/binary_classification/gbhmlr.conf LABEL_AND_PREDICT value auc 
