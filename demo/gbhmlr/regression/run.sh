#!/usr/bin/env bash
# demo: gbhmlr/regression (gbhmlr). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbhmlr demo/gbhmlr/regression/gbhmlr.conf 1 
bash bin/predict.sh gbhmlr demo/data/ytklearn/machine.test.ytklearn demo/gbhmlr/regression/gbhmlr.conf LABEL_AND_PREDICT value rmse 
