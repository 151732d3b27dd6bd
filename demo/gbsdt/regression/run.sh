#!/usr/bin/env bash
# demo: gbsdt/regression (gbsdt). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbsdt demo/gbsdt/regression/gbsdt.conf 1 
bash bin/predict.sh gbsdt demo/data/ytklearn/machine.test.ytklearn demo/gbsdt/regression/gbsdt.conf LABEL_AND_PREDICT value rmse 
