#!/usr/bin/env bash
# demo: gbhsdt/regression (gbhsdt). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbhsdt demo/gbhsdt/regression/gbhsdt.conf 1 
bash bin/predict.sh gbhsdt demo/data/ytklearn/machine.test.ytklearn demo/gbhsdt/regression/gbhsdt.conf LABEL_AND_PREDICT value rmse 
