#!/usr/bin/env bash
# demo: linear/regression (linear). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh linear demo/linear/regression/linear.conf 1 
bash bin/predict.sh linear demo/data/ytklearn/machine.test.ytklearn demo/linear/regression/linear.conf LABEL_AND_PREDICT value rmse 
