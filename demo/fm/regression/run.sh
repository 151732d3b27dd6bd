#!/usr/bin/env bash
# demo: fm/regression (fm). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh fm demo/fm/regression/fm.conf 1 
bash bin/predict.sh fm demo/data/ytklearn/machine.test.ytklearn demo/fm/regression/fm.conf LABEL_AND_PREDICT value rmse 
