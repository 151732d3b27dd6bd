#!/usr/bin/env bash
# demo: ffm/regression (ffm). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh ffm demo/ffm/regression/ffm.conf 1 
bash bin/predict.sh ffm demo/data/ytklearn/machine.test.ytklearn demo/ffm/regression/ffm.conf LABEL_AND_PREDICT value rmse 
