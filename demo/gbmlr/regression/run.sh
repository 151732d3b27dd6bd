#!/usr/bin/env bash
# demo: gbmlr/regression (gbmlr). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbmlr demo/gbmlr/regression/gbmlr.conf 1 
bash bin/predict.sh gbmlr demo/data/ytklearn/machine.test.ytklearn demo/gbmlr/regression/gbmlr.conf LABEL_AND_PREDICT value rmse 
