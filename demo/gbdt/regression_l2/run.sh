#!/usr/bin/env bash
# demo: gbdt/regression_l2 (gbdt). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/../../.."
bash demo/prepare_data.sh
bash bin/local_optimizer.sh gbdt demo/gbdt/regression_l2/gbdt.conf 1 demo/gbdt/regression_l2/transform.py
bash bin/predict.sh gbdt demo/data/libsvm/machine.test.libsvm demo/gbdt/regression_l2/gbdt.conf LABEL_AND_PREDICT value rmse demo/gbdt/regression_l2/transform.py
