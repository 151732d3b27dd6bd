#!/usr/bin/env bash
# Batch-predict experiment/higgs/higgs.test with the trained model (auc + logloss).
set -euo pipefail
cd "$(dirname "$0")/../.."
bash bin/predict.sh gbdt experiment/higgs/higgs.test experiment/higgs/local_gbdt.conf LABEL_AND_PREDICT value auc
