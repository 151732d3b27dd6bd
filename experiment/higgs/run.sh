#!/usr/bin/env bash
# Higgs GBDT experiment: data (download or synthetic), train on N GPUs (one process per GPU,
# RCCL histogram all-reduce), predict the test split.
#   usage: experiment/higgs/run.sh [NUM_GPUS=1] [--synthetic]
set -euo pipefail
cd "$(dirname "$0")/../.."
gpus=${1:-1}
if [ "${2:-}" = "--synthetic" ]; then
  [ -s experiment/higgs/higgs.train ] || python experiment/higgs/make_synthetic.py
else
  bash experiment/higgs/get_data.sh
fi
bash bin/local_optimizer.sh gbdt experiment/higgs/local_gbdt.conf "${gpus}"
bash experiment/higgs/predict.sh
