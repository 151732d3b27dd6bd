#!/usr/bin/env bash
# Fetch HIGGS.csv (UCI) and split it into higgs.train (10.5M) / higgs.test (0.5M) in
# ytk-learn format. Without network access use make_synthetic.py for Higgs-shaped data.
set -euo pipefail
cd "$(dirname "$0")"
if [ -s higgs.train ] && [ -s higgs.test ]; then echo "higgs.train / higgs.test already exist"; exit 0; fi
if [ ! -s HIGGS.csv ]; then
  if [ ! -s HIGGS.csv.gz ]; then
    url=https://archive.ics.uci.edu/ml/machine-learning-databases/00280/HIGGS.csv.gz
    echo "downloading ${url}"
    curl -fL -o HIGGS.csv.gz "${url}" || wget -O HIGGS.csv.gz "${url}" || {
      echo "download failed (no network?): run 'python make_synthetic.py' for synthetic Higgs-shaped data"; exit 1; }
  fi
  gunzip -k HIGGS.csv.gz
fi
python higgs2ytklearn.py HIGGS.csv higgs.train higgs.test
