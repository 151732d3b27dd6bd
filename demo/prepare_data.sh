#!/usr/bin/env bash
# Convert the demo LibSVM datasets into ytk-learn format + the dictionaries the demos use.
#   source: $YTK_DEMO_DATA (default demo/data/libsvm) holding agaricus/dermatology/machine
#           .{train,test}.libsvm (the public files the reference ships under demo/data/libsvm)
#   output: demo/data/ytklearn/*.ytklearn, *.feat_dict (feature names), *.field.dict (FFM fields)
set -euo pipefail
cd "$(dirname "$0")/.."
src=${YTK_DEMO_DATA:-demo/data/libsvm}
out=demo/data/ytklearn
mkdir -p "${out}" demo/data/libsvm
conv() {  # mode name
  for part in train test; do
    if [ ! -s "${out}/$2.${part}.ytklearn" ]; then
      bash bin/libsvm_convert_2_ytklearn.sh "$1" "${src}/$2.${part}.libsvm" "${out}/$2.${part}.ytklearn"
    fi
  done
  # every feature name of the training file; each name is its own FFM field (no field delim)
  if [ ! -s "${out}/$2.feat_dict" ]; then
    python - "${out}/$2.train.ytklearn" "${out}/$2.feat_dict" "${out}/$2.field.dict" <<'PY'
import sys
names = set()
for line in open(sys.argv[1]):
    cols = line.rstrip("\n").split("###")
    if len(cols) >= 3 and cols[2]:
        names.update(kv.rsplit(":", 1)[0] for kv in cols[2].split(","))
order = sorted(names, key=lambda s: (len(s), s))
for path in sys.argv[2:]:
    open(path, "w").write("\n".join(order) + "\n")
PY
  fi
}
conv "binary_classification@0,1" agaricus
conv "multi_classification@0,1,2,3,4,5" dermatology
conv regression machine
# the exact-greedy GBDT demo reads the raw LibSVM lines through its transform hook
for part in train test; do
  [ -s "demo/data/libsvm/machine.${part}.libsvm" ] || cp "${src}/machine.${part}.libsvm" demo/data/libsvm/
done
echo "demo data ready in ${out}"
