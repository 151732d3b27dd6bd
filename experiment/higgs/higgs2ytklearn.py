#!/usr/bin/env python3
"""HIGGS.csv (UCI: label, 28 features per line) -> ytk-learn lines ``1###label###0:v,1:v,...``.
The first 10.5M rows become higgs.train, the rest (0.5M) higgs.test -- the split the
reference's experiment uses (docs/gbdt_experiments.md:9). Streams; O(1) memory.
usage: higgs2ytklearn.py [HIGGS.csv] [train_out] [test_out] [num_train]"""
import sys


def convert(src="HIGGS.csv", train_out="higgs.train", test_out="higgs.test", num_train=10_500_000):
    n = 0
    with open(src) as fin, open(train_out, "w") as ftr, open(test_out, "w") as fte:
        for line in fin:
            tok = line.strip().split(",")
            if len(tok) < 2:
                continue
            feats = ",".join(f"{i}:{float(v)!r}" for i, v in enumerate(tok[1:]))
            (ftr if n < num_train else fte).write(f"1###{int(float(tok[0]))}###{feats}\n")
            n += 1
    return n


if __name__ == "__main__":
    args = sys.argv[1:4] + ([int(sys.argv[4])] if len(sys.argv) > 4 else [])
    print(f"converted {convert(*args)} rows")
