#!/usr/bin/env python3
"""Higgs-shaped synthetic data in ytk-learn format (28 dense float features, binary label)
for machines without network access: same generator as bench.py
(ytk_learn_amd.data.synthetic.higgs_like). usage: make_synthetic.py [train_rows] [test_rows]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import numpy as np  # noqa: E402


def write(path, X, y, chunk=200_000):
    with open(path, "w") as f:
        for s in range(0, len(y), chunk):
            xs, ys = X[s:s + chunk], y[s:s + chunk]
            f.write("".join("1###%d###%s\n" % (int(ys[i]), ",".join(f"{j}:{xs[i, j]:.6g}" for j in range(xs.shape[1])))
                            for i in range(len(ys))))


if __name__ == "__main__":
    from ytk_learn_amd.data.synthetic import higgs_like
    ntr = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    nte = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    X, y = higgs_like(ntr + nte, seed=7)
    X, y = np.asarray(X), np.asarray(y).reshape(-1)
    write(os.path.join(HERE, "higgs.train"), X[:ntr], y[:ntr])
    write(os.path.join(HERE, "higgs.test"), X[ntr:], y[ntr:])
    print(f"wrote {ntr} train / {nte} test rows")
