"""Offline batch prediction CLI.

Reference: ``J/predictor/Predicts.java:36-54`` and ``bin/predict.sh`` (positional
``conf model fileOrDir needPy pyScript saveMode suffix maxErrTol metrics [value|leafid]``).

  python -m ytk_learn_amd.cli.predict CONF MODEL FILE_OR_DIR NEED_PY PY_SCRIPT SAVE_MODE SUFFIX
         MAX_ERROR_TOL METRICS [value|leafid] [--device cuda|cpu]
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="ytk_learn_amd.cli.predict")
    ap.add_argument("conf")
    ap.add_argument("model")
    ap.add_argument("path")
    ap.add_argument("need_py", nargs="?", default="false")
    ap.add_argument("py_script", nargs="?", default="")
    ap.add_argument("save_mode", nargs="?", default="PREDICT_RESULT_ONLY")
    ap.add_argument("suffix", nargs="?", default=None)
    ap.add_argument("max_error_tol", nargs="?", type=int, default=100)
    ap.add_argument("metrics", nargs="?", default="")
    ap.add_argument("predict_type", nargs="?", default="value")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    a = ap.parse_args(sys.argv[1:] if argv is None else argv)
    from ..config.hocon import parse_file, parse_override_value
    from ..predict.predictor import create_predictor
    cfg = parse_file(a.conf)
    for kv in a.set:
        k, v = kv.split("=", 1)
        cfg = cfg.with_value(k.strip(), parse_override_value(v))
    p = create_predictor(a.model, cfg, a.device)
    script = a.py_script if a.need_py.lower() == "true" and a.py_script else None
    p.batch_predict_from_files(a.path, script, a.save_mode, a.suffix, a.max_error_tol, a.metrics, a.predict_type)
    return 0


if __name__ == "__main__":
    sys.exit(main())
