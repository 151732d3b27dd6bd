"""LibSVM -> ytk-learn data format converter.

Reference: ``J/utils/LibsvmConvertTool.java:43-187`` and ``bin/libsvm_convert_2_ytklearn.sh``.
Usage (positional, as the reference):
  python -m ytk_learn_amd.tools.libsvm_convert MODE X_DELIM Y_DELIM FEATURES_DELIM KV_DELIM FS IN OUT
MODE: ``binary_classification@neg,pos`` | ``multi_classification@l0,l1,...`` | ``regression``.
Every output line gets weight 1; classification labels are mapped to their index in the
MODE list (multi-class lines carry the class index); a line without a label keeps an empty
label field (predict data).
"""
from __future__ import annotations

import sys
from typing import Dict, List

from ..io.fs import create_fs
from ..utils.errors import YtkLearnError
from ..utils.javafmt import java_float_str


def convert_line(line: str, mode: str, label_map: Dict[str, int], xd: str, fd: str, kvd: str, counts: List[int]) -> str:
    info = line.strip().split()
    if not info:
        return ""
    has_label = len(info[0].split(":")) == 1
    out = ["1", xd]
    if has_label:
        if mode.startswith("binary_classification") or mode.startswith("multi_classification"):
            if info[0] not in label_map:
                raise YtkLearnError(f"unknown label:{info[0]}")
            lab = label_map[info[0]]
            out.append(str(lab))
            counts[lab] += 1
        elif mode.startswith("regression"):
            out.append(java_float_str(float(info[0])))
        else:
            raise YtkLearnError(f"unsupport mode:{mode}")
        out.append(xd)
        feats = info[1:]
    else:
        out.append(xd)
        feats = info[1:]
    out.append(fd.join(kv.split(":")[0] + kvd + kv.split(":")[1] for kv in feats))
    return "".join(out)


def convert(mode: str, xd: str, yd: str, fd: str, kvd: str, fs_scheme: str, inp: str, outp: str, log=print) -> int:
    label_map: Dict[str, int] = {}
    k = 2
    if "classification" in mode:
        labels = mode.split("@")[1].strip().split(",")
        k = len(labels)
        label_map = {l: i for i, l in enumerate(labels)}
    counts = [0] * k
    fs = create_fs(fs_scheme)
    n = 0
    log(f"libsvm format data path:{inp}")
    with fs.open_read(inp) as fi, fs.open_write(outp) as fo:
        for line in fi:
            s = convert_line(line, mode, label_map, xd, fd, kvd, counts)
            if s == "":
                continue
            fo.write(s + "\n")
            n += 1
    log(f"convert finished! convert count:{n}")
    for lab, i in label_map.items():
        log(f"libsvm classification label:{lab} ----> ytklearn classification label:{i}, count:{counts[i]}")
    log(f"ytk-learn format data path:{outp}")
    return n


def main(argv=None):
    a = list(sys.argv[1:] if argv is None else argv)
    if len(a) != 8:
        sys.stderr.write("usage: libsvm_convert MODE X_DELIM Y_DELIM FEATURES_DELIM KV_DELIM FS IN OUT\n")
        return 2
    convert(*a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
