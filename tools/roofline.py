#!/usr/bin/env python3
"""Roofline table from rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / LDS counters).

usage: tools/roofline.py PMC1_CSV PMC2_CSV > table.md
FETCH_SIZE is doubled for the bandwidth estimate (MI355X_MICROARCH.md: on gfx950 it reports
half the bytes of a wide coalesced streaming read); WRITE_SIZE is taken as is."""
import collections
import csv
import sys

PEAK_TBS = 8.0
rows = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for path in sys.argv[1:]:
    seen = set()
    for x in csv.DictReader(open(path)):
        k = x["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        if not k.startswith("ytk::"):
            continue
        rows[k][x["Counter_Name"]].append(float(x["Counter_Value"]))
        key = (path, x["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000.0)


def mean(v):
    return sum(v) / len(v) if v else float("nan")


print("| kernel | us/launch | read MB (2 x FETCH_SIZE) | write MB | achieved TB/s | % of 8 TB/s | LDS busy cyc/CU | LDS bank-conflict % | VALU instr / launch |")
print("|---|---|---|---|---|---|---|---|---|")
for k, c in sorted(rows.items(), key=lambda kv: -sum(dur[kv[0]])):
    us = mean(dur[k])
    rd = 2 * mean(c.get("FETCH_SIZE", [])) / 1024.0
    wr = mean(c.get("WRITE_SIZE", [])) / 1024.0
    tbs = (rd + wr) / 1e6 / (us * 1e-6) if us > 0 else float("nan")
    lds = mean(c.get("SQ_LDS_IDX_ACTIVE", []))
    bc = mean(c.get("SQ_LDS_BANK_CONFLICT", []))
    valu = mean(c.get("SQ_INSTS_VALU", []))
    print(f"| {k} | {us:.1f} | {rd:.1f} | {wr:.1f} | {tbs:.2f} | {100 * tbs / PEAK_TBS:.0f}% | "
          f"{lds / 256:.0f} | {100 * bc / lds if lds else 0:.0f}% | {valu:.3g} |")
