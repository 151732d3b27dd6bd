#!/usr/bin/env python3
"""Per-kernel mean PMC counters from rocprofv3 --pmc counter_collection CSVs."""
import collections
import csv
import sys

for f in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for x in csv.DictReader(open(f)):
        k = x["Kernel_Name"].split("(")[0][:48]
        agg[k][x["Counter_Name"]] += float(x["Counter_Value"])
        disp[k].add(x["Dispatch_Id"])
        dur[k][x["Dispatch_Id"]] = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000.0
    rows = sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]].values()))
    for k, v in rows[:14]:
        n = len(disp[k])
        us = sum(dur[k].values()) / n
        print(f"{k:50s} n={n:4d} us={us:9.1f} " + " ".join(f"{c}={val / n:.4g}" for c, val in sorted(v.items())))
