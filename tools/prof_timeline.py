#!/usr/bin/env python3
"""One round of a rocprofv3 kernel trace as a timeline: kernel, start offset, duration, gap
before it. Usage: prof_timeline.py run_kernel_trace.csv [marker-regex] [round-index-from-end]"""
import csv
import re
import sys

path = sys.argv[1]
marker = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"tree_grad_(hist_)?kernel")
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if marker.search(x["Kernel_Name"])]
s, e = idx[-back - 1] + 1, idx[-back]
t0 = int(r[s]["Start_Timestamp"])
prev = t0
for x in r[s:e + 1]:
    a, b = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    name = re.sub(r"^void ", "", x["Kernel_Name"]).split("(")[0][:60]
    print(f"{(a - t0) / 1000:8.1f} {(b - a) / 1000:7.1f} gap {(a - prev) / 1000:6.1f}  {name}")
    prev = b
