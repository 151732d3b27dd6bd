#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 *_kernel_stats.csv: name, calls, total ms, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for x in rows[:top]:
    print(f"{float(x['TotalDurationNs']) / 1e6:9.2f} ms {int(x['Calls']):6d} calls "
          f"{float(x['Percentage']):6.2f}%  {x['Name'][:110]}")
