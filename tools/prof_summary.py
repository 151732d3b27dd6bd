#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals and the last K-round timeline."""
import csv, sys, collections
path = sys.argv[1]
import re
marker = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"tree_grad_(hist_)?kernel")
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x['Start_Timestamp']))
ev = [(x['Kernel_Name'], int(x['Start_Timestamp']), int(x['End_Timestamp']), x) for x in r]
idx = [i for i, e in enumerate(ev) if marker.search(e[0])]
if len(idx) >= 3:
    s, e = idx[-3] + 1, idx[-2]
    t0, t1 = ev[s][1], ev[e][2]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, a, b, x in ev[s:e + 1]:
        k = n.split('(')[0][:70]
        agg[k][0] += 1
        agg[k][1] += (b - a) / 1000
    busy = sum(v[1] for v in agg.values())
    print(f"one round: wall {(t1 - t0) / 1000:.1f} us, kernel-busy {busy:.1f} us")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t:9.1f} us  {c:3d}x  {k}")
