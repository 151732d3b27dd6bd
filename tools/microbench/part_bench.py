#!/usr/bin/env python3
"""Partition-kernel microbenchmark: the same 10.5M rows split into 1, 32, 512 or
one-split-per-chunk segments (cursor-atomic contention sweep), identity vs gathered
rows. Prints kernel ms per configuration (hipEvent, mean of 10 launches)."""
import sys

import torch

sys.path.insert(0, ".")
from ytk_learn_amd.ops._ext import hip, ptr, stream  # noqa: E402

N, F = 10_500_000, 28
CH = 2048
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
binsT = torch.randint(0, 255, (F, N), dtype=torch.uint8, device=dev, generator=g)
gh = torch.randn((N, 2), device=dev, generator=g)
rows_out = torch.empty(N, dtype=torch.int32, device=dev)
gh_out = torch.empty((N, 2), device=dev)
perm = torch.randperm(N, device=dev, generator=g).to(torch.int32)
# level-4-like order: rows grouped by a random node id of 16 (ascending inside a node)
node16 = torch.randint(0, 16, (N,), device=dev, generator=g)
lvl4 = torch.sort(node16 * N + torch.arange(N, device=dev)).indices.to(torch.int32)
h = hip()


def run(nsplit, gathered, count_only=False, reps=10):
    # gathered: 0 identity rows, 1 random permutation, 2 level-4-like (16 interleaved nodes)
    seg = N // nsplit
    begins = torch.arange(nsplit, dtype=torch.int32) * seg
    counts = torch.full((nsplit,), seg, dtype=torch.int32)
    counts[-1] = N - int(begins[-1])
    nblk = (counts + CH - 1) // CH
    first = torch.zeros(nsplit, dtype=torch.int32)
    first[1:] = torch.cumsum(nblk, 0)[:-1].to(torch.int32)
    nb = int(nblk.sum())
    st = torch.tensor([nsplit, nb], dtype=torch.int32, device=dev)
    feat = (torch.arange(nsplit, dtype=torch.int32) % F).to(dev)
    thr = torch.full((nsplit,), 127, dtype=torch.int32, device=dev)
    begins, counts, first = begins.to(dev), counts.to(dev), first.to(dev)
    cursor = torch.zeros(nsplit, dtype=torch.int64, device=dev)
    rows_in = (0, ptr(perm), ptr(lvl4))[gathered]
    s = stream(binsT)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for i in range(reps + 2):
        cursor.zero_()
        e0.record()
        h.partition_atomic(ptr(binsT), 1, N, rows_in, ptr(rows_out), ptr(gh), ptr(gh_out), ptr(first),
                           st.data_ptr(), st.data_ptr() + 4, nb, ptr(feat), ptr(thr), ptr(begins), ptr(counts),
                           ptr(cursor), 1 if count_only else 0, 0, s)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
    return sum(ts) / len(ts), nb


for gathered in (0, 2, 1):
    for nsplit in (1, 32, 512, N // CH):
        for co in (False, True):
            ms, nb = run(nsplit, gathered, co)
            print(f"gathered={gathered} nsplit={nsplit:5d} blocks={nb} count_only={int(co)}  {ms * 1000:8.1f} us",
                  flush=True)
