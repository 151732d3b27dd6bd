"""Weighted per-slot sums for the AUC / confusion-matrix evaluators: torch.bincount (fp64
atomics, clustered predictions contend on few slots) vs sort + segment_reduce
(metrics/evaluators.py:slot_sums). Prints ms per call and the max abs difference."""
import time

import torch

from ytk_learn_amd.metrics.evaluators import slot_sums


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for n, S in ((500_000, 100_000), (10_500_000, 100_000), (10_500_000, 2)):
        p = torch.sigmoid(torch.randn(n, device="cuda", generator=g) * 0.6)
        y = (torch.rand(n, device="cuda", generator=g) < p).float()
        w = torch.rand(n, device="cuda", generator=g).double() + 0.5
        idx = (p * S).long().clamp(0, S - 1)
        slot = idx * 2 + (y != 1.0).long()
        tb, hb = bench(lambda: torch.stack([torch.bincount(slot, weights=w, minlength=2 * S),
                                            torch.bincount(slot, minlength=2 * S).double()]))
        ts, hs = bench(lambda: slot_sums(slot, w, 2 * S))
        print(f"n={n} slots={2 * S}: bincount {tb:.3f} ms, sort+segment {ts:.3f} ms, "
              f"max|diff| {float((hb - hs).abs().max()):.3e}", flush=True)


if __name__ == "__main__":
    main()
