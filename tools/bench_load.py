#!/usr/bin/env python3
"""Load + preprocess benchmark at Higgs scale.

The reference publishes 35.46 s to load and preprocess the 11M-line Higgs text file
(docs/gbdt_experiments.md:103; pipeline DataFlow.java:483-540 + CoreData.java:536-611:
parse, feature dictionary, dense matrix, missing-value fill, sample_by_quantile
binning). This tool times the same stages of this framework on a Higgs-FORMAT synthetic
file (ytk text format ``weight###label###f:v,...``, 28 dense features; no network for the
real data) with the experiment's own config (experiment/higgs/local_gbdt.conf):

  parse_train    native multi-threaded parser (csrc/native/parser.cpp) -> CSR shard
  dictionary     user feat_dict / hash-partitioned count merge
  dense_train    CSR -> dense [N, 28] on the device (scatter)
  parse_test / dense_test
  prepare        GBDTTrainer.prepare(): missing fill, BinMapper.fit (device sort /
                 unique / quantiles), bin_assign kernel, builder setup

The file is generated once (untimed) by worker processes writing parts that are
concatenated into one file, as the reference reads one file.

usage: python tools/bench_load.py [--rows 10500000] [--test-rows 500000] [--dir /tmp/higgs_load]
                                  [--device cuda|cpu] [--threads 0] [--gen-procs 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REFERENCE_S = 35.46  # docs/gbdt_experiments.md:103 (load + preprocess, Higgs 11M lines)


def _gen_part(args):
    path, start, n, seed = args
    import numpy as np
    from ytk_learn_amd.data.synthetic import higgs_like
    X, y = higgs_like(n, seed=seed)
    X, y = np.asarray(X, dtype=np.float32), np.asarray(y).reshape(-1)
    with open(path, "w") as f:
        step = 100_000
        for s in range(0, n, step):
            xs, ys = X[s:s + step], y[s:s + step]
            cols = [np.char.add(f"{j}:", np.char.mod("%.6g", xs[:, j])) for j in range(xs.shape[1])]
            feats = cols[0]
            for c in cols[1:]:
                feats = np.char.add(np.char.add(feats, ","), c)
            lines = np.char.add(np.char.add(np.char.mod("1###%d###", ys.astype(np.int64)), feats), "\n")
            f.write("".join(lines.tolist()))
    return path


def generate(path, rows, procs, seed):
    import multiprocessing as mp
    step = max(1, -(-rows // (procs * 4)))
    jobs = [(f"{path}.part{i:04d}", s, min(step, rows - s), seed * 7919 + i)
            for i, s in enumerate(range(0, rows, step))]
    with mp.get_context("spawn").Pool(procs) as pool:
        for i, _ in enumerate(pool.imap(_gen_part, jobs)):
            print(f"[bench_load] generated part {i + 1}/{len(jobs)}", file=sys.stderr, flush=True)
    parts = [j[0] for j in jobs]
    with open(path + ".tmp", "wb") as out:
        for p in parts:
            with open(p, "rb") as f:
                while True:
                    b = f.read(1 << 24)
                    if not b:
                        break
                    out.write(b)
            os.remove(p)
    os.replace(path + ".tmp", path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_500_000)
    ap.add_argument("--test-rows", type=int, default=500_000)
    ap.add_argument("--dir", default="/tmp/higgs_load")
    ap.add_argument("--device", default=None)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--gen-procs", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    a = ap.parse_args()

    os.makedirs(a.dir, exist_ok=True)
    tr_path = os.path.join(a.dir, f"higgs_{a.rows}.train")
    te_path = os.path.join(a.dir, f"higgs_{a.test_rows}.test")
    tg = time.perf_counter()
    if not os.path.exists(tr_path):
        generate(tr_path, a.rows, a.gen_procs, 1)
    if a.test_rows and not os.path.exists(te_path):
        generate(te_path, a.test_rows, a.gen_procs, 2)
    gen_s = time.perf_counter() - tg
    print(f"[bench_load] data ready in {gen_s:.1f}s ({os.path.getsize(tr_path) / 2**30:.2f} GiB train)",
          file=sys.stderr, flush=True)

    import torch
    from ytk_learn_amd.config.hocon import parse_file
    from ytk_learn_amd.data.dataflow import build_dictionary, read_dict_files
    from ytk_learn_amd.models.gbdt.operation import GBDTLoader
    from ytk_learn_amd.models.gbdt.trainer import GBDTTrainer
    from ytk_learn_amd.parallel.comm import Comm
    from ytk_learn_amd.utils.logging import get_logger

    comm = Comm.from_env(a.device)
    dev = comm.device
    cfg = parse_file(os.path.join(ROOT, "experiment/higgs/local_gbdt.conf"))
    cfg = cfg.with_value("data.train.data_path", tr_path).with_value("data.test.data_path", te_path if a.test_rows else "")
    cfg = cfg.with_value("model.dict_path", os.path.join(ROOT, "experiment/higgs/feat_dict"))
    log = get_logger(comm)
    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
    if dev.type == "cuda":  # context + allocator warm (not part of the reference's timing either)
        torch.zeros(1, device=dev)
        sync()

    st = {}
    comm.barrier()
    t_all = time.perf_counter()
    loader = GBDTLoader(cfg, comm, dev, log, None, None, a.threads)
    gp, dp, mp = loader.gp, loader.dp, loader.mp

    t = time.perf_counter()
    raw = loader._parse(dp.train_path, dp.train_max_error_tol, None)
    st["parse_train"] = time.perf_counter() - t
    t = time.perf_counter()
    user = read_dict_files(loader.fs, mp.dict_path) if mp.need_dict else None
    name2idx, names = build_dictionary(raw, comm, gp.filter_threshold, False, "", user)
    st["dictionary"] = time.perf_counter() - t
    t = time.perf_counter()
    softmax = gp.loss_function.startswith("softmax")
    train = loader._data(raw, name2idx, len(names), gp.class_num, softmax)
    sync()
    st["dense_train"] = time.perf_counter() - t
    n_train = raw.n_rows
    del raw
    test = None
    if a.test_rows:
        t = time.perf_counter()
        rt = loader._parse(dp.test_path, dp.test_max_error_tol, None)
        st["parse_test"] = time.perf_counter() - t
        t = time.perf_counter()
        test = loader._data(rt, name2idx, len(names), gp.class_num, softmax)
        sync()
        st["dense_test"] = time.perf_counter() - t
        del rt
    t = time.perf_counter()
    tr = GBDTTrainer(gp, train, test, comm, names, None, log=log)
    if not hasattr(tr, "mapper"):
        tr.prepare()
    sync()
    st["prepare"] = time.perf_counter() - t
    total = time.perf_counter() - t_all
    tot = comm.allreduce_scalars([total], op="max")[0]
    if comm.is_master:
        res = {"metric": "load_preprocess_seconds", "value": round(tot, 3), "unit": "s", "higher_is_better": False,
               "reference_s": REFERENCE_S, "speedup_vs_reference": round(REFERENCE_S / tot, 2),
               "n_gpus": comm.world, "device": dev.type, "train_rows": n_train, "features": len(names),
               "max_bins": int(tr.mapper.max_bins), "file_gib": round(os.path.getsize(tr_path) / 2**30, 3),
               "stages_s": {k: round(v, 3) for k, v in st.items()},
               "data": "synthetic Higgs-format text (experiment/higgs make_synthetic generator)"}
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    comm.close()


if __name__ == "__main__":
    main()
