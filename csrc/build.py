#!/usr/bin/env python3
"""In-tree build of the native extensions (no JIT cache, no hipify).

* ``ytk_learn_amd/ops/_ytk_hip*.so``   -- HIP/CDNA4 kernels (hipcc --offload-arch=gfx950)
* ``ytk_learn_amd/_native/_ytk_native*.so`` -- C++ host runtime (parser, hashing,
  quantile sketch, tree/predict helpers, comm-free CPU kernels)

Usage: ``python csrc/build.py [--force] [--jobs N]``. Rebuilds only stale objects.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("YTK_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _py_includes():
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[-1]}")
    return r


def _headers(d):
    return [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp"))]


HIP_MODULE = {
    "name": "_ytk_hip",
    "out_dir": os.path.join(ROOT, "ytk_learn_amd", "ops"),
    "src_dir": os.path.join(CSRC, "hip"),
}
NATIVE_MODULE = {
    "name": "_ytk_native",
    "out_dir": os.path.join(ROOT, "ytk_learn_amd", "_native"),
    "src_dir": os.path.join(CSRC, "native"),
}


def build_hip(force=False, jobs=8):
    d = HIP_MODULE["src_dir"]
    hdrs = _headers(d)
    srcs = sorted(f for f in os.listdir(d) if f.endswith(".hip"))
    inc = ["-I" + d] + ["-I" + p for p in _py_includes()]
    os.makedirs(BUILD, exist_ok=True)
    objs, jobs_list = [], []
    for s in srcs:
        src = os.path.join(d, s)
        obj = os.path.join(BUILD, s + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs_list.append([HIPCC, "-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17",
                              "-munsafe-fp-atomics", "-c", src, "-o", obj] + inc)
    bind_src = os.path.join(d, "bind.cpp")
    bind_obj = os.path.join(BUILD, "hip_bind.cpp.o")
    objs.append(bind_obj)
    if force or _stale(bind_obj, [bind_src]):
        jobs_list.append([CXX, "-O2", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-c",
                          bind_src, "-o", bind_obj] + inc)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, jobs_list))
    out = os.path.join(HIP_MODULE["out_dir"], HIP_MODULE["name"] + EXT_SUFFIX)
    if force or jobs_list or _stale(out, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs)
    return out


def build_native(force=False, jobs=8):
    d = NATIVE_MODULE["src_dir"]
    hdrs = _headers(d)
    srcs = sorted(f for f in os.listdir(d) if f.endswith(".cpp"))
    inc = ["-I" + d] + ["-I" + p for p in _py_includes()]
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(NATIVE_MODULE["out_dir"], exist_ok=True)
    objs, jobs_list = [], []
    for s in srcs:
        src = os.path.join(d, s)
        obj = os.path.join(BUILD, "native_" + s + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs_list.append([CXX, "-O3", "-fPIC", "-std=c++17", "-fvisibility=hidden",
                              "-fopenmp", "-c", src, "-o", obj] + inc)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, jobs_list))
    out = os.path.join(NATIVE_MODULE["out_dir"], NATIVE_MODULE["name"] + EXT_SUFFIX)
    if objs and (force or jobs_list or _stale(out, objs)):
        _run([CXX, "-shared", "-fPIC", "-fopenmp", "-o", out] + objs)
    return out


def build_all(force=False, jobs=8):
    return [build_hip(force, jobs), build_native(force, jobs)]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    for p in build_all(a.force, a.jobs):
        print("built", os.path.relpath(p, ROOT))
