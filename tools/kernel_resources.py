"""Per-kernel resource table of the HIP extension (gfx950 code objects, no GPU needed).

Compiles each ``csrc/hip/*.hip`` to device assembly with the build's flags and reads the
code-object metadata of every kernel: VGPR / AGPR / SGPR counts, spills, LDS (group segment)
and per-thread scratch (private segment). Scratch in a hot kernel is a red flag: a
runtime index into a kernel-argument array, for instance, copies the whole argument block to
scratch in every thread (ex_part_kernel: 13.0 -> 5.7 ms per level once removed).

    python tools/kernel_resources.py [--only NAME_SUBSTR] [--scratch-only] [files...]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIP_DIR = os.path.join(ROOT, "csrc", "hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
KEYS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "group_segment_fixed_size", "private_segment_fixed_size")


def device_asm(src: str, out_dir: str) -> str:
    out = os.path.join(out_dir, os.path.basename(src) + ".s")
    cmd = [HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17", "-munsafe-fp-atomics", "--offload-device-only",
           "-S", src, "-o", out, "-I" + HIP_DIR]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)}\n{r.stderr[-2000:]}")
    return out


def parse_kernels(asm_path: str) -> list[dict]:
    """The amdhsa.kernels metadata entries of one assembly file (a YAML block)."""
    text = open(asm_path).read()
    i = text.find(".amdgpu_metadata")
    if i < 0:
        return []
    j = text.find(".end_amdgpu_metadata", i)
    meta = yaml.safe_load(text[text.find("\n", i) + 1:text.rfind("\n", i, j) + 1])
    out = []
    for k in meta.get("amdhsa.kernels", []):
        out.append({"name": k[".name"], **{key: int(k.get("." + key, 0)) for key in KEYS}})
    return out


def kernel_table(files: list[str], jobs: int = 4) -> list[dict]:
    with tempfile.TemporaryDirectory() as td, ThreadPoolExecutor(max_workers=jobs) as ex:
        asms = list(ex.map(lambda f: device_asm(f, td), files))
        rows = []
        for f, a in zip(files, asms):
            for k in parse_kernels(a):
                k["file"] = os.path.basename(f)
                rows.append(k)
        return rows


def demangle(names: list[str]) -> list[str]:
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
        return r.stdout.splitlines() if r.returncode == 0 else names
    except OSError:
        return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*")
    ap.add_argument("--only", default="")
    ap.add_argument("--scratch-only", action="store_true")
    args = ap.parse_args()
    files = args.files or sorted(os.path.join(HIP_DIR, f) for f in os.listdir(HIP_DIR) if f.endswith(".hip"))
    rows = kernel_table(files)
    names = demangle([r["name"] for r in rows])
    print("| file | kernel | VGPR | AGPR | SGPR | spills (v/s) | LDS B | scratch B/thread |")
    print("|---|---|---|---|---|---|---|---|")
    for r, n in zip(rows, names):
        if args.only and args.only not in n:
            continue
        if args.scratch_only and not r.get("private_segment_fixed_size"):
            continue
        short = n if len(n) <= 90 else n[:87] + "..."
        print(f"| {r['file']} | `{short}` | {r.get('vgpr_count', '?')} | {r.get('agpr_count', 0)} | "
              f"{r.get('sgpr_count', '?')} | {r.get('vgpr_spill_count', 0)}/{r.get('sgpr_spill_count', 0)} | "
              f"{r.get('group_segment_fixed_size', '?')} | {r.get('private_segment_fixed_size', '?')} |")


if __name__ == "__main__":
    sys.exit(main())
