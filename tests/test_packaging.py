"""Installable package (the reference's Maven build + zip assembly)."""
import glob
import os
import subprocess
import sys
import zipfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not glob.glob(os.path.join(ROOT, "ytk_learn_amd", "ops", "_ytk_hip*.so")),
                    reason="native extensions not built")
def test_wheel_carries_extensions_and_entry_points(tmp_path):
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-deps", "--no-build-isolation", "-w",
                        str(tmp_path), ROOT], capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    whl = glob.glob(str(tmp_path / "ytk_learn_amd-*.whl"))
    assert len(whl) == 1
    names = zipfile.ZipFile(whl[0]).namelist()
    assert any(n.startswith("ytk_learn_amd/ops/_ytk_hip") and n.endswith(".so") for n in names)
    assert any(n.startswith("ytk_learn_amd/_native/_ytk_native") and n.endswith(".so") for n in names)
    ep = [n for n in names if n.endswith("entry_points.txt")]
    text = zipfile.ZipFile(whl[0]).read(ep[0]).decode()
    assert "ytk-train" in text and "ytk-predict" in text
