"""The native host runtime (csrc/native: multi-threaded parser, hashing, java random,
quantile summaries) under ASan+UBSan and TSan (tools/sanitize_native.sh)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("setarch") is None, reason="no g++/setarch")
def test_native_code_sanitizer_clean(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_native.sh")], cwd=ROOT,
                       env=dict(os.environ, OUT=str(tmp_path)), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "sanitizers clean" in r.stdout
