#!/bin/bash
# Reference-style distribution (tool/package.sh + src/main/assembly/package.xml of ytk-learn):
# build the native extensions for gfx950, then zip bin/ config/ demo/ experiment/ docs/ and
# the package (with its .so files) into dist/ytk-learn-amd-<version>.zip.
set -euo pipefail
cd "$(dirname "$0")/.."
python csrc/build.py
VER=$(python -c "import tomllib,sys;print(tomllib.load(open('pyproject.toml','rb'))['project']['version'])" 2>/dev/null || echo 0.2.0)
OUT=dist/ytk-learn-amd-$VER
rm -rf "$OUT" && mkdir -p "$OUT"
cp -r bin config demo experiment docs README.md pyproject.toml "$OUT"/
python - "$OUT" <<'PY'
import shutil, sys
shutil.copytree("ytk_learn_amd", sys.argv[1] + "/ytk_learn_amd",
                ignore=shutil.ignore_patterns("__pycache__", "*.pyc"))
PY
(cd dist && rm -f "ytk-learn-amd-$VER.zip" && python -m zipfile -c "ytk-learn-amd-$VER.zip" "ytk-learn-amd-$VER")
echo "dist/ytk-learn-amd-$VER.zip"
