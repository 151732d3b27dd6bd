set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
timeout -k 10 200 python tools/dbg_spec.py 1000000 2 0,1 2>&1 | grep -E "booster|identical"
timeout -k 10 200 python tools/dbg_cmp.py 1000000 level 1 2>&1 | grep identical
timeout -k 10 200 python tools/dbg_cmp.py 300000 loss 1 2>&1 | grep identical
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --policy loss 2>&1 | tail -1 | cut -c1-200
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --policy loss --profile 2>&1 | grep TimeStats
