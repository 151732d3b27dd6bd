set -o pipefail
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --policy loss --profile 2>&1 | grep -E "TimeStats|trees=|metric" | cut -c1-300
