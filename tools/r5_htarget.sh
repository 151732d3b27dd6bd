#!/bin/bash
# Histogram blocks per level (YTK_HIST_TARGET) A/B at the 1/8 shard (plain + forced-dist) and
# full size: the staged flush + slot reduce scale with the block count, the row work with
# the shard.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ht}
mkdir -p $O
export TMPDIR=/tmp
cd $R
E8="--train-rows 1312500 --test-rows 62500"
for t in 256 128 64 32; do
  YTK_HIST_TARGET=$t timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 --leafwise-steps 0 > $O/eighth_t$t.json 2> $O/eighth_t$t.err || { tail -30 $O/eighth_t$t.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/eighth_t$t.json').read().strip().splitlines()[-1]); print('eighth', $t, d['ms_per_step'], d.get('train_loss'))"
done
for t in 128 64; do
  YTK_FORCE_DIST=1 MASTER_PORT=$((29630 + t)) YTK_HIST_TARGET=$t timeout -k 10 300 python bench.py --steps 50 --warmup 5 $E8 --leafwise-steps 0 > $O/eighth_forced_t$t.json 2> $O/eighth_forced_t$t.err || { tail -30 $O/eighth_forced_t$t.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/eighth_forced_t$t.json').read().strip().splitlines()[-1]); print('forced', $t, d['ms_per_step'])"
done
for t in 256 128; do
  YTK_HIST_TARGET=$t timeout -k 10 300 python bench.py --steps 20 --warmup 3 --leafwise-steps 0 > $O/full_t$t.json 2> $O/full_t$t.err || { tail -30 $O/full_t$t.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/full_t$t.json').read().strip().splitlines()[-1]); print('full', $t, d['ms_per_step'])"
done
echo "ht ok"
