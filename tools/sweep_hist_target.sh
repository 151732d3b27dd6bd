# Sweep of YTK_HIST_TARGET (histogram blocks per level launch) on the full and 1/8-shard
# Higgs-shape benches. Round-1 result (ms/tree, full / eighth): 192 1.81/0.559, 256 1.87/0.545,
# 320 1.98/0.574, 384 1.89/0.562, 512 1.89/0.560 -- within run-to-run noise; 256 kept.
set -o pipefail
mkdir -p gpurun_out/sweep
for t in 192 256 320 384 512; do
  YTK_HIST_TARGET=$t timeout -k 10 120 python bench.py --steps 40 --warmup 3 > gpurun_out/sweep/full_$t.log 2>&1 || exit 1
  YTK_HIST_TARGET=$t timeout -k 10 120 python bench.py --steps 40 --warmup 3 --train-rows 1312500 --test-rows 62500 > gpurun_out/sweep/e_$t.log 2>&1 || exit 1
  echo "$t full $(tail -1 gpurun_out/sweep/full_$t.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') eighth $(tail -1 gpurun_out/sweep/e_$t.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
