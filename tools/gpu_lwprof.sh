set -o pipefail
mkdir -p gpurun_out/lp
YTK_LW_PROF=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --policy loss --leafwise-steps 0 > gpurun_out/lp/b.log 2>&1 && grep "planner profile" gpurun_out/lp/b.log
