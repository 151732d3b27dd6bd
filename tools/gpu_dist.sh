set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_distributed.py -m gpu -x -q > gpurun_out/dist_gpu.log 2>&1 || { tail -40 gpurun_out/dist_gpu.log; exit 1; }
tail -2 gpurun_out/dist_gpu.log
YTK_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --train-rows 2000000 --test-rows 100000 > gpurun_out/bench2.log 2>&1 || { tail -30 gpurun_out/bench2.log; exit 1; }
tail -1 gpurun_out/bench2.log
