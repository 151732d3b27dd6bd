set -e
mkdir -p gpurun_out/zr
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gbdt_graph.py tests/test_gbdt_kernels.py tests/test_gbdt_train.py tests/test_gbdt_materialize.py tests/test_gbdt_objectives_gpu.py > gpurun_out/zr/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --leafwise-steps 0 --quiet > gpurun_out/zr/new_full_$i.json 2>&1
  YTK_ZERO_AT_END=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --leafwise-steps 0 --quiet > gpurun_out/zr/old_full_$i.json 2>&1
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --train-rows 1312500 --test-rows 62500 --leafwise-steps 0 --quiet > gpurun_out/zr/new_e_$i.json 2>&1
  YTK_ZERO_AT_END=1 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --train-rows 1312500 --test-rows 62500 --leafwise-steps 0 --quiet > gpurun_out/zr/old_e_$i.json 2>&1
done
