# FFM kernels: GPU tests, then the FFM sparse bench + kernel profile
set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_sparse_kernels.py -m gpu -x -q > gpurun_out/ffm_tests.log 2>&1 || { tail -30 gpurun_out/ffm_tests.log; exit 1; }
tail -2 gpurun_out/ffm_tests.log
timeout -k 10 400 python bench_sparse.py --model ffm --rows 4000000 --steps 5 --warmup 1 2>gpurun_out/bs_ffm.err | tail -1 || { tail -20 gpurun_out/bs_ffm.err; exit 1; }
rm -rf gpurun_out/prof_ffm
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ffm -o run -- python $GRAFT_REPO_ROOT/bench_sparse.py --model ffm --rows 4000000 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_ffm.log 2>&1
echo prof ok
