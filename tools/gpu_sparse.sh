# sparse-model benchmarks + profiles on one GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in linear fm ffm; do
  timeout -k 10 400 python bench_sparse.py --model $m --rows 4000000 --steps 5 --warmup 1 2>gpurun_out/bs_$m.err | tail -1 || { tail -20 gpurun_out/bs_$m.err; exit 1; }
done
rm -rf gpurun_out/prof_fm gpurun_out/prof_ffm
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fm -o run -- python bench_sparse.py --model fm --rows 4000000 --steps 3 --warmup 1 > gpurun_out/prof_fm.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ffm -o run -- python bench_sparse.py --model ffm --rows 4000000 --steps 3 --warmup 1 > gpurun_out/prof_ffm.log 2>&1 || exit 1
echo prof ok
