# rocprofv3 kernel stats of one sparse-model bench: bash tools/prof_sparse.sh <linear|fm|ffm>
set -eo pipefail
m=${1:-fm}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$m
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$m -o run -- python $R/bench_sparse.py --model $m --rows 4000000 --steps 3 --warmup 1 > $R/gpurun_out/prof_$m.log 2>&1
python $R/tools/kstats.py $R/gpurun_out/prof_$m/run_kernel_stats.csv
