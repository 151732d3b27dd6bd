set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/bf2; mkdir -p $O; export TMPDIR=/tmp
for dt in fp32 bf16; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$dt -o run -- python $GRAFT_REPO_ROOT/bench_sparse.py --model ffm --optimizer sgd --dtype $dt --steps 2 --warmup 1) > $O/p_$dt.log 2>&1 || { tail -20 $O/p_$dt.log; exit 1; }
  cp $O/p_$dt/run_kernel_stats.csv $O/stats_$dt.csv; rm -rf $O/p_$dt
  python -c "
import csv,sys
r=list(csv.DictReader(open('$O/stats_$dt.csv')))
r.sort(key=lambda x:-float(x['TotalDurationNs']))
for x in r[:8]: print('$dt', x['Name'][:70], x['Calls'], round(float(x['TotalDurationNs'])/1e6,2),'ms', round(float(x['AverageNs'])/1e3,1),'us')
"
done
