set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-st1}; mkdir -p $O; export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --leafwise-steps 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('level', d['ms_per_step'], 'leaf', d.get('leafwise_s_per_tree'))"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --leafwise-steps 0 --train-rows 1312500 --test-rows 62500 > $O/e8.json 2> $O/e8.err || { tail -20 $O/e8.err; exit 1; }
tail -1 $O/e8.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eighth', d['ms_per_step'])"
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pf -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --leafwise-steps 0) > $O/pf.log 2>&1 || { tail -20 $O/pf.log; exit 1; }
python tools/prof_timeline.py $O/pf/run_kernel_trace.csv > $O/timeline.txt 2>/dev/null || true
python tools/prof_summary.py $O/pf/run_kernel_trace.csv > $O/round.txt; rm -rf $O/pf
head -6 $O/round.txt
grep partition_children $O/timeline.txt | tail -5 | cut -c1-60
