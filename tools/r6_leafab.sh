# leaf-wise 500-tree A/B of the first-batch partition scan + forced-dist eighth: tools/r6_leafab.sh <tag>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lab}; mkdir -p $O; cd $GRAFT_REPO_ROOT
for v in 2 0 2 0; do
  YTK_LW_PART_SCAN=$v timeout -k 10 300 python bench.py --policy loss --steps 500 --warmup 5 > $O/leaf_s$v.json 2> $O/leaf_s$v.err || { tail -20 $O/leaf_s$v.err; exit 1; }
  echo "lw_scan=$v $(tail -1 $O/leaf_s$v.json | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
YTK_FORCE_DIST=1 MASTER_PORT=29641 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --train-rows 1312500 --test-rows 62500 > $O/e8f.json 2> $O/e8f.err || { tail -20 $O/e8f.err; exit 1; }
echo "eighth_forced $(tail -1 $O/e8f.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["graph_replays"], d["warmup_autotune_extra"])')"
