# YTK_PART_SCAN_LEVELS A/B (50-tree level-wise bench): tools/r6_scan_ab.sh <tag> [levels...]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sab}; mkdir -p $O; cd $GRAFT_REPO_ROOT
shift
for L in ${*:-2 3 4 5 2 5}; do
  YTK_PART_SCAN_LEVELS=$L timeout -k 10 200 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 > $O/l$L.json 2> $O/l$L.err || { tail -20 $O/l$L.err; exit 1; }
  echo "levels=$L $(tail -1 $O/l$L.json | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
