set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-hd}; mkdir -p $O; cd $GRAFT_REPO_ROOT
shift
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --leafwise-steps 0 "$@" > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  echo "run$i $(tail -1 $O/b$i.json | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
