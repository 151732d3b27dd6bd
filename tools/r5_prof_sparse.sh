#!/bin/bash
# rocprofv3 kernel stats of the SGD epochs (FM fp32 / FFM) and the soft-tree L-BFGS evaluations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-psp}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
if [ -n "$CFGS" ]; then LIST="fm:sgd ffm:sgd"; else LIST="fm:sgd ffm:sgd gbhsdt:lbfgs gbmlr:lbfgs"; fi
for cc in $LIST; do
  cfg="${cc/:/ }"
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 $R/bench_sparse.py --model $1 --optimizer $2 --rows 4000000 --steps 1 --warmup 1 > $O/p_$1_$2.log 2>&1 || { tail -20 $O/p_$1_$2.log; exit 1; }
  python3 - $O/p_$1_$2/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(sys.argv[1])
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d}x {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
done
echo "prof sparse ok"
