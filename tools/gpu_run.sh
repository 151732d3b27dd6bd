#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_*.sh scripts).
#
#   tools/gpu_run.sh <name> "<seconds>|<log>|<command>" ["<seconds>|<log>|<command>" ...]
#
# Each step runs from the repo root under its own `timeout -k 10 <seconds>`, writes
# stdout+stderr to gpurun_out/<name>/<log> and prints that log's last line. The chain
# stops at the first failing step (GPU fault, abort, time limit): nothing more runs on
# the GPU in that call. A command starting with "prof:" runs under
#   rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/<name>/<log>.d -o run --
# from /tmp (the program itself after `--`), and its one-round breakdown is written to
# gpurun_out/<name>/<log>.round.txt. A command starting with "env:K=V,K2=V2;" sets
# environment variables for that step only.
#
# Example:
#   gpurun --timeout 900 -- tools/gpu_run.sh lvl \
#     "500|pytest.log|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
#     "300|bench.log|python bench.py --steps 500 --warmup 5" \
#     "300|prof.log|prof:python bench.py --steps 10 --warmup 2 --leafwise-steps 0"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1
shift
O=$R/gpurun_out/$NAME
rm -rf "$O" && mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
for spec in "$@"; do
  t=${spec%%|*}
  rest=${spec#*|}
  log=${rest%%|*}
  cmd=${rest#*|}
  envs=()
  if [[ $cmd == env:* ]]; then
    e=${cmd#env:}
    e=${e%%;*}
    cmd=${cmd#*;}
    IFS=',' read -r -a envs <<< "$e"
  fi
  if [[ $cmd == pmc:* ]]; then
    # "pmc:CTR1 CTR2 ...;python bench.py ..." -- one counter pass (its own run, no tracing
    # domains; the per-block counter limits of rocprofv3 apply), summarised by pmc_summary.py
    ctrs=${cmd#pmc:}
    ctrs=${ctrs%%;*}
    cmd=${cmd#*;}
    read -r -a argv <<< "$cmd"
    for i in "${!argv[@]}"; do
      [[ ${argv[$i]} == *.py && -f $R/${argv[$i]} ]] && argv[$i]=$R/${argv[$i]}
    done
    read -r -a cv <<< "$ctrs"
    (cd /tmp && env "${envs[@]}" timeout -s KILL "$t" rocprofv3 --pmc "${cv[@]}" --output-format csv \
        -d "$O/$log.d" -o run -- "${argv[@]}") > "$O/$log" 2>&1
    rc=$?
    if [ $rc -eq 0 ]; then
      csv=$(ls "$O/$log.d"/*counter_collection.csv 2>/dev/null | head -1)
      [ -n "$csv" ] && python tools/pmc_summary.py "$csv" > "$O/$log.summary.txt" 2>&1
    fi
  elif [[ $cmd == prof:* ]]; then
    cmd=${cmd#prof:}
    # rocprofv3 must exec the program itself: resolve relative script paths against the repo
    read -r -a argv <<< "$cmd"
    for i in "${!argv[@]}"; do
      [[ ${argv[$i]} == *.py && -f $R/${argv[$i]} ]] && argv[$i]=$R/${argv[$i]}
    done
    (cd /tmp && env "${envs[@]}" timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/$log.d" -o run -- "${argv[@]}") > "$O/$log" 2>&1
    rc=$?
    if [ $rc -eq 0 ]; then
      csv=$(ls "$O/$log.d"/*kernel_trace.csv 2>/dev/null | head -1)
      [ -n "$csv" ] && python tools/prof_summary.py "$csv" > "$O/$log.round.txt" 2>&1
      st=$(ls "$O/$log.d"/*kernel_stats.csv 2>/dev/null | head -1)
      [ -n "$st" ] && cp "$st" "$O/$log.kernel_stats.csv"
    fi
  else
    env "${envs[@]}" timeout -k 10 "$t" bash -c "$cmd" > "$O/$log" 2>&1
    rc=$?
  fi
  if [ $rc -ne 0 ]; then
    echo "FAILED ($rc): $log"
    tail -40 "$O/$log"
    exit 1
  fi
  echo "[$log] $(tail -1 "$O/$log" | cut -c1-400)"
done
echo "$NAME ok"
