set -o pipefail
mkdir -p gpurun_out/spec
for p in ${PCTS:-100 75 50 35}; do
  YTK_LW_SPEC_PCT=$p timeout -k 10 200 python bench.py --steps 20 --warmup 3 --policy loss --leafwise-steps 0 > gpurun_out/spec/b$p.log 2>&1 || exit 1
  echo "pct $p: $(tail -1 gpurun_out/spec/b$p.log | cut -c100-200)"
done
