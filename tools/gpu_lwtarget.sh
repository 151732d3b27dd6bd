set -o pipefail
mkdir -p gpurun_out/lwt
for t in ${TGTS:-256 384 512 768}; do
  YTK_HIST_TARGET=$t timeout -k 10 200 python bench.py --steps 20 --warmup 3 --policy loss --leafwise-steps 0 > gpurun_out/lwt/b$t.log 2>&1 || exit 1
  echo "target $t: $(tail -1 gpurun_out/lwt/b$t.log | cut -c100-200)"
done
