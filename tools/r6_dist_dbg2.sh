set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/dd2; mkdir -p $O/w2; cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=2 YTK_DIST_BACKEND=gloo YTK_HIST_SYNC=allreduce YTK_TEST_FSAMPLE=1.0 \
  YTK_PEER_REDUCE=1 YTK_COMM_LOG=1 YTK_HIST_OVERLAP_MIN_ROWS=0 YTK_PEER_OVERLAP=0 YTK_PART_SCAN_MIN_ROWS=0 YTK_PEER_TIMEOUT_S=40
timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 \
  tests/dist_worker.py gbdt_loss $O/w2 cuda > $O/out.log 2> $O/err.log
echo "rc=$?"
tail -40 $O/err.log | grep -v "amdgpu.ids\|hostname of the client"
