#!/usr/bin/env bash
# The reference ran training inside hadoop containers (bin/hadoop_optimizer.sh). ytk-learn-amd
# runs one process per GPU with torch.distributed; launch the same job with
# bin/cluster_optimizer.sh on the GPU nodes (data can stay on HDFS/S3 via fs_scheme + fsspec).
echo "hadoop launcher is not supported: use bin/cluster_optimizer.sh (torch.distributed over RCCL)" >&2
exit 2
