#!/bin/bash
# r06 session 8: where async T=16 per-block calls lose time (kernel trace).
set -o pipefail
O=gpurun_out/r06s8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for T in 1 16; do
  SHMR_PB_TUNE=coalesce_depth=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=$T SHMR_PB_FLOOR_SKIP=1 \
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_t$T -o run -- tools/_abx/perblock_dev 1024 3 > $O/perblock_t$T.jsonl 2> $O/perblock_t$T.err || exit 1
done
echo "exit=$?"
