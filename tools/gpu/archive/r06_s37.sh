#!/bin/bash
# r06 session 37: where the 256-block T=16 per-block case loses its time --
# the queue's event log lined up with each rep's release of the threads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s37
mkdir -p $O
SHMR_PB_GO=1 SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T16.jsonl 2> $O/pb256_T16.trace || exit 1
SHMR_PB_GO=1 SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=1 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T1.jsonl 2> $O/pb256_T1.trace || exit 1
echo done-s37
