#!/bin/bash
# r06 session 25: where a merged launch's host time goes (phase log), T=16 / 256 and T=32 / 1024.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s25
mkdir -p $O
SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T16.jsonl 2> $O/pb256_T16.trace || exit 1
SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=32 timeout -k 10 120 tools/_abx/perblock_dev 1024 3 > $O/pb1024_T32.jsonl 2> $O/pb1024_T32.trace || exit 1
echo done-s25
