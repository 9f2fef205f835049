#!/bin/bash
# r06 session 23: sleepers and the launcher on separate locks; the watcher launches before it wakes sleepers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s23
mkdir -p $O
SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=32 timeout -k 10 120 tools/_abx/perblock_dev 1024 3 > $O/pb1024_T32.jsonl 2> $O/pb1024_T32.trace || exit 1
SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T16.jsonl 2> $O/pb256_T16.trace || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 > $O/perblock256.jsonl 2> $O/perblock256.err || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_submit.py tests/test_gpu_soak.py > $O/pytest_queue.log 2>&1 || exit $?
echo done-s23
