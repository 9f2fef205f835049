#!/bin/bash
# r06 session 26: the inbox as a ring of request pointers (no linked-list walk); tests, soaks, perblock_dev, traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s26
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_submit.py tests/test_gpu_pool.py \
  tests/test_gpu_hol.py tests/test_gpu_soak.py > $O/pytest_queue.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/soak.py --seconds 40 --threads 16 --ops 5,8,9 > $O/soak_queue.jsonl 2>&1 || exit $?
SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=32 timeout -k 10 120 tools/_abx/perblock_dev 1024 3 > $O/pb1024_T32.jsonl 2> $O/pb1024_T32.trace || exit 1
SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T16.jsonl 2> $O/pb256_T16.trace || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 > $O/perblock256.jsonl 2> $O/perblock256.err || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err || exit 1
timeout -k 10 300 tools/_abx/perblock_host 128 5 > $O/perblock_host.jsonl 2> $O/perblock_host.err || exit 1
echo done-s26
