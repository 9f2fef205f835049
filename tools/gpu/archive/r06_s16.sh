#!/bin/bash
# r06 session 16: a cold thread's first queue call hands its launch to the
# watcher (the thread warms outside the launcher flag): queue tests and soak,
# perblock_dev 256 / 1024, the 256-block T=16 async case traced again.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s16
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_submit.py tests/test_gpu_pool.py \
  tests/test_gpu_hol.py tests/test_gpu_soak.py > $O/pytest_queue.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/soak.py --seconds 40 --threads 16 --ops 5,8,9 > $O/soak_queue.jsonl 2>&1 || exit $?
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 > $O/perblock256.jsonl 2> $O/perblock256.err || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err || exit 1
SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d $O/kt -o pb16 -- tools/_abx/perblock_dev 256 5 > $O/perblock256_T16_traced.jsonl 2> $O/kt.err || exit 1
echo done-s16
