#!/bin/bash
# r06 session 40: the queue's completion sleepers on a futex (no mutex): queue,
# pool and soak tests; the HOL test alone and after the queue / pool tests
# (order dependence); a soak of the queue ops, per-block rates, the traced
# 256-block T = 16 run with each rep's release.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s40
mkdir -p $O
# a test failure (exit 1) is recorded and the session goes on; anything else ends it
t() { local n=$1; shift; timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > $O/pytest_$n.log 2>&1; local rc=$?; echo "$n rc=$rc" >> $O/rcs.txt; [ $rc -le 1 ]; }
t queue tests/test_gpu_submit.py tests/test_gpu_pool.py tests/test_gpu_soak.py || exit 1
t hol_alone tests/test_gpu_hol.py || exit 1
t hol_after_submit tests/test_gpu_submit.py tests/test_gpu_hol.py || exit 1
t hol_after_pool tests/test_gpu_pool.py tests/test_gpu_hol.py || exit 1
timeout -k 10 120 python -u tools/soak.py --seconds 40 --threads 16 --ops 5,8,9 > $O/soak_queue.jsonl 2>&1 || exit $?
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 > $O/perblock256.jsonl 2> $O/perblock256.err || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err || exit 1
SHMR_PB_GO=1 SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T16.jsonl 2> $O/pb256_T16.trace || exit 1
echo done-s40
