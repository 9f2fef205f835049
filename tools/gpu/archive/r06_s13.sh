#!/bin/bash
# r06 session 13: the queue with a lock-free inbox and the watcher's early
# launch (coalesce_lead_us): queue tests, a soak of the queue ops, and
# perblock_dev over lead 0 (completion launches only) / 30 (default) / 60.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s13
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_submit.py tests/test_gpu_pool.py \
  tests/test_gpu_hol.py tests/test_gpu_soak.py > $O/pytest_queue.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/soak.py --seconds 40 --threads 16 --ops 5,8,9 > $O/soak_queue.jsonl 2>&1 || exit $?
for tune in coalesce_lead_us=30 coalesce_lead_us=0 coalesce_lead_us=60; do
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 5 >> $O/perblock256.jsonl 2>> $O/perblock256.err || exit 1
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done
echo done-s13
