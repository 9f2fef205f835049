#!/bin/bash
# r06 session 4: completion markers; the queue with a sleeping watcher.
set -o pipefail
O=gpurun_out/r06s4
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 tools/_abx/mark_probe > $O/mark_probe.jsonl 2> $O/mark_probe.err &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_submit.py tests/test_gpu_pool.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
for tune in coalesce_target=64 coalesce_target=256 coalesce_target=256,coalesce_watch_us=1000; do
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 3 >> $O/perblock256.jsonl 2>> $O/perblock256.err || exit 1
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done
echo "exit=$?"
