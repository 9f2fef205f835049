#!/bin/bash
# r06 session 5: force-launch on wait; the drop-in on mapped host buffers.
set -o pipefail
O=gpurun_out/r06s5
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 python -u tools/hol_held.py --hold 1.0 > $O/hol_held.jsonl 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_submit.py tests/test_gpu_pool.py tests/test_gpu_hol.py tests/test_gpu_ptrs.py tests/test_gpu_capture.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 tools/_abx/perblock_host 128 5 > $O/perblock_host.jsonl 2> $O/perblock_host.err &&
for tune in coalesce_target=64 coalesce_target=128; do
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 5 >> $O/perblock256.jsonl 2>> $O/perblock256.err || exit 1
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done
echo "exit=$?"
