#!/bin/bash
# r06 session 6: queue depth 1 vs 2 (device and mapped host per-block calls).
set -o pipefail
O=gpurun_out/r06s6
mkdir -p $O
for tune in coalesce_depth=1 coalesce_depth=1,coalesce_target=128 coalesce_depth=2; do
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 5 >> $O/perblock256.jsonl 2>> $O/perblock256.err || exit 1
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done
for tune in coalesce_depth=1 coalesce_depth=2; do
  SHMR_PB_TUNE=$tune timeout -k 10 300 tools/_abx/perblock_host 128 5 >> $O/perblock_host.jsonl 2>> $O/perblock_host.err || exit 1
done
echo "exit=$?"
