#!/bin/bash
# r06 session 7: completion by mark kernel vs by the watcher's event poll.
set -o pipefail
O=gpurun_out/r06s7
mkdir -p $O
for tune in coalesce_depth=1,coalesce_mark=1 coalesce_depth=1,coalesce_mark=0 coalesce_depth=2,coalesce_mark=0 coalesce_depth=1,coalesce_mark=0,coalesce_target=256; do
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 5 >> $O/perblock256.jsonl 2>> $O/perblock256.err || exit 1
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done
echo "exit=$?"
