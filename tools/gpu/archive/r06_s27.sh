#!/bin/bash
# r06 session 27: the watcher's idle spin before it sleeps (knob coalesce_idle_us)
# 200 / 1000 / 5000 us, interleaved: perblock_dev 256 and 1024 queue modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s27
mkdir -p $O
for idle in 200 1000 5000; do
  SHMR_PB_TUNE=coalesce_idle_us=$idle SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 >> $O/perblock256.jsonl 2>> $O/perblock256.err || exit 1
  SHMR_PB_TUNE=coalesce_idle_us=$idle SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done
echo done-s27
