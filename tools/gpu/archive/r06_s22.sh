#!/bin/bash
# r06 session 22: does the watcher's blocking event wait on the queue's stream
# hold back launches onto that stream?  Traced runs with coalesce_watch_us
# 200 (default) and 100000 (the watcher never sleeps on the event).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s22
mkdir -p $O
for w in 200 100000; do
  SHMR_PB_TUNE=coalesce_watch_us=$w SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 120 tools/_abx/perblock_dev 256 5 > $O/pb256_T16_w$w.jsonl 2> $O/pb256_T16_w$w.trace || exit 1
  SHMR_PB_TUNE=coalesce_watch_us=$w SHMR_QUEUE_TRACE=1 SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 timeout -k 10 120 tools/_abx/perblock_dev 1024 3 > $O/pb1024_w$w.jsonl 2> $O/pb1024_w$w.trace || exit 1
done
echo done-s22
