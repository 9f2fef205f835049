#!/bin/bash
# r06 session 28: per-block calls on mapped host buffers through the queue
# (knob coalesce=1) with queue depth 1 / 2 / 4 and a 20 us window, against one
# zero-copy launch per call (coalesce=0) and the host batch, interleaved legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s28
mkdir -p $O
for tune in coalesce_depth=1 coalesce_depth=2 coalesce_depth=4 coalesce_us=20; do
  SHMR_PB_TUNE=$tune timeout -k 10 300 tools/_abx/perblock_host 128 5 >> $O/perblock_host.jsonl 2>> $O/perblock_host.err || exit 1
done
echo done-s28
