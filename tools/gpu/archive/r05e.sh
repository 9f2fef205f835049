#!/bin/bash
# Round 5 (session 5): capture-block release timing behind a queued replay; O_DIRECT shard
# files after the descriptor-table race fix; config 5 with and without O_DIRECT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05e
mkdir -p $O
PT="python -u -m pytest -x -q -s --timeout 120 --timeout-method thread"
timeout -k 10 200 $PT tests/test_gpu_capture.py -k queued > $O/pytest_queued.log 2>&1
rc=$?; echo "queued rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 $PT tests/test_host_cpp.py -k "encode_failure or direct_io" > $O/pytest_direct.log 2>&1
rc=$?; echo "direct rc=$rc"; [ $rc -le 1 ] || exit $rc
for fsy in 0 1; do
  for d in 0 1; do
    SHMR_VFS_DIRECT=$d SHMR_VFS_PINNED_ONLY=1 timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench /tmp/vb_$d 256 4 $fsy 3 \
      > $O/vfs_direct${d}_fsync${fsy}.jsonl 2>&1 || exit $?
    rm -rf /tmp/vb_$d
  done
done
echo done-e
