#!/bin/bash
# Round 5 (session 16): config 5 with streaming-store copy-in / copy-out
# (VfsOptions::streaming_copies) against memcpy, interleaved (0, 1, 0, 1, 0, 1), mapped
# Block Cache, fsync off and on; then the host C++ GPU tests (the fuzz draws the option).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q
mkdir -p $O
cp gpurun_out/r05p/copy_probe.jsonl $O/ 2>/dev/null
for fsy in 0 1; do
  for st in 0 1 0 1 0 1; do
    SHMR_VFS_STREAM=$st SHMR_VFS_PINNED_ONLY=1 timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 $fsy 3 \
      >> $O/e2e_vf_stream${st}_fsync${fsy}.jsonl 2>> $O/e2e_vf.err || exit $?
    rm -rf /tmp/vb
  done
done
timeout -k 10 600 python -u -m pytest tests/test_host_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_host_cpp.log 2>&1 || exit $?
echo done-q
