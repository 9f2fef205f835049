#!/bin/bash
# Round 5 (session 11): config 5 with 16 vs 24 concurrent per-block tasks, interleaved
# (16, 24, 16, 24), mapped Block Cache, fsync off and on -- a fourth box for the r04 question
# (+13 / +14 % on two boxes, -1 % on a third).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05k
mkdir -p $O
for fsy in 0 1; do
  for n in 16 24 16 24; do
    SHMR_VFS_TASKS=$n SHMR_VFS_PINNED_ONLY=1 timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 $fsy 3 \
      >> $O/e2e_vf_tasks${n}_fsync${fsy}.jsonl 2>> $O/e2e_vf.err || exit $?
    rm -rf /tmp/vb
  done
done
echo done-k
