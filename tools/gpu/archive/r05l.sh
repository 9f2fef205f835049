#!/bin/bash
# Round 5 (session 12): config 5 with the r05 defaults (24 load tasks), fsync off and on, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05l
mkdir -p $O
for r in 1 2; do
  for fsy in 0 1; do
    SHMR_VFS_PINNED_ONLY=1 timeout -k 10 300 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 $fsy 3 \
      >> $O/e2e_vf_fsync${fsy}.jsonl 2>> $O/e2e_vf.err || exit $?
    rm -rf /tmp/vb
  done
done
timeout -k 10 300 python tools/e2e_bench.py > $O/e2e_host_path.json 2> $O/e2e_host_path.err || exit $?
echo done-l
