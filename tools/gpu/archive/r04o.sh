#!/bin/bash
# Round 4 (session 15): the soak slice test; config 5 with 16 vs 24 per-block tasks (third box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_soak.py > $O/pytest_soak.log 2>&1 || exit $?
mkdir -p /tmp/vb
for n in 16 24 16 24; do
  SHMR_VFS_TASKS=$n timeout -k 10 400 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 0 3 >> $O/e2e_vf_tasks$n.jsonl 2>> $O/e2e_vf.err || exit $?
done
echo done-o
