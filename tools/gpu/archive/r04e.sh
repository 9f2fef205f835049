#!/bin/bash
# Round 4 (session 5): pointer tables against slots in one process (tools/ptrs_ab.py) --
# the table's own cost vs the allocations' placement; config 5 on the final host code.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04e
mkdir -p $O
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 300 python tools/ptrs_ab.py --config $c --rounds 11 > $O/ptrs_ab_$c.txt 2>&1 || exit $?
done
mkdir -p /tmp/vb
timeout -k 10 400 shmr_amd/_lib/shmr_vfs_bench /tmp/vb 256 4 0 3 > $O/e2e_virtual_file_nofsync.jsonl 2> $O/e2e_vf.err || exit $?
echo done-e
