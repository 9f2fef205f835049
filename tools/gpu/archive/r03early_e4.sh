#!/bin/bash
# 4-erasure compact rebuilds (4 rows, U = 2): the early prologue with sc1 stores against the policy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
D="chunks=2,wave_run=1,depth=2,nt_load=1,sc1_store=1,peel=1,fuse_tail=1"
for r in 1 2; do
$T python tools/tune.py --config decode104e4 --compact --align 4096 --rounds 11 --variants "$D;$D,early=1" \
  >> gpurun_out/early_decode104e4.txt 2>&1 || exit $?
done
