#!/bin/bash
# Repeat: RS(10,4) compact rebuild, early prologue with sc1 stores against the policy (two processes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
D="depth=2,nt_load=1,sc1_store=1,peel=1,fuse_tail=1"
for r in 1 2; do
$T python tools/tune.py --config decode104 --compact --align 4096 --rounds 21 --variants "$D;$D,early=1" \
  >> gpurun_out/early_decode104_rep.txt 2>&1 || exit $?
$T python tools/tune.py --config decode83e3 --compact --pad 4096 --rounds 11 --variants "$D;$D,early=1" \
  >> gpurun_out/early_decode83e3_rep.txt 2>&1 || exit $?
done
