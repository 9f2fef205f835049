#!/bin/bash
# Compact rebuilds on the padded slots: the early prologue with sc1 stores against the policy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
D="depth=2,nt_load=1,sc1_store=1,peel=1,fuse_tail=1"
$T python tools/tune.py --config decode83 --compact --pad 4096 --rounds 11 --variants "$D;$D,early=1" \
  > gpurun_out/early_decode83.txt 2>&1 || exit $?
$T python tools/tune.py --config decode104 --compact --align 4096 --rounds 11 --variants "$D;$D,early=1" \
  > gpurun_out/early_decode104.txt 2>&1
