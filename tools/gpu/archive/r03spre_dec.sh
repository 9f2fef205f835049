#!/bin/bash
# Compact rebuilds: scalar-loaded tables (no LDS staging, no barrier) with sc1 stores against the policy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
D="depth=2,nt_load=1,sc1_store=1,fuse_tail=1"
$T python tools/tune.py --config decode83 --compact --pad 4096 --rounds 11 --variants "$D,peel=1;$D,spre=1" \
  > gpurun_out/spre_decode83.txt 2>&1 || exit $?
$T python tools/tune.py --config decode104 --compact --align 4096 --rounds 11 --variants "$D,peel=1,early=1;$D,peel=1;$D,spre=1" \
  > gpurun_out/spre_decode104.txt 2>&1
