#!/bin/bash
# Pointer-table reconstructs: segment launches vs the uploaded block/plan table (knob ptrs_segs),
# then the final records of this build (tools/gpu/r03final2.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
D="depth=2,nt_load=1,sc1_store=1,peel=1,early=1"
$T python tools/tune.py --config decode83 --ptrs --rounds 9 --variants "$D,ptrs_segs=1;$D,ptrs_segs=0" \
  > gpurun_out/ptrs_segs_decode83.txt 2>&1 || exit $?
$T python tools/tune.py --config decode104 --ptrs --rounds 9 \
  --variants "$D,fuse_tail=1,ptrs_segs=1;$D,fuse_tail=1,ptrs_segs=0" > gpurun_out/ptrs_segs_decode104.txt 2>&1 || exit $?
bash tools/gpu/r03final2.sh
