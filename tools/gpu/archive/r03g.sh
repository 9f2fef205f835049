#!/bin/bash
# Round 3: the wave-run DPP realign tile (tools) on the packed layout: parity,
# then in-process A/B against the unaligned vector path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03g
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -k "contiguous_layout_realigned" -x -q --timeout 120 --timeout-method thread > $O/pytest_realign.log 2>&1 &&
$T 400 python tools/tune.py --config encode104 --packed --rounds 11 \
  --variants "chunks=2,nt_load=1,nt_store=1,depth=2,early=1,serial=1,fuse_tail=1;chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1;chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1,serial=1,realign=1;chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1" > $O/tune_encode104_packed_realign_run.txt 2>&1 &&
$T 400 python tools/tune.py --config decode104 --packed --rounds 11 \
  --variants "compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1;compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1;compact=0,chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1;compact=0,chunks=2,nt_load=1,nt_store=1,depth=2,fuse_tail=1" > $O/tune_decode104_packed_realign_run.txt 2>&1
