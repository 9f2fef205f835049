#!/bin/bash
# Round 3: wave-contiguous slot mapping (tools knob wave_run) -- parity, then
# the packed-layout split and the aligned-slot headline configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03k
mkdir -p $O
T="timeout -k 10"
E104="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
D4="nt_load=1,nt_store=1,depth=2,fuse_tail=1,peel=1,chunks=2"
$T 300 python -u -m pytest tests/test_gpu_parity.py -k "wave_run" -x -q --timeout 200 --timeout-method thread > $O/pytest_wave_run.log 2>&1 &&
$T 300 python tools/misalign_split.py > $O/misalign_split_104.txt 2>&1 &&
$T 300 python tools/tune.py --config encode104 --rounds 11 --variants "$E104;$E104,wave_run=1" > $O/tune_encode104_wave_run.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104e4 --rounds 11 --variants "compact=0,$D4;compact=0,$D4,wave_run=1" > $O/tune_decode104e4_wave_run.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --packed --rounds 11 --variants "compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,peel=1;compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,peel=1,chunks=2,wave_run=1;compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1" > $O/tune_decode104_packed_wave_run.txt 2>&1
