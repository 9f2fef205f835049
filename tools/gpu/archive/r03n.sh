#!/bin/bash
# Round 3: aligned-store runs for misaligned output rows (tools knob st_align).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03n
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -k "st_align" -x -q --timeout 200 --timeout-method thread > $O/pytest_st_align.log 2>&1 &&
$T 300 python tools/misalign_split.py > $O/misalign_split_104.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --packed --rounds 11 --variants "compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,peel=1;compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,peel=1,st_align=1" > $O/tune_decode104_packed_st_align.txt 2>&1
