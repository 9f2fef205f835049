#!/bin/bash
# Round 3: the peeled depth-2 shard ring (tools knob peel=1): parity over the
# peel variants, then in-process A/B against each headline policy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03h
mkdir -p $O
T="timeout -k 10"
E83="nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1"
E104="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
D83C="compact=1,nt_load=1,depth=2,fuse_tail=1,sc1_store=1"
D104C="compact=1,nt_load=1,depth=2,fuse_tail=1,sc1_store=1"
D83I="compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,wgs_per_cu=7"
$T 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -k "peel or reconstruct_variants_match or store_policies" -x -q --timeout 200 --timeout-method thread > $O/pytest_peel.log 2>&1 &&
$T 300 python tools/tune.py --config encode83 --rounds 11 --variants "$E83;$E83,peel=1" > $O/tune_encode83_peel.txt 2>&1 &&
$T 300 python tools/tune.py --config encode104 --rounds 11 --variants "$E104;$E104,peel=1" > $O/tune_encode104_peel.txt 2>&1 &&
$T 300 python tools/tune.py --config decode83 --rounds 11 --variants "$D83C;$D83C,peel=1;$D83I;$D83I,peel=1" > $O/tune_decode83_peel.txt 2>&1 &&
$T 300 python tools/tune.py --config decode104 --rounds 11 --variants "$D104C;$D104C,peel=1" > $O/tune_decode104_peel.txt 2>&1 &&
$T 300 python tools/tune.py --config encode42 --rounds 11 --variants "$E83;$E83,peel=1" > $O/tune_encode42_peel.txt 2>&1
[ $? -eq 0 ] &&
$T 300 python tools/tune.py --config decode104 --packed --rounds 11 --variants "$D104C;$D104C,realign=1;compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1;compact=0,nt_load=1,nt_store=1,depth=2,fuse_tail=1,realign=1" > $O/tune_decode104_packed_realign.txt 2>&1 &&
$T 300 python tools/tune.py --config decode83 --packed --rounds 11 --variants "$D83C;$D83C,realign=1;$D83I;$D83I,realign=1" > $O/tune_decode83_packed_realign.txt 2>&1 &&
$T 300 python -u -m pytest tests/test_gpu_compact.py -k "packed_layout" -x -q --timeout 120 --timeout-method thread > $O/pytest_compact_packed.log 2>&1
