#!/bin/bash
# Round 3: packed-layout loss split by side (inputs / outputs misaligned), policy vs DPP realign.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03j
mkdir -p $O
T="timeout -k 10"
$T 300 python tools/misalign_split.py > $O/misalign_split_104.txt 2>&1 &&
$T 300 python tools/misalign_split.py --k 8 --p 3 --block-mib 4 --blocks 512 > $O/misalign_split_83.txt 2>&1
