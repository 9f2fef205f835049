#!/bin/bash
# Encodes: sc1 stores vs nontemporal stores (parity rows into their own allocation), aligned slots.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
E="depth=2,early=1,fuse_tail=1,nt_load=1"
$T python tools/tune.py --config encode83 --pad 4096 --rounds 11 --variants "$E,nt_store=1;$E,sc1_store=1" \
  > gpurun_out/sc1_encode83.txt 2>&1 || exit $?
$T python tools/tune.py --config encode42 --pad 4096 --rounds 11 --variants "$E,nt_store=1;$E,sc1_store=1" \
  > gpurun_out/sc1_encode42.txt 2>&1 || exit $?
E="chunks=2,depth=2,early=1,fuse_tail=1,nt_load=1,serial=1,wave_run=1"
$T python tools/tune.py --config encode104 --align 4096 --rounds 11 --variants "$E,nt_store=1;$E,sc1_store=1" \
  > gpurun_out/sc1_encode104.txt 2>&1
