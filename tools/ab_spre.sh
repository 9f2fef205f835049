#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
S2="chunks=2,nt_load=1,nt_store=1,depth=2,spre=1,fuse_tail=1,serial=1"
S2N="chunks=2,nt_load=1,nt_store=1,depth=2,spre=1,fuse_tail=1"
S1="chunks=1,nt_load=1,nt_store=1,depth=2,spre=1,fuse_tail=1,serial=1"
V="$P;$S2;$S2,wgs_per_cu=4;$S2N;$S1;$S1,wgs_per_cu=6;$S1,wgs_per_cu=5;$S1,wgs_per_cu=4"
timeout -k 10 300 python -u tools/tune.py --config encode104 --pad 1536 --rounds 9 --iters 10 --variants "$V" \
    > gpurun_out/ab_spre_encode104.txt 2>&1 || exit $?
cat gpurun_out/ab_spre_encode104.txt
P83="chunks=1,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1"
Q83="chunks=1,nt_load=1,nt_store=1,depth=2,spre=1"
V="$P83;$Q83;$Q83,wgs_per_cu=6;$Q83,wgs_per_cu=5;$Q83,wgs_per_cu=4"
timeout -k 10 300 python -u tools/tune.py --config encode83 --pad 4096 --rounds 9 --iters 10 --variants "$V" \
    > gpurun_out/ab_spre_encode83.txt 2>&1 || exit $?
cat gpurun_out/ab_spre_encode83.txt
