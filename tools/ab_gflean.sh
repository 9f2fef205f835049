#!/bin/bash
# Lean GF probe (tools/gflean.hip) against the product kernels' policy
# variants on the same box: RS(10,4) (tile-multiple S = 1,671,168 in the
# probe; the product at the reference's S = 1,677,722) and RS(8,3), both on
# the bench's shard slots.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
[ -x tools/_probe/gflean ] || exit 3
GFLEAN_ONLY=104 timeout -k 10 120 tools/_probe/gflean 1671168 64 20 1679360 9 > gpurun_out/gflean_104.jsonl 2>&1 || exit $?
cat gpurun_out/gflean_104.jsonl
GFLEAN_ONLY=83 timeout -k 10 120 tools/_probe/gflean 524288 512 20 528384 9 > gpurun_out/gflean_83.jsonl 2>&1 || exit $?
cat gpurun_out/gflean_83.jsonl
timeout -k 10 200 python -u tools/tune.py --config encode104 --pad 1536 --rounds 9 --iters 10 \
    --variants "chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1" > gpurun_out/gflean_prod104.txt 2>&1 || exit $?
tail -1 gpurun_out/gflean_prod104.txt
timeout -k 10 200 python -u tools/tune.py --config encode83 --pad 4096 --rounds 9 --iters 10 \
    --variants "chunks=1,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1" > gpurun_out/gflean_prod83.txt 2>&1 || exit $?
tail -1 gpurun_out/gflean_prod83.txt
