#!/bin/bash
# Parity-slot padding A/B (RS(8,3) / RS(4,2) encode, product policy variant):
# data shard slots padded by one 4 KiB page (the bench layout), parity slots
# padded by 0 / 4 / 8 / 12 / 16 KiB.  One process per parity pad (the pitch is
# a buffer property), alternating order over two passes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P83="chunks=1,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1"
for pass in 1 2; do
  for pp in 0 4096 8192 12288 16384; do
    timeout -k 10 120 python -u tools/tune.py --config encode83 --pad 4096 --ppad $pp --rounds 7 --iters 10 \
        --variants "$P83" > gpurun_out/ppad_83_${pp}_$pass.txt 2>&1 || exit $?
    echo "encode83 ppad=$pp pass=$pass $(tail -1 gpurun_out/ppad_83_${pp}_$pass.txt)"
  done
done
