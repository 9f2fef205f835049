#!/bin/bash
# RS(10,4) shard-slot sweep (encode and 2-erasure decode, product policy
# variants): slots of 410 (the bench's 4 KiB-aligned slot) .. 414 pages and
# 410.5 pages, one process per slot, two alternating passes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
E="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
D="chunks=1,nt_load=1,nt_store=1,depth=2,fuse_tail=1"
for pass in 1 2; do
  for pad in 1536 3584 5632 9728 13824 17920; do   # S rounded to 256 B = 1,677,824; +1536 = 410 pages
    timeout -k 10 120 python -u tools/tune.py --config encode104 --pad $pad --rounds 7 --iters 10 --variants "$E" \
        > gpurun_out/pad104_e_${pad}_$pass.txt 2>&1 || exit $?
    timeout -k 10 120 python -u tools/tune.py --config decode104 --pad $pad --rounds 7 --iters 10 --variants "$D" \
        > gpurun_out/pad104_d_${pad}_$pass.txt 2>&1 || exit $?
    echo "pad=$pad pass=$pass encode $(tail -1 gpurun_out/pad104_e_${pad}_$pass.txt | sed 's/.*"frac"/frac/') decode $(tail -1 gpurun_out/pad104_d_${pad}_$pass.txt | sed 's/.*"frac"/frac/')"
  done
done
