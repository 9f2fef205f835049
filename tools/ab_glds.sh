#!/bin/bash
# A/B of the LDS-DMA input ring (glds) against the register ring, one process
# per config, interleaved rounds (tools/tune.py).  Output: gpurun_out/ab_glds_<cfg>.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1"
run() {  # config variants
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 7 --variants "$2" > "gpurun_out/ab_glds_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -12 "gpurun_out/ab_glds_$1.txt"; return $rc
}
run encode104 "chunks=2,$N,depth=2,fuse_tail=1;chunks=2,$N,depth=2;glds=1,$N;glds=1,$N,depth=5;glds=1,$N,depth=9;glds=1,chunks=2,$N;glds=1,chunks=2,$N,depth=5;glds=1,$N,depth=5,fuse_tail=1;glds=1,chunks=2,$N,fuse_tail=1" &&
run encode83 "$N,depth=2;glds=1,$N;glds=1,$N,depth=5;glds=1,$N,depth=9;glds=1,chunks=2,$N;glds=1,chunks=2,$N,depth=5" &&
run decode104 "$N,depth=2,fuse_tail=1;glds=1,$N,fuse_tail=1;glds=1,$N,depth=5,fuse_tail=1;glds=1,$N,depth=5;glds=1,chunks=2,$N,fuse_tail=1" &&
run decode83 "$N,depth=2;glds=1,$N;glds=1,$N,depth=5;glds=1,$N,depth=9" &&
run encode42 "$N,depth=2,early=1;$N,depth=2;glds=1,$N;glds=1,$N,depth=5;glds=1,$N,depth=9"
