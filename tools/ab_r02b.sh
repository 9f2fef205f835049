#!/bin/bash
# Decode / RS(10,4) launch-shape sweep (tools build, tools/tune.py interleaved
# rounds).  Output: gpurun_out/ab_r02b_<cfg>.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1"
run() {  # config variants [extra args]
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 7 --variants "$2" ${3:-} > "gpurun_out/ab_r02b_$1$4.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -12 "gpurun_out/ab_r02b_$1$4.txt"; return $rc
}
run decode83 "$N,depth=2;$N,depth=2,chunks=2;$N;$N,depth=2,threads=512;$N,depth=2,threads=128;$N,depth=2,early=1" "" "" &&
run decode83 "$N,depth=2;$N,depth=2,chunks=2;$N;$N,depth=2,threads=512" "--same-pattern" "_same" &&
run decode104 "$N,depth=2,fuse_tail=1;$N,depth=2,chunks=2,fuse_tail=1;$N,fuse_tail=1;$N,depth=2,fuse_tail=1,threads=512" "" "" &&
run encode104 "$N,depth=2,chunks=2,fuse_tail=1;$N,chunks=2,fuse_tail=1;$N,depth=2,chunks=2,fuse_tail=1,threads=128;$N,depth=2,fuse_tail=1,threads=512;$N,depth=2,fuse_tail=1" "" ""
