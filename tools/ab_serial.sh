#!/bin/bash
# A/B of the per-dword-ordered GF math ("serial": fewer live VGPRs, more waves
# per SIMD) against the default policy, tools/tune.py interleaved rounds.
# Output: gpurun_out/ab_serial_<cfg>.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1"
run() {
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 9 --variants "$2" > "gpurun_out/ab_serial_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -8 "gpurun_out/ab_serial_$1.txt"; return $rc
}
run encode83 "$N,depth=2;$N,depth=2,serial=1;$N,serial=1;$N,depth=5,serial=1;$N,depth=2,chunks=2,serial=1" &&
run encode104 "$N,depth=2,chunks=2,fuse_tail=1;$N,depth=2,chunks=2,fuse_tail=1,serial=1;$N,depth=2,fuse_tail=1,serial=1;$N,fuse_tail=1,serial=1" &&
run decode83 "$N,depth=2;$N,depth=2,serial=1" &&
run decode104 "$N,depth=2,fuse_tail=1;$N,depth=2,fuse_tail=1,serial=1;$N,fuse_tail=1,serial=1" &&
run encode42 "$N,depth=2,early=1;$N,depth=2,early=1,serial=1;$N,depth=2,serial=1"
