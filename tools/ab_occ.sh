#!/bin/bash
# Occupancy caps (tuning wgs_per_cu: LDS padding limits resident 256-lane
# workgroups per CU = waves per SIMD) for the shapes whose kernels fit 7-8
# waves/SIMD.  Output: gpurun_out/ab_occ_<cfg>.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1,depth=2"
run() {
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 9 --variants "$2" > "gpurun_out/ab_occ_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -8 "gpurun_out/ab_occ_$1.txt"; return $rc
}
run decode83 "$N;$N,wgs_per_cu=7;$N,wgs_per_cu=6;$N,wgs_per_cu=5;$N,wgs_per_cu=4" &&
run decode104 "$N,fuse_tail=1;$N,fuse_tail=1,wgs_per_cu=7;$N,fuse_tail=1,wgs_per_cu=6;$N,fuse_tail=1,wgs_per_cu=5" &&
run encode42 "$N,early=1;$N,early=1,wgs_per_cu=6;$N,early=1,wgs_per_cu=5;$N,early=1,wgs_per_cu=4" &&
run encode83 "$N;$N,wgs_per_cu=5;$N,wgs_per_cu=4"
