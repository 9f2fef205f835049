#!/bin/bash
# Serial-ordered GF math under occupancy caps: separates the cost of the
# ordering from the cost of the extra waves (tools/ab_serial.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1,depth=2"
run() {
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 11 --variants "$2" > "gpurun_out/ab_occ3_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -8 "gpurun_out/ab_occ3_$1.txt"; return $rc
}
run encode83 "$N;$N,serial=1;$N,serial=1,wgs_per_cu=7;$N,serial=1,wgs_per_cu=6" &&
run encode104 "$N,chunks=2,fuse_tail=1;$N,chunks=2,fuse_tail=1,serial=1;$N,fuse_tail=1,serial=1;$N,fuse_tail=1,serial=1,wgs_per_cu=5" &&
run decode83 "$N,wgs_per_cu=7;$N,wgs_per_cu=7,serial=1;$N,serial=1,wgs_per_cu=6"
