#!/bin/bash
# Pacing (s_sleep before each look-ahead load) against the default policy.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1,depth=2"
run() {
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 11 --variants "$2" > "gpurun_out/ab_pace_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -6 "gpurun_out/ab_pace_$1.txt"; return $rc
}
run encode83 "$N;$N,pace=1;$N,pace=2" &&
run encode104 "$N,chunks=2,fuse_tail=1;$N,chunks=2,fuse_tail=1,pace=1;$N,chunks=2,fuse_tail=1,pace=2" &&
run decode83 "$N,wgs_per_cu=7;$N,wgs_per_cu=7,pace=1;$N,wgs_per_cu=7,pace=2;$N,pace=1"
