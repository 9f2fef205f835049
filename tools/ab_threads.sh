#!/bin/bash
# Workgroup size (128 / 256 / 512 lanes) at the default policy, interleaved rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1,depth=2"
run() {
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 11 --variants "$2" > "gpurun_out/ab_threads_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -4 "gpurun_out/ab_threads_$1.txt"; return $rc
}
run encode83 "$N;$N,threads=128;$N,threads=512" &&
run encode42 "$N,early=1;$N,threads=128;$N,threads=512"
