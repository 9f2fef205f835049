#!/bin/bash
# GF kernel vs its XOR-only twin in the SAME launch shape (diag=1: identical
# loads/stores/tiling, XOR instead of GF multiply -- wrong results by design),
# interleaved rounds: the ceiling of the kernel structure itself.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
N="nt_load=1,nt_store=1,depth=2"
run() {
  timeout -k 10 240 python tools/tune.py --config "$1" --rounds 11 --variants "$2" > "gpurun_out/ab_diag_$1.txt" 2>&1
  local rc=$?; echo "tune $1 rc=$rc"; tail -6 "gpurun_out/ab_diag_$1.txt"; return $rc
}
run encode104 "$N,chunks=2,fuse_tail=1;$N,chunks=2,fuse_tail=1,diag=1;$N,fuse_tail=1;$N,fuse_tail=1,diag=1" &&
run encode83 "$N;$N,diag=1;$N,chunks=2;$N,chunks=2,diag=1" &&
run decode83 "$N,wgs_per_cu=7;$N,wgs_per_cu=7,diag=1"
