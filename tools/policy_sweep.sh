#!/bin/bash
# Kernel-policy sweep over shapes outside the bench configs (tools build,
# tools/tune.py interleaved rounds): tile width U = 1 / 2 and the early
# prologue for encodes of 1-4 rows, U for reconstructs of 1-4 rows.
# Output: gpurun_out/policy_<shape>.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="nt_load=1,nt_store=1,depth=2,fuse_tail=1"
run() {  # config variants
  local tag=${1//,/_}
  timeout -k 10 200 python tools/tune.py --config "$1" --rounds 9 --variants "$2" > "gpurun_out/policy_$tag.txt" 2>&1
  local rc=$?; echo "$1 rc=$rc"; grep knobs "gpurun_out/policy_$tag.txt" | head -4; return $rc
}
ENC="$B,chunks=1;$B,chunks=2;$B,chunks=1,early=1;$B,chunks=2,early=1"
DEC="$B,chunks=1;$B,chunks=2"
run 8,1,4,512 "$ENC" &&
run 8,2,4,512 "$ENC" &&
run 10,3,16,64 "$ENC" &&
run 12,4,16,64 "$ENC" &&
run 16,4,16,64 "$ENC" &&
run 6,4,4,512 "$ENC" &&
run 8,3,4,512,2 "$DEC" &&
run 10,4,16,64,1 "$DEC" &&
run 12,4,16,64,4 "$DEC" &&
run 6,4,4,512,4 "$DEC" &&
run 16,4,16,64,3 "$DEC"
