#!/bin/bash
# Shard-pitch padding x early prologue on the bench configs (tools build,
# tools/tune.py interleaved rounds).  "cur" = the bench's r02 pitch
# (roundup(S, 4096)), "pad" = that plus one 4 KiB page per shard slot.
# Output: gpurun_out/ab_pad_<config>_<cur|pad>.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="nt_load=1,nt_store=1,depth=2,fuse_tail=1"
run() {  # config pad tag variants
  timeout -k 10 240 python tools/tune.py --config "$1" --pad "$2" --rounds 13 --variants "$4" > "gpurun_out/ab_pad_$1_$3.txt" 2>&1
  local rc=$?; echo "$1 $3 rc=$rc"; grep knobs "gpurun_out/ab_pad_$1_$3.txt"; return $rc
}
E83="$B,chunks=1;$B,chunks=1,early=1"
E104="$B,chunks=2,early=1,serial=1;$B,chunks=2"
E42="$B,chunks=1,early=1;$B,chunks=1"
D1="$B,chunks=1,wgs_per_cu=7"
D2="$B,chunks=1"
run encode83 0 cur "$E83" && run encode83 4096 pad "$E83" &&
run encode104 1536 cur "$E104" && run encode104 5632 pad "$E104" &&
run encode42 0 cur "$E42" && run encode42 4096 pad "$E42" &&
run decode83 0 cur "$D1" && run decode83 4096 pad "$D1" &&
run decode104 1536 cur "$D2" && run decode104 5632 pad "$D2"
