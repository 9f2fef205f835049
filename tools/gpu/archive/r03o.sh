#!/bin/bash
# Round 3: XOR access-pattern replica on the packed RS(10,4) layout: shard slot
# 1677722 (off 16-byte alignment) vs 1677728 (16-byte) vs 1679360 (4 KiB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03o
mkdir -p $O gpurun_out/bin
T="timeout -k 10"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o gpurun_out/bin/membench &&
for P in 1679360 1677728 1677722; do
  for ONLY in 104 102; do
    MEMBENCH_ONLY=$ONLY MEMBENCH_PITCH=$P $T 120 gpurun_out/bin/membench 1671168 64 20 >> $O/membench_packed.jsonl 2>&1 || exit 1
  done
done
