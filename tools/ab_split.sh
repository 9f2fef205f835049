#!/bin/bash
# Split drain A/B (tools build): RS(10,4) 16 MiB encode with its policy variant
# (U = 2, early prologue, fused tails, per-dword math) against the same kernel
# whose last N full 8 KiB tiles run as 4 KiB halves (knob split=N).  Parity of
# the split variants first, then interleaved rounds in one process.
# Usage: tools/ab_split.sh [tag]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tag=${1:-split}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread \
    -k "split" > gpurun_out/ab_${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ab_${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
P="chunks=2,nt_load=1,nt_store=1,depth=2,early=1,fuse_tail=1,serial=1"
V="$P;$P,split=512;$P,split=1024;$P,split=2048;$P,split=4096;$P,split=8192"
# --pad 1536: the bench's 4 KiB-aligned shard slot (1,679,360 B) over tune.py's 256 B alignment
timeout -k 10 300 python -u tools/tune.py --config encode104 --pad 1536 --rounds 11 --iters 10 --variants "$V" \
    > gpurun_out/ab_${tag}_encode104.txt 2>&1
rc=$?; cat gpurun_out/ab_${tag}_encode104.txt; exit $rc
