#!/bin/bash
# Round 3: misaligned 16-byte access cost microbenchmark (vec / dw / x16 load forms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03m
mkdir -p $O gpurun_out/bin
T="timeout -k 10"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/misalign_bench.hip -o gpurun_out/bin/misalign_bench &&
$T 200 gpurun_out/bin/misalign_bench 2048 20 > $O/misalign_bench.jsonl 2>&1
