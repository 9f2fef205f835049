#!/bin/bash
# Round 3: the RS(10,4) memory-pipeline counter table (GF kernel on slots and
# on the packed buffer, the 10 -> 4 XOR replica).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 bash tools/counter_passes.sh $O/ctr > $O/counter_passes.txt 2>&1 &&
python tools/counter_table.py $O/ctr --json $O/counters_encode104.json > $O/counters_encode104.md 2>&1
