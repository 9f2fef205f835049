#!/bin/bash
# Round 5 (session 6): rocprofv3 kernel traces + PMC traffic of the pointer-table layouts
# (bench.py --layout ptrs: slab buffers on a slot grid, and torch buffers through the table kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05f
mkdir -p $O
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/profile_all.sh r05 3 > $O/profile_all_r05_part3.log 2>&1 || exit $?
find gpurun_out -name '*_kernel_trace.csv' -delete
find gpurun_out -name 'pmc_counter_collection.csv' -delete
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
for c in encode83 decode83 encode104; do
  timeout -k 10 300 python bench.py --config $c --layout ptrs --no-cpu >> $O/bench_ptrs.jsonl 2>> $O/bench.err || exit $?
done
echo done-f
