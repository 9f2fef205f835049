#!/bin/bash
# Round 5 (session 15): rocprofv3 kernel traces + PMC traffic of the six bench configs on the
# final r05 tree (bench.py defaults: K = 100, two-event timed region).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05o
mkdir -p $O
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/profile_all.sh r05final 1 > $O/profile_all_r05_part1.log 2>&1 || exit $?
find gpurun_out -name '*_kernel_trace.csv' -delete
find gpurun_out -name 'pmc_counter_collection.csv' -delete
echo done-o
