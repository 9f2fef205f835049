#!/bin/bash
# r06 session 36: kernel traces + PMC traffic of the pointer-table layouts
# (bench.py --layout ptrs, slab and torch buffers) on the r06 kernel build,
# then their bench lines with the traffic matched.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s36
mkdir -p $O
export TMPDIR=/tmp
bash tools/profile_all.sh r06 3 > $O/profile_ptrs.log 2>&1 || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python bench.py --layout ptrs --no-cpu > $O/bench_ptrs.jsonl 2>> $O/bench.err || exit $?
echo done-s36
