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
cp gpurun_out/pmc_traffic.json $O/pmc_traffic.json
for d in gpurun_out/prof_r06_*; do   # keep the summaries only (gpurun_out must stay under 64 MiB)
  k=$(basename $d)
  f=$(find $d/kt -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$O/${k#prof_r06_}_kernel_stats.csv"
done
rm -rf gpurun_out/prof_r06_*
timeout -k 10 300 python bench.py --layout ptrs --no-cpu > $O/bench_ptrs.jsonl 2>> $O/bench.err || exit $?
echo done-s36
