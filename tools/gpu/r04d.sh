#!/bin/bash
# Round 4 final (part 1): rocprofv3 kernel traces + PMC traffic of the six bench configs on the
# final build, the whole GPU suite, smoke and the bench lines (`bash tools/gpu/r04d.sh [part]`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04d
mkdir -p $O
PART=${1:-1}
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/profile_all.sh r04 $PART > $O/profile_all_r04_part$PART.log 2>&1 || exit $?
find gpurun_out -name '*_kernel_trace.csv' -delete
find gpurun_out -name 'pmc_counter_collection.csv' -delete
if [ "$PART" = 1 ]; then
  cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json   # (the box's copy) bench lines then match traffic
  for c in encode83 decode83 encode104 decode104 encode42 codec104; do
    timeout -k 10 300 python bench.py --config $c >> $O/bench_final.jsonl 2>> $O/bench_final.err || exit $?
  done
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.log 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu_final.log 2>&1 || exit $?
fi
echo done-final-$PART
