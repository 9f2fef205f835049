#!/bin/bash
# Round 3 (session 2), build with the pointer-table early prologue: profiles (both parts), the whole
# GPU suite, smoke, bench lines (the six configs, then the pointer-table layout).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/profile_all.sh r03 > gpurun_out/profile_all_r03.log 2>&1 || exit $?
# per-dispatch traces are merged already (pmc_traffic.json): keep gpurun_out under the 64 MiB copy-back
find gpurun_out -name '*_kernel_trace.csv' -delete
find gpurun_out -name 'pmc_counter_collection.csv' -delete
du -sh gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json   # this build's records, for the bench lines below
for c in encode83 decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err || exit $?
done
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 300 python bench.py --config $c --layout ptrs >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err || exit $?
done
timeout -k 10 300 python bench.py >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err
