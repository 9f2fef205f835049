#!/bin/bash
# Final records without the profile passes (they are committed for this build): the whole GPU
# suite, smoke, bench lines (the six configs, then the pointer-table layout).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
for c in encode83 decode83 encode104 decode104 encode42 codec104; do
  timeout -k 10 300 python bench.py --config $c >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err || exit $?
done
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 300 python bench.py --config $c --layout ptrs >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err || exit $?
done
timeout -k 10 300 python bench.py >> gpurun_out/bench_final.jsonl 2>> gpurun_out/bench_final.err
