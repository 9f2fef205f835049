#!/bin/bash
# End of round 3: the whole GPU suite, smoke and the default bench line on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_end.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_end.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_end.jsonl 2> gpurun_out/bench_end.err
