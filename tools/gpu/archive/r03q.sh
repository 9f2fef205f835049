#!/bin/bash
# Round 3 (session 2): pointer-table entry points' GPU tests, then the profile part given as $1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ptrs.py \
  "tests/test_gpu_bench.py::test_bench_line_contract" > gpurun_out/pytest_ptrs.log 2>&1
rc=$?
echo "pytest rc=$rc"
# 0 passed, 1 test failures: the GPU is fine, go on; anything else (fault, abort, time limit): stop
[ $rc -le 1 ] || exit $rc
[ -n "${1:-}" ] || exit $rc
bash tools/profile_all.sh r03 "$1" > gpurun_out/profile_all_r03_part$1.log 2>&1
