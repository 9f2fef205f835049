#!/bin/bash
# Pointer-table cache: its tests, then bench lines of the pointer-table layout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ptrs.py tests/test_gpu_capture.py \
  tests/test_gpu_bench.py > gpurun_out/pytest_ptrs3.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
for c in encode83 decode83 encode104 decode104; do
  $T python bench.py --config $c --layout ptrs >> gpurun_out/bench_ptrs.jsonl 2>> gpurun_out/bench_ptrs.err || exit $?
  $T python bench.py --config $c >> gpurun_out/bench_ptrs.jsonl 2>> gpurun_out/bench_ptrs.err || exit $?
done
