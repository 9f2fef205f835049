#!/bin/bash
# Round 5 (session 1): slab allocator + slot-grid pointer tables: GPU tests, then
# the pointer-table A/B (tools/ptrs_ab.py) on all four configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05a
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_slab.py > $O/pytest_slab2.log 2>&1 || exit $?
timeout -k 10 500 $PT tests/test_gpu_bench.py > $O/pytest_bench_ptrs.log 2>&1 || exit $?
for c in encode83 decode83 encode104 decode104; do
  timeout -k 10 240 python -u tools/ptrs_ab.py --config $c --rounds 9 > $O/ptrs_ab_$c.txt 2>&1 || exit $?
done
echo done-a
