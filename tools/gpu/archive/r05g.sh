#!/bin/bash
# Round 5 (session 7): the random grid-table sweep at 1x and 20x; host sanitizers (ASan + UBSan,
# kernel TU included) on the r05 host code (grid dispatch, slab allocator, O_DIRECT, flush failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05g
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_slab.py tests/test_gpu_random_sweep.py -k "grid or slab" > $O/sweep_grid_1x.txt 2>&1 || exit $?
SHMR_SWEEP_SCALE=20 timeout -k 10 600 $PT tests/test_gpu_random_sweep.py -k grid > $O/sweep_grid_20x.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/asan_host.sh build > $O/asan_build.log 2>&1 || exit $?
timeout -k 10 900 bash tools/asan_host.sh run $O/asan > $O/asan_host.log 2>&1 || exit $?
echo done-g
