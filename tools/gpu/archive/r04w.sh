#!/bin/bash
# Round 4 (session 23): the new random pointer-table and compact-rebuild sweeps, at 1x then 50x.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_random_sweep.py -k "ptrs or reconstruct_out" > $O/sweep_new_1x.txt 2>&1 || exit $?
SHMR_SWEEP_SCALE=50 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_random_sweep.py -k "ptrs or reconstruct_out" > $O/sweep_new_50x.txt 2>&1 || exit $?
echo done-w
