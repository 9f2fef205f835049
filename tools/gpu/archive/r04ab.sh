#!/bin/bash
# Round 4 (session 28): the r04 random sweeps (pointer tables, compact rebuilds, started calls) at 200x.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04ab
mkdir -p $O
SHMR_SWEEP_SCALE=200 timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_random_sweep.py -k "ptrs or reconstruct_out or started" > $O/sweep_r04_200x.txt 2>&1 || exit $?
echo done-ab
