#!/bin/bash
# Round 4 (session 25): the random started-call sweep at 1x and 30x.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_random_sweep.py -k started > $O/sweep_started_1x.txt 2>&1 || exit $?
SHMR_SWEEP_SCALE=30 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_random_sweep.py -k started > $O/sweep_started_30x.txt 2>&1 || exit $?
echo done-y
