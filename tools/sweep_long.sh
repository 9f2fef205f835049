#!/bin/bash
# Long seeded random sweep of the device-resident and host-batch entry points
# against the CPU oracle (tests/test_gpu_random_sweep.py at SHMR_SWEEP_SCALE x
# the suite's case count).  Run on a GPU box:  tools/sweep_long.sh [scale=25]
set -eu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SHMR_SWEEP_SCALE=${1:-25} timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_random_sweep.py -m gpu > gpurun_out/sweep_long.txt 2>&1
tail -3 gpurun_out/sweep_long.txt
