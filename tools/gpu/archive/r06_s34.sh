#!/bin/bash
# r06 session 34: robustness on the final tree -- a 600 s soak of every entry
# point on 12 threads (queue and pool ops included) and the seeded random
# sweep at 100x.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s34
mkdir -p $O
timeout -k 10 720 python -u tools/soak.py --seconds 600 --threads 12 > $O/soak600.jsonl 2>&1 || exit $?
SHMR_SWEEP_SCALE=100 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_random_sweep.py -m gpu > $O/sweep100.txt 2>&1 || exit $?
echo done-s34
