#!/bin/bash
# r06 session 35: rebuild lattices pinned by every present shard (k = 1 fresh
# rebuilds on a grid); the sweep's grid expectation made precise (no-op
# rebuilds launch nothing): the seeded random sweep at 100x, slab / pool /
# submit tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s35
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_pool.py \
  tests/test_gpu_submit.py tests/test_ptr_grid.py > $O/pytest_lattice.log 2>&1 || exit $?
SHMR_SWEEP_SCALE=100 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread \
    tests/test_gpu_random_sweep.py -m gpu > $O/sweep100.txt 2>&1 || exit $?
echo done-s35
