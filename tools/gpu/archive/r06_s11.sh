#!/bin/bash
# r06 session 11: the changed GPU tests (soak slice with pool + queue ops, pool,
# submission queue, HOL probe, kernel sweep), a standalone soak of the new ops
# and of every op, the host ASan/UBSan run (build copied to tools/_asanrun),
# the pool legs of ptrs_ab after the multi-pattern routing change.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_soak.py tests/test_gpu_pool.py \
  tests/test_gpu_submit.py tests/test_gpu_hol.py tests/test_gpu_kernel_sweep.py > $O/pytest_changed.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/soak.py --seconds 60 --threads 12 --ops 8,9 > $O/soak_pool.jsonl 2>&1 || exit $?
timeout -k 10 240 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak_all.jsonl 2>&1 || exit $?
ASAN_DIR=tools/_asanrun timeout -k 10 900 bash tools/asan_host.sh run $O/asan > $O/asan.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ptrs_ab.py --config decode83 --rounds 7 --legs slots,slab,pool_dense,pool_dense_tab,pool_holed,pool_holed_tab > $O/ptrs_ab_decode83.jsonl 2>&1 || exit $?
echo done-s11
