#!/bin/bash
# r06 session 30: lattice tables needing an uploaded slot list take the table
# kernels (knob lattice_list=0): pool / slab / sweep / submit tests, soak of the
# pool ops, ptrs_ab pool legs (lattice, table, list; few holes = segment runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s30
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pool.py tests/test_gpu_slab.py \
  tests/test_gpu_submit.py tests/test_gpu_kernel_sweep.py tests/test_gpu_random_sweep.py > $O/pytest_routing.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/soak.py --seconds 40 --threads 12 --ops 8,9 > $O/soak_pool.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/ptrs_ab.py --config encode83 --rounds 7 --legs slots,slab_sep,slab,pool_dense,pool_dense_tab,pool_holed,pool_holed_tab,pool_holed_list,pool_few,pool_few_tab,pool_few_list > $O/ptrs_ab_encode83.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u tools/ptrs_ab.py --config decode83 --rounds 7 --legs slots,slab,pool_dense,pool_dense_tab,pool_holed,pool_holed_tab,pool_holed_list,pool_few,pool_few_tab,pool_few_list > $O/ptrs_ab_decode83.jsonl 2>&1 || exit $?
echo done-s30
