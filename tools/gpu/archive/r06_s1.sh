#!/bin/bash
# r06 session 1: the submission queue and the slot pool -- correctness, then
# per-block rates and the pool / joint-slot placement A/B.
set -o pipefail
O=gpurun_out/r06s1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_submit.py tests/test_gpu_pool.py -x -v --timeout 120 --timeout-method thread > $O/pytest_submit.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_ptrs.py tests/test_gpu_slab.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ptrs.log 2>&1 &&
timeout -k 10 300 tools/_abx/perblock_dev 256 3 > $O/perblock256.jsonl 2> $O/perblock256.err &&
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err &&
timeout -k 10 300 python -u tools/ptrs_ab.py --config encode83 --rounds 7 --legs slots,slab_sep,slab,pool_dense,pool_dense_tab,pool_holed,pool_holed_tab,joint_pad0k,joint_pad4k,joint_pad8k,joint_pad64k,joint_pad68k,joint_pad1024k > $O/ptrs_ab_encode83.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/ptrs_ab.py --config decode83 --rounds 7 --legs slots,slab,slab_inplace,pool_dense,pool_dense_tab,pool_holed,pool_holed_tab > $O/ptrs_ab_decode83.jsonl 2>&1
echo "exit=$?"
