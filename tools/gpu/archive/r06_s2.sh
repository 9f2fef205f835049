#!/bin/bash
# r06 session 2: the queue with host-word completion; allocation / naming A/B.
set -o pipefail
O=gpurun_out/r06s2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_submit.py tests/test_gpu_pool.py -x -q --timeout 120 --timeout-method thread > $O/pytest_submit.log 2>&1 &&
timeout -k 10 300 tools/_abx/perblock_dev 256 3 > $O/perblock256.jsonl 2> $O/perblock256.err &&
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err &&
timeout -k 10 300 python -u tools/alloc_ab.py --op encode > $O/alloc_ab_encode.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/alloc_ab.py --op decode > $O/alloc_ab_decode.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/ptrs_ab.py --config decode83 --rounds 7 --legs slots,slab,pool_dense,pool_dense_tab,pool_dense_pl,pool_holed,pool_holed_tab,pool_holed_pl > $O/ptrs_ab_decode83.jsonl 2>&1
echo "exit=$?"
