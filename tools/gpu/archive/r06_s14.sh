#!/bin/bash
# r06 session 14: per-block device calls through the lock-free queue (submit
# span, cgroup throttling), a kernel trace of the 256-block T=16 async case,
# then s11's list: changed GPU tests incl. the kernel sweep, soaks (pool + queue
# ops; every op), host ASan/UBSan, ptrs_ab pool legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06s14
mkdir -p $O
export TMPDIR=/tmp
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 256 7 > $O/perblock256.jsonl 2> $O/perblock256.err || exit 1
SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 > $O/perblock1024.jsonl 2> $O/perblock1024.err || exit 1
SHMR_PB_QUEUE_ONLY=1 SHMR_PB_ASYNC_ONLY=1 SHMR_PB_THREADS=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d $O/kt -o pb16 -- tools/_abx/perblock_dev 256 5 > $O/perblock256_T16_traced.jsonl 2> $O/kt.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_submit.py tests/test_gpu_pool.py \
  tests/test_gpu_hol.py tests/test_gpu_soak.py tests/test_gpu_kernel_sweep.py > $O/pytest_changed.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/soak.py --seconds 60 --threads 12 --ops 8,9 > $O/soak_pool.jsonl 2>&1 || exit $?
timeout -k 10 240 python -u tools/soak.py --seconds 120 --threads 12 > $O/soak_all.jsonl 2>&1 || exit $?
ASAN_DIR=tools/_asanrun timeout -k 10 900 bash tools/asan_host.sh run $O/asan > $O/asan.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ptrs_ab.py --config decode83 --rounds 7 --legs slots,slab,pool_dense,pool_dense_tab,pool_holed,pool_holed_tab > $O/ptrs_ab_decode83.jsonl 2>&1 || exit $?
echo done-s14
