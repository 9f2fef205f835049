#!/bin/bash
# r06 session 3: queue with watcher + encode segment launches; kernel sweep.
set -o pipefail
O=gpurun_out/r06s3
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_submit.py tests/test_gpu_pool.py tests/test_gpu_kernel_sweep.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 tools/_abx/perblock_dev 256 3 > $O/perblock256.jsonl 2> $O/perblock256.err &&
for tune in coalesce_target=64 coalesce_target=128 coalesce_target=256 coalesce_target=128,coalesce_spin_us=2000 coalesce_target=128,coalesce_depth=3; do
  SHMR_PB_TUNE=$tune SHMR_PB_QUEUE_ONLY=1 timeout -k 10 300 tools/_abx/perblock_dev 1024 3 >> $O/perblock1024.jsonl 2>> $O/perblock1024.err || exit 1
done &&
timeout -k 10 300 python -u tools/ptrs_ab.py --config encode83 --rounds 7 --legs slots,slab_sep,slab,pool_dense,pool_holed,pool_holed_tab,joint_pad0k > $O/ptrs_ab_encode83.jsonl 2>&1
echo "exit=$?"
